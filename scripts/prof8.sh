#!/bin/bash
# GPU box: the 8-bit model (BASELINE configs[4]) at a throughput shape: bench line, rocprofv3 kernel
# stats and separate PMC passes (FETCH_SIZE, WRITE_SIZE, SQ) of one 10-round step over NB blocks.
set -o pipefail
ROOT=/root/repo
OUT=$ROOT/gpurun_out/prof8
NB=${NB:-64}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
ARGS="--model 8bit --blocks-per-gpu $NB --steps 1 --warmup 0 --cpu-baseline off --single-block off --host-buffers off --key-schedule plain"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 $ROOT/bench.py $ARGS > $OUT/kt_bench.json 2> $OUT/kt.err || { echo "kt rc=$?"; tail -20 $OUT/kt.err; exit 1; }
cat $OUT/kt_bench.json
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 $ROOT/bench.py $ARGS > /dev/null 2> $OUT/pmc_fetch.err || { echo "fetch rc=$?"; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 $ROOT/bench.py $ARGS > /dev/null 2> $OUT/pmc_write.err || { echo "write rc=$?"; exit 1; }
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY --output-format csv -d $OUT/pmc_sq -o run -- python3 $ROOT/bench.py $ARGS > /dev/null 2> $OUT/pmc_sq.err || { echo "sq rc=$?"; exit 1; }
python3 $ROOT/scripts/prof_split_summary.py $OUT $OUT/prof8_summary.json > /dev/null 2>&1 || exit 1
# bench.py --model 8bit reads the CBS launch's traffic from profiles/pmc8_latest.json (copy this file there)
python3 - "$OUT" "$NB" <<'PY'
import json, sys
out, nb = sys.argv[1], int(sys.argv[2])
d = json.load(open(out + "/prof8_summary.json"))
src = ("rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE passes of bench.py --model 8bit --steps 1 --key-schedule plain "
       "(scripts/prof8.sh -> scripts/prof_split_summary.py); bytes = 2 x FETCH_SIZE + WRITE_SIZE")
json.dump({"blocks_per_gpu": nb, "model": "8bit", "source": src, "launches": d}, open(out + "/pmc8_latest.json", "w"), indent=1)
PY
echo done
