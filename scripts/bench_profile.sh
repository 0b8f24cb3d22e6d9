#!/bin/bash
# GPU-box: 1-GPU bench line, then rocprofv3 passes of the same workload (kernel-trace + stats, then
# separate --pmc passes for FETCH_SIZE, WRITE_SIZE and SQ occupancy/stall counters, as
# MI355X_MICROARCH.md's HBM/rocprofv3 section prescribes), summarised by scripts/prof_summary.py.
# The profiled runs use --key-schedule plain so every hot-path launch has the bench's batch shape.
set -o pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
STEPS=${STEPS:-2}
BLOCKS=${BLOCKS:-128}
timeout -k 10 ${BENCH_TIMEOUT:-900} python "$ROOT/bench.py" --steps $STEPS --warmup 1 --blocks-per-gpu $BLOCKS > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed rc=$?"; tail -30 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
[ "${PROFILE:-1}" = "1" ] || exit 0
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 1 --warmup 0 --cpu-baseline off --single-block off --model8-leg off --host-buffers off --key-schedule plain --blocks-per-gpu $BLOCKS"
T=${PROF_TIMEOUT:-600}
timeout -k 10 $T rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 "$ROOT/bench.py" $ARGS > "$OUT/prof_bench.json" 2> "$OUT/prof.err" || { echo "rocprof failed rc=$?"; tail -30 "$OUT/prof.err"; exit 1; }
if [ "${PMC:-1}" = "1" ]; then
  timeout -k 10 $T rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 "$ROOT/bench.py" $ARGS > /dev/null 2> "$OUT/pmc_fetch.err" || { echo "pmc fetch failed rc=$?"; tail -30 "$OUT/pmc_fetch.err"; exit 1; }
  timeout -k 10 $T rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- python3 "$ROOT/bench.py" $ARGS > /dev/null 2> "$OUT/pmc_write.err" || { echo "pmc write failed rc=$?"; tail -30 "$OUT/pmc_write.err"; exit 1; }
  timeout -k 10 $T rocprofv3 --pmc TCC_EA0_RDREQ TCC_EA0_RDREQ_DRAM --output-format csv -d "$OUT/pmc_dram" -o run -- python3 "$ROOT/bench.py" $ARGS > /dev/null 2> "$OUT/pmc_dram.err" || { echo "pmc dram failed rc=$?"; tail -30 "$OUT/pmc_dram.err"; }
  timeout -k 10 $T rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY --output-format csv -d "$OUT/pmc_sq" -o run -- python3 "$ROOT/bench.py" $ARGS > /dev/null 2> "$OUT/pmc_sq.err" || { echo "pmc sq failed rc=$?"; tail -30 "$OUT/pmc_sq.err"; }
  timeout -k 10 $T rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmc_mfma" -o run -- python3 "$ROOT/bench.py" $ARGS > /dev/null 2> "$OUT/pmc_mfma.err" || { echo "pmc mfma failed rc=$?"; tail -30 "$OUT/pmc_mfma.err"; }
fi
python3 "$ROOT/scripts/prof_summary.py" "$OUT" $BLOCKS > "$OUT/prof_summary.txt" 2>&1 || true
cat "$OUT/prof_summary.txt"
