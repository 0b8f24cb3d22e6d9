#!/bin/bash
# GPU-box: PMC passes (one per counter group) over one bench step; summary of every kernel in
# gpurun_out/pmc_bench.txt.  usage: pmc_bench.sh [bench args...]
set -o pipefail
ROOT="$(cd "$(dirname "$0")/../.." && pwd)"
OUT="$ROOT/gpurun_out"
ARGS="${*:---steps 1 --warmup 0 --cpu-baseline off --key-schedule plain}"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_I8 SQ_LDS_BANK_CONFLICT" \
           "GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES" \
           "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d "$OUT/pmcb_$i" -o run -- python3 "$ROOT/bench.py" $ARGS > "$OUT/pmcb_$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/pmcb_$i.log"; exit 1; }
done
python3 - "$OUT" > "$OUT/pmc_bench.txt" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(out + "/pmcb_*/**/*counter_collection.csv", recursive=True):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("(anonymous namespace)::", "")
        per[(k, r.get("Dispatch_Id"), r["Counter_Name"])] += float(r["Counter_Value"])
    for (k, d, c), v in per.items():
        agg[k][c].append(v)
for k, cs in sorted(agg.items()):
    if "copyBuffer" in k: continue
    print(k)
    for c, v in sorted(cs.items()):
        print("   %-28s %.4g (avg of %d)" % (c, sum(v) / len(v), len(v)))
PY
cat "$OUT/pmc_bench.txt"
