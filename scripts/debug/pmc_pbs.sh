#!/bin/bash
# GPU-box: PMC passes over the PBS-only timing script (scripts/ab/time_stage.py pbs1), one pass per
# counter group; raw CSVs under gpurun_out/pmc_pbs_*/, summary in gpurun_out/pmc_pbs.txt.
set -o pipefail
ROOT="$(cd "$(dirname "$0")/../.." && pwd)"
OUT="$ROOT/gpurun_out"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_THREAD_CYCLES_VALU SQ_INSTS_LDS SQ_INSTS_SALU" \
           "GRBM_GUI_ACTIVE GRBM_COUNT SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INST_LEVEL_LDS SQ_INSTS_VALU_CVT SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/pmc_pbs_$i" -o run -- python3 "$ROOT/scripts/ab/time_stage.py" pbs1 > "$OUT/pmc_pbs_$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/pmc_pbs_$i.log"; exit 1; }
done
python3 - "$OUT" > "$OUT/pmc_pbs.txt" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(out + "/pmc_pbs_*/**/*counter_collection.csv", recursive=True):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        per[(k, r.get("Dispatch_Id"), r["Counter_Name"])] += float(r["Counter_Value"])
    for (k, d, c), v in per.items():
        agg[k][c].append(v)
for k, cs in agg.items():
    if "br" not in k: continue
    print(k)
    for c, v in sorted(cs.items()):
        print("   %-28s %.4g (avg of %d)" % (c, sum(v) / len(v), len(v)))
PY
cat "$OUT/pmc_pbs.txt"
