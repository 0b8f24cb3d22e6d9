#!/bin/bash
# GPU-box: PMC passes over the PFKS-only timing script (scripts/ab/time_stage.py pfks1), one pass per
# counter group; raw CSVs under gpurun_out/pmc_pfks_*/, per-kernel averages in gpurun_out/pmc_pfks.txt.
set -o pipefail
ROOT="$(cd "$(dirname "$0")/../.." && pwd)"
OUT="$ROOT/gpurun_out"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INST_CYCLES_VMEM_RD" \
           "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL" \
           "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum SQ_WAVES SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU" \
           "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/pmc_pfks_$i" -o run -- python3 "$ROOT/scripts/ab/time_stage.py" pfks1 > "$OUT/pmc_pfks_$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/pmc_pfks_$i.log"; exit 1; }
done
python3 - "$OUT" > "$OUT/pmc_pfks.txt" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(out + "/pmc_pfks_*/**/*counter_collection.csv", recursive=True):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        per[(k, r.get("Dispatch_Id"), r["Counter_Name"])] += float(r["Counter_Value"])
    for (k, d, c), v in per.items():
        agg[k][c].append(v)
for k, cs in agg.items():
    if "gemm" not in k: continue
    print(k)
    for c, v in sorted(cs.items()):
        print("   %-30s %.4g (avg of %d)" % (c, sum(v) / len(v), len(v)))
PY
cat "$OUT/pmc_pfks.txt"
