#!/bin/bash
# GPU-box: 1-GPU bench line, then a rocprofv3 kernel-trace/stats pass of the same command.
set -o pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
STEPS=${STEPS:-2}
timeout -k 10 ${BENCH_TIMEOUT:-900} python "$ROOT/bench.py" --steps $STEPS --warmup 1 > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed rc=$?"; tail -30 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
if [ "${PROFILE:-1}" = "1" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 ${PROF_TIMEOUT:-900} rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- python3 "$ROOT/bench.py" --steps 1 --warmup 0 --cpu-baseline off > "$OUT/prof_bench.json" 2> "$OUT/prof.err" || { echo "rocprof failed rc=$?"; tail -30 "$OUT/prof.err"; exit 1; }
  find "$OUT/prof" -name "*stats*" | head
fi
