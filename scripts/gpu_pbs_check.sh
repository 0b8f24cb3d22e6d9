#!/bin/bash
# GPU-box: PBS-kernel iteration check -- the blind-rotation parity tests, then the PBS-stage timing
# (scripts/debug/time_pbs.py, 16383 ciphertexts: br512x4 + br512lat remainder) and a 1-step bench.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py -x -q --timeout 240 --timeout-method thread > gpurun_out/pbs_check_tests.log 2>&1
rc=$?
tail -5 gpurun_out/pbs_check_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/debug/time_pbs.py > gpurun_out/pbs_check_time.log 2>&1 || { tail -20 gpurun_out/pbs_check_time.log; exit 1; }
tail -2 gpurun_out/pbs_check_time.log
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 300 python bench.py --steps 2 --warmup 1 --cpu-baseline off --model8-leg off > gpurun_out/pbs_check_bench.json 2> gpurun_out/pbs_check_bench.err || { tail -20 gpurun_out/pbs_check_bench.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/pbs_check_bench.json')); r=d['roofline']; print('value', round(d['value'],2), 'blocks/s; pbs kernel', round(r['avg_launch_ms'],2), 'ms frac', round(r['frac'],3), 'stage', d['stage_ms_per_step'], 'single', d['single_block']['s_per_block'], d['single_block'].get('stage_ms'))"
fi
