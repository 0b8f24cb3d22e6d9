set -o pipefail
cd /root/repo
PASSES=2 CLOCK=1 bash scripts/ab/ab.sh pbs1 2>&1 | tee gpurun_out/ab_x4_bounds.txt
