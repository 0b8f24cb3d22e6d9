set -o pipefail
cd /root/repo
PASSES=2 VARIANTS="base:: noswap:noswap.so: nodec:nodec.so: notorus:notorus.so: all3:all3.so:" CLOCK=1 bash scripts/ab/ab.sh pbs1 > gpurun_out/ab_x4_bounds.txt 2>&1
