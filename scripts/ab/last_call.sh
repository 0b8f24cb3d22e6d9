set -o pipefail
cd /root/repo
timeout -k 10 500 python -u scripts/probes/stage_overlap.py 224 236 240 > gpurun_out/overlap2.txt 2>&1
