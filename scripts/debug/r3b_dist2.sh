#!/bin/bash
# 2-rank rehearsal of the multi-rank bench path on one GPU (gloo: RCCL refuses two ranks on one device):
# key broadcast, device-key contexts, sharded counters, max-over-ranks timing, min-over-ranks correctness
cd /root/repo
mkdir -p gpurun_out
TAE_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 1 --warmup 1 --blocks-per-gpu 32 --cpu-baseline off --single-block off --model8-leg off --host-buffers off > gpurun_out/dist2.json 2> gpurun_out/dist2.err || { echo "rc=$?"; tail -20 gpurun_out/dist2.err; exit 1; }
tail -c 600 gpurun_out/dist2.json
