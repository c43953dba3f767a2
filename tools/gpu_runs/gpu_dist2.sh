#!/bin/bash
# GPU box: 2-rank rehearsal of bench.py's distributed path on ONE GPU (gloo collectives,
# RCCL refuses two ranks on one device).  The 8-GPU RCCL run is the driver's.
set -o pipefail
mkdir -p gpurun_out
export G2048_BENCH_BACKEND=gloo
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 400 --warmup 50 --train-updates 20 --no-cpu-baseline > gpurun_out/dist2.json 2> gpurun_out/dist2.err || { tail -30 gpurun_out/dist2.err; exit 1; }
cat gpurun_out/dist2.json
