#!/bin/bash
# bench.py's N > 1 contract on one GPU: two ranks under torch.distributed.run sharing the GPU
# through the host-staged backend (RCCL needs one GPU per rank)
set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29611 bench.py --gpus 2 --steps 3 --warmup 2 --backend gloo --batch 64 > gpurun_out/r3mr_bench.log 2>&1
grep '^{' gpurun_out/r3mr_bench.log
