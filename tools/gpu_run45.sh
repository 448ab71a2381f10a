#!/bin/bash
# 3x3 policy (ours fwd at 28x28/7x7, ours dgrad stride 1, ours wgrad except 64x64): tests + ResNet bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv1x1.py > gpurun_out/t45.log 2>&1 || exit 1
timeout -k 10 600 python3 bench.py --steps 30 --warmup 10 > gpurun_out/b45.log 2>&1 || exit 1
DCP_KXK_GEMM=0 timeout -k 10 600 python3 bench.py --steps 30 --warmup 10 > gpurun_out/b45_off.log 2>&1 || exit 1
echo done
