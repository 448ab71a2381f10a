#!/bin/bash
# implicit-GEMM 3x3 conv: numerics tests, 3x3 bench vs MIOpen, ResNet bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv1x1.py tests/test_gpu_batchnorm.py > gpurun_out/t43.log 2>&1 || exit 1
timeout -k 10 300 python3 tools/gemm_bench.py --only3x3 --iters 20 > gpurun_out/gemm43.log 2>&1 || exit 1
timeout -k 10 600 python3 bench.py --steps 30 --warmup 10 > gpurun_out/b43.log 2>&1 || exit 1
echo done
