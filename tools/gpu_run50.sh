#!/bin/bash
# wgrad BK=64 (2-deep ring): tests, GEMM bench (1x1 + 3x3 wgrad), ResNet bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv1x1.py tests/test_gpu_transformer_ops.py > gpurun_out/t50.log 2>&1 || exit 1
timeout -k 10 300 python3 tools/gemm_bench.py --iters 20 > gpurun_out/gemm50.log 2>&1 || exit 1
timeout -k 10 600 python3 bench.py --steps 30 --warmup 10 > gpurun_out/b50.log 2>&1 || exit 1
echo done
