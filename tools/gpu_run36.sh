#!/bin/bash
# BN after LDS-staged apply coefficients + per-kind slab caps: sweep, BN tests, ResNet bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python3 tools/bn_sweep.py --iters 20 > gpurun_out/bn_sweep36.log 2>&1 || exit 1
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_batchnorm.py tests/test_gpu_conv1x1.py tests/test_gpu_convnet.py > gpurun_out/t36.log 2>&1 || exit 1
timeout -k 10 600 python3 bench.py --steps 30 --warmup 10 > gpurun_out/b36.log 2>&1 || exit 1
echo done
