#!/bin/bash
# maxpool k3s2 block-owner backward + one-launch conv weight casts: tests, kernel bench, ResNet bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv1x1.py tests/test_gpu_kernels.py tests/test_gpu_convnet.py tests/test_gpu_batchnorm.py > gpurun_out/t55.log 2>&1 || exit 1
timeout -k 10 300 python3 tools/kernel_bench.py --iters 20 > gpurun_out/kb55.log 2>&1 || exit 1
timeout -k 10 600 python3 bench.py --steps 30 --warmup 10 > gpurun_out/b55.log 2>&1 || exit 1
echo done
