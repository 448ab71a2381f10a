#!/bin/bash
# BN-backward reduce in the dgrad GEMM epilogue: tests, ResNet bench (fused on / off)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv1x1.py tests/test_gpu_batchnorm.py > gpurun_out/t52.log 2>&1 || exit 1
timeout -k 10 600 python3 bench.py --steps 30 --warmup 10 > gpurun_out/b52.log 2>&1 || exit 1
DCP_BN_CONV_FUSE=0 timeout -k 10 600 python3 bench.py --steps 30 --warmup 10 > gpurun_out/b52_off.log 2>&1 || exit 1
echo done
