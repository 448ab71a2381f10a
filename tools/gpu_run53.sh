#!/bin/bash
# launch_bounds(256,2) gemm_nt + RED epilogue with LDS coefficients: tests, GEMM bench, ResNet fused on/off
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv1x1.py > gpurun_out/t53.log 2>&1 || exit 1
timeout -k 10 300 python3 tools/gemm_bench.py --iters 20 > gpurun_out/gemm53.log 2>&1 || exit 1
timeout -k 10 600 python3 bench.py --steps 30 --warmup 10 > gpurun_out/b53.log 2>&1 || exit 1
DCP_BN_CONV_FUSE=0 timeout -k 10 600 python3 bench.py --steps 30 --warmup 10 > gpurun_out/b53_off.log 2>&1 || exit 1
echo done
