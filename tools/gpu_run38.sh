#!/bin/bash
# gemm_nt with incremental counters + conflict-free swizzle: GEMM tests + 1x1 bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv1x1.py tests/test_gpu_transformer_ops.py > gpurun_out/t40.log 2>&1 || exit 1
timeout -k 10 300 python3 tools/gemm_bench.py --no3x3 --iters 20 > gpurun_out/gemm40.log 2>&1 || exit 1
echo done
