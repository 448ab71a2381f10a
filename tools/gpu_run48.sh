#!/bin/bash
# gemm_nt BK=64 (2-stage ring) vs BK=32 (3-stage): tests, 1x1 + 3x3 bench each
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv1x1.py > gpurun_out/t48.log 2>&1 || exit 1
timeout -k 10 300 python3 tools/gemm_bench.py --iters 20 > gpurun_out/gemm48_bk64.log 2>&1 || exit 1
DCP_GEMM_BK=32 timeout -k 10 300 python3 tools/gemm_bench.py --iters 20 > gpurun_out/gemm48_bk32.log 2>&1 || exit 1
echo done
