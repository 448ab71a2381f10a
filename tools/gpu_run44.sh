#!/bin/bash
# gathered wgrad with incremental pixel tracking: tests + 3x3 bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv1x1.py > gpurun_out/t44.log 2>&1 || exit 1
timeout -k 10 300 python3 tools/gemm_bench.py --only3x3 --iters 20 > gpurun_out/gemm44.log 2>&1 || exit 1
echo done
