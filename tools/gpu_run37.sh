#!/bin/bash
# 1x1 GEMM variants: plain / +stats / +bn-relu prologue / both
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/gemm_bench.py --no3x3 --iters 20 > gpurun_out/gemm37.log 2>&1 || exit 1
echo done
