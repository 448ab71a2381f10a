#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/graph_numerics.py > gpurun_out/graph_num21.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/gemm_bench.py --iters 10 > gpurun_out/gemm21.log 2>&1 || exit 1
echo done
