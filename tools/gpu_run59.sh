#!/bin/bash
# 3x3 bench incl. parity stride-2 dgrad vs MIOpen; ResNet bench with the parity path on
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/gemm_bench.py --only3x3 --iters 20 > gpurun_out/gemm59.log 2>&1 || exit 1
DCP_S2_DGRAD_PARITY=1 timeout -k 10 600 python3 bench.py --steps 30 --warmup 10 > gpurun_out/b59_par.log 2>&1 || exit 1
timeout -k 10 600 python3 bench.py --steps 30 --warmup 10 > gpurun_out/b59.log 2>&1 || exit 1
echo done
