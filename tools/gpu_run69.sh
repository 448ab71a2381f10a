#!/bin/bash
# wgrad ring configs: 64x2 (default) vs 32x2 (4 WG/CU) — Linear + conv wgrad benches
set -o pipefail
mkdir -p gpurun_out
for c in 64x2 32x2; do
DCP_WGRAD_CFG=$c timeout -k 10 300 python3 tools/linear_wgrad_bench.py --iters 20 > gpurun_out/lw69_$c.log 2>&1 || exit 1
DCP_WGRAD_CFG=$c timeout -k 10 300 python3 tools/gemm_bench.py --iters 20 > gpurun_out/gemm69_$c.log 2>&1 || exit 1
done
echo done
