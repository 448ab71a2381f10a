#!/bin/bash
# Linear wgrad backends at BERT/GPT-2 shapes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/linear_wgrad_bench.py --iters 20 > gpurun_out/lw65.log 2>&1 || exit 1
echo done
