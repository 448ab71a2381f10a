#!/bin/bash
# attention grids: heads on x (XCD balance), heaviest causal tiles first
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_attention.py tests/test_gpu_models.py > gpurun_out/t67.log 2>&1 || exit 1
timeout -k 10 300 python3 tools/attn_bench.py > gpurun_out/attn67.log 2>&1 || exit 1
timeout -k 10 500 python3 bench.py --model gpt2 --steps 20 --warmup 5 > gpurun_out/b67_gpt2.log 2>&1 || exit 1
timeout -k 10 500 python3 bench.py --model bert --steps 20 --warmup 5 > gpurun_out/b67_bert.log 2>&1 || exit 1
echo done
