#!/bin/bash
# in-place grad accumulation + bf16 weight cache: tests, GPT-2 and BERT benches
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_transformer_ops.py tests/test_gpu_models.py tests/test_gpu_ddp.py tests/test_gpu_graphs.py > gpurun_out/t66.log 2>&1 || exit 1
timeout -k 10 500 python3 bench.py --model gpt2 --steps 20 --warmup 5 > gpurun_out/b66_gpt2.log 2>&1 || exit 1
timeout -k 10 500 python3 bench.py --model bert --steps 20 --warmup 5 > gpurun_out/b66_bert.log 2>&1 || exit 1
echo done
