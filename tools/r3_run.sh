#!/bin/bash
set -eo pipefail
bash tools/gpu.sh r3p tests py=tools/attn_bench.py:--iters,10 bench=--model,gpt2 bench=--model,bert bench=--steps,20,--warmup,10 smoke
