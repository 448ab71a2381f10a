#!/bin/bash
set -eo pipefail
bash tools/gpu.sh r3j tests=wgrad,or,conv1x1,or,transformer,or,numerics,or,fusions py=tools/linear_bench.py:--wgrad-only bench=--steps,20,--warmup,10 bench=--model,gpt2 bench=--model,bert
