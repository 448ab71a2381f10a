#!/bin/bash
set -eo pipefail
bash tools/gpu.sh r3u tests=attention,or,attn,or,gpt2,or,bert,or,models py=tools/attn_bench.py:--iters,10 bench=--model,gpt2 bench=--model,bert
