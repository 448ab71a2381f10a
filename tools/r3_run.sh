#!/bin/bash
set -eo pipefail
bash tools/gpu.sh r3y tests=fused_mlp,or,linear,or,gpt2,or,bert bench=--model,bert bench=--model,bert,--linear-path,ours-unfused-mlp bench=--model,gpt2 bench=--model,gpt2,--linear-path,ours-unfused-mlp
