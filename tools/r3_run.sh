#!/bin/bash
set -eo pipefail
bash tools/gpu.sh r3s tests=layer_norm,or,bert,or,models,or,gpt2 bench=--model,bert bench=--model,gpt2
