#!/bin/bash
set -eo pipefail
bash tools/gpu.sh r3q tests=layer_norm,or,gpt2,or,models bench=--model,gpt2 prof=--model,gpt2,--steps,4,--warmup,3
