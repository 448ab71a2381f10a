#!/bin/bash
set -eo pipefail
bash tools/gpu.sh r3n tests=transformer,or,models bench=--model,bert bench=--model,gpt2 bench=--model,bert,--linear-path,aten
