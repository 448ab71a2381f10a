#!/bin/bash
set -eo pipefail
bash tools/gpu.sh r3f_gpt2 prof=--model,gpt2,--steps,4,--warmup,3
bash tools/gpu.sh r3f_bert prof=--model,bert,--steps,4,--warmup,3
bash tools/gpu.sh r3f bench=--model,bert bench=--model,bert,--linear-path,aten-fwd bench=--model,bert,--linear-path,aten bench=--model,gpt2 bench=--model,gpt2,--linear-path,aten-fwd bench=--model,gpt2,--linear-path,aten
