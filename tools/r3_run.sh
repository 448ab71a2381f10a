#!/bin/bash
# round-3 final-tree evidence on one box: GPU suite, smoke, ours vs stock (same box, back to back), ResNet profile
set -eo pipefail
bash tools/gpu.sh r3z tests smoke \
  bench=--steps,30,--warmup,10 bench=--impl,torch,--steps,30,--warmup,10 \
  bench=--model,gpt2 bench=--model,gpt2,--impl,torch \
  bench=--model,bert bench=--model,bert,--impl,torch \
  bench=--model,convnet,--steps,200,--warmup,30 bench=--model,convnet,--impl,torch,--steps,200,--warmup,30 \
  prof=--steps,8,--warmup,5
