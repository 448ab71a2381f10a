#!/bin/bash
# same-box ours vs stock torch DDP (RCCL) + torch.optim, all three GPU configs
set -o pipefail
mkdir -p gpurun_out
for m in resnet50 bert gpt2; do
for impl in ours torch; do
A=""; [ $m != resnet50 ] && A="--steps 20 --warmup 5"
timeout -k 10 400 python3 bench.py --model $m --impl $impl $A > gpurun_out/b76_${m}_$impl.log 2>&1 || exit 1
grep '^{' gpurun_out/b76_${m}_$impl.log >> gpurun_out/b76_pairs.jsonl
done
done
python3 -c "
import json
for l in open('gpurun_out/b76_pairs.jsonl'):
    d=json.loads(l); print(d['config']['model'], d['config']['impl'], d['value'], d['ms_per_step'])"
