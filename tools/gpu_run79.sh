#!/bin/bash
# ResNet-50 per-GPU batch 512 (288 GB HBM leaves room): ours vs stock on one box
set -o pipefail
mkdir -p gpurun_out
for impl in ours torch; do
timeout -k 10 500 python3 bench.py --batch 512 --steps 20 --warmup 8 --impl $impl > gpurun_out/b79_$impl.log 2>&1 || exit 1
grep '^{' gpurun_out/b79_$impl.log >> gpurun_out/b79_pairs.jsonl
done
python3 -c "
import json
for l in open('gpurun_out/b79_pairs.jsonl'):
    d=json.loads(l); print(d['config']['impl'], d['config']['per_gpu_batch'], d['value'], d['ms_per_step'])"
