#!/bin/bash
# Optimizer overlap (DDP overlap_optimizer) under the 8-rank contention
# emulation: exposed comm and step time with / without, GPT-2 / BERT /
# ResNet-50 -> gpurun_out/${TAG}.jsonl
set -o pipefail
TAG=${1:-r4_overlap_ab}; STEPS=${STEPS:-12}; MODELS=${MODELS:-"gpt2 bert resnet50"}
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$O"
for m in $MODELS; do
  for ov in 0 1; do
    timeout -k 10 300 python3 -u bench.py --model "$m" --steps "$STEPS" --warmup 6 --comm-timing 1 --emulate-world 8 \
      --overlap-optimizer $ov > "$O/${TAG}_run.log" 2>&1 || { tail -30 "$O/${TAG}_run.log"; exit 1; }
    grep '^{' "$O/${TAG}_run.log" | tail -1 | python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); d['label'] = '$m ov$ov'; print(json.dumps(d))" | tee -a "$O/${TAG}.jsonl" | python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); print(d['label'], d['ms_per_step'], d['comm']['exposed_comm_ms'])"
  done
done
