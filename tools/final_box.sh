#!/bin/bash
# Same-box end-of-round numbers: every BASELINE workload on this framework
# and on stock torch (bench.py --impl torch: torch DDP + torch.optim + ATen /
# SDPA, same model code), back to back on ONE box (box-to-box spread is a
# few %) -> gpurun_out/${TAG}.jsonl, one labelled JSON line per run.
set -o pipefail
TAG=${TAG:-r4_final_box}; MODELS=${MODELS:-"resnet50 gpt2 bert convnet"}; STEPS=${STEPS:-20}
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$O"
for m in $MODELS; do
  for impl in ${IMPLS:-ours torch}; do
    timeout -k 10 ${RUN_TIMEOUT:-500} python3 -u bench.py --model "$m" --impl "$impl" --steps "$STEPS" --warmup 8 \
      > "$O/${TAG}_run.log" 2>&1 || { echo "[final_box] $m $impl failed"; tail -20 "$O/${TAG}_run.log"; exit 1; }
    grep '^{' "$O/${TAG}_run.log" | tail -1 | python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); d['label'] = '$m $impl'; print(json.dumps(d))" | tee -a "$O/${TAG}.jsonl" |
      python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); print(d['label'], d['value'], d['ms_per_step'])"
  done
done
echo "[final_box] done"
