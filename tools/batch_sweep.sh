#!/bin/bash
# ResNet-50 per-GPU batch sweep, ours and stock (bench.py --impl torch) on one
# box -> gpurun_out/${TAG}.jsonl (one labelled line per run)
set -o pipefail
TAG=${TAG:-r6_batch}; BATCHES=${BATCHES:-"512 768 1024"}; STEPS=${STEPS:-12}; IMPLS=${IMPLS:-"ours torch"}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
for b in $BATCHES; do
  for impl in $IMPLS; do
    timeout -k 10 ${RUN_TIMEOUT:-400} python3 -u "$R/bench.py" --impl "$impl" --batch "$b" --steps "$STEPS" --warmup 6 > "$O/${TAG}_run.log" 2>&1 || {
      echo "[batch_sweep] b=$b $impl failed"; tail -5 "$O/${TAG}_run.log"; continue; }
    grep '^{' "$O/${TAG}_run.log" | tail -1 | python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); d['label'] = 'resnet50 b$b $impl'; print(json.dumps(d))" | tee -a "$O/${TAG}.jsonl" | python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); print(d['label'], d['value'], d['ms_per_step'])"
  done
done
echo "[batch_sweep] done"
