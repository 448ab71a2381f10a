#!/bin/bash
# Same-box A/B of two bench.py argument sets, interleaved A B A B ->
# gpurun_out/${TAG}.jsonl (labelled JSON lines).
#   TAG=x MODEL=resnet50 A="--res-prologue 1" B="--res-prologue 0" REPS=2 bash tools/ab_args.sh
set -o pipefail
TAG=${TAG:-ab_args}; MODEL=${MODEL:-resnet50}; STEPS=${STEPS:-20}; REPS=${REPS:-2}
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$O"
for r in $(seq "$REPS"); do
  for lab in A B; do
    args=${!lab}
    timeout -k 10 400 python3 -u bench.py --model "$MODEL" --steps "$STEPS" --warmup 8 $args > "$O/${TAG}_run.log" 2>&1 ||
      { echo "[ab_args] $lab failed"; tail -20 "$O/${TAG}_run.log"; exit 1; }
    grep '^{' "$O/${TAG}_run.log" | tail -1 | python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); d['label'] = '$MODEL $lab $args'; print(json.dumps(d))" | tee -a "$O/${TAG}.jsonl" |
      python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); print(d['label'], d['value'], d['ms_per_step'])"
  done
done
echo "[ab_args] done"
