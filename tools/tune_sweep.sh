#!/bin/bash
# One box, one model: bench.py under each gemm_tune setting of TUNES (space-
# separated; "-" = defaults), twice in interleaved order -> gpurun_out/${TAG}.jsonl
set -o pipefail
TAG=${TAG:-tune}; MODEL=${MODEL:-resnet50}; STEPS=${STEPS:-15}; REPS=${REPS:-2}
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$O"
for r in $(seq "$REPS"); do
  for tune in $TUNES; do
    arg=""; [ "$tune" != "-" ] && arg="--gemm-tune $tune"
    timeout -k 10 300 python3 -u bench.py --model "$MODEL" --steps "$STEPS" --warmup 6 $arg $BENCH_ARGS \
      > "$O/${TAG}_run.log" 2>&1 || { echo "[tune_sweep] $tune failed"; tail -20 "$O/${TAG}_run.log"; exit 1; }
    grep '^{' "$O/${TAG}_run.log" | tail -1 | python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); d['label'] = '$MODEL $tune'; print(json.dumps(d))" | tee -a "$O/${TAG}.jsonl" |
      python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); print(d['label'], d['value'], d['ms_per_step'])"
  done
done
echo "[tune_sweep] done"
