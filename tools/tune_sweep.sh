#!/bin/bash
# Same-box sweep of one gemm_tune key over several values (bench.py
# --gemm-tune KEY=V), interleaved REPS times -> gpurun_out/${TAG}.jsonl.
#   TAG=r6_bncap KEY=bn_apply_cap VALS="1024 2048 4096" MODEL=resnet50 bash tools/tune_sweep.sh
set -o pipefail
TAG=${TAG:-sweep}; MODEL=${MODEL:-resnet50}; STEPS=${STEPS:-15}; WARMUP=${WARMUP:-5}; REPS=${REPS:-2}
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$O"
for r in $(seq "$REPS"); do
  for v in $VALS; do
    timeout -k 10 300 python3 -u bench.py --model "$MODEL" --steps "$STEPS" --warmup "$WARMUP" --gemm-tune "$KEY=$v" \
      $BENCH_ARGS > "$O/${TAG}_run.log" 2>&1 || { echo "[tune_sweep] $KEY=$v failed"; tail -20 "$O/${TAG}_run.log"; exit 1; }
    grep '^{' "$O/${TAG}_run.log" | tail -1 | python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); d['label'] = '$MODEL $KEY=$v'; print(json.dumps(d))" | tee -a "$O/${TAG}.jsonl" |
      python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); print(d['label'], d['value'], d['ms_per_step'])"
  done
done
echo "[tune_sweep] done"
