#!/bin/bash
# Same-box A/B of two GEMM tuning settings (bench.py --gemm-tune), interleaved
# A B A B per model -> gpurun_out/${TAG}.jsonl (one labelled JSON line a run).
#   TAG=r4_wgfuse A=wg_fuse=1 B=wg_fuse=0 MODELS="gpt2 bert resnet50" bash tools/ab_tune.sh
set -o pipefail
TAG=${TAG:-ab}; MODELS=${MODELS:-"gpt2 bert resnet50"}; STEPS=${STEPS:-20}; REPS=${REPS:-2}
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$O"
for m in $MODELS; do
  for r in $(seq "$REPS"); do
    for lab in A B; do
      tune=${!lab}
      timeout -k 10 400 python3 -u bench.py --model "$m" --steps "$STEPS" --warmup 8 --gemm-tune "$tune" $BENCH_ARGS \
        > "$O/${TAG}_run.log" 2>&1 || { echo "[ab_tune] $m $lab failed"; tail -20 "$O/${TAG}_run.log"; exit 1; }
      grep '^{' "$O/${TAG}_run.log" | tail -1 | python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); d['label'] = '$m $lab $tune'; print(json.dumps(d))" | tee -a "$O/${TAG}.jsonl" |
        python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); print(d['label'], d['value'], d['ms_per_step'])"
    done
  done
done
echo "[ab_tune] done"
