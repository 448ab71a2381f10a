#!/bin/bash
# Eager vs whole-step HIP graph for the transformer workloads with the GEMM
# choices pinned (the first eager run's autotune table, via DCP_LINEAR_CHOICES)
# so both arms run the same kernels; alternating runs on one box ->
# gpurun_out/${TAG}.jsonl
set -o pipefail
TAG=${TAG:-r6_graph_ab}; MODELS=${MODELS:-"bert gpt2"}; STEPS=${STEPS:-20}; REPS=${REPS:-2}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
for m in $MODELS; do
  timeout -k 10 300 python3 -u "$R/bench.py" --model "$m" --steps 5 --warmup 3 > "$O/${TAG}_${m}_tune.log" 2>&1 || {
    tail -20 "$O/${TAG}_${m}_tune.log"; exit 1; }
  grep '^{' "$O/${TAG}_${m}_tune.log" | python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); json.dump(d['config']['linear_gemm_choice'], open('$O/${TAG}_${m}_choices.json', 'w'))"
  for rep in $(seq $REPS); do
    for gr in 0 1; do
      DCP_LINEAR_CHOICES="$O/${TAG}_${m}_choices.json" timeout -k 10 300 python3 -u "$R/bench.py" --model "$m" --graph $gr \
        --steps "$STEPS" --warmup 5 > "$O/${TAG}_run.log" 2>&1 || { tail -20 "$O/${TAG}_run.log"; exit 1; }
      grep '^{' "$O/${TAG}_run.log" | tail -1 | python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); d['label'] = '$m graph=$gr'; print(json.dumps(d))" | tee -a "$O/${TAG}.jsonl" | python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); print(d['label'], d['value'], d['ms_per_step'])"
    done
  done
done
echo "[graph_ab] done"
