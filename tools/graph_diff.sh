#!/bin/bash
# Eager vs whole-step HIP-graph kernel lists of one transformer workload:
# rocprofv3 kernel traces of bench.py --graph 0 and --graph 1 (databases under
# /tmp on the box), diffed by tools/graph_kernel_diff.py -> gpurun_out/${TAG}_<model>.txt
set -o pipefail
TAG=${TAG:-r6_graphdiff}; MODELS=${MODELS:-"bert gpt2"}; STEPS=${STEPS:-5}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for m in $MODELS; do
  for gr in 0 1; do
    timeout -k 10 400 rocprofv3 --kernel-trace -d "/tmp/${TAG}_${m}_g$gr" -o run -- python3 "$R/bench.py" --model "$m" \
      --graph $gr --steps "$STEPS" --warmup 3 > "$O/${TAG}_${m}_g$gr.log" 2>&1 || { tail -20 "$O/${TAG}_${m}_g$gr.log"; exit 1; }
    grep '^{' "$O/${TAG}_${m}_g$gr.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$m graph=$gr', d['value'], d['ms_per_step'])"
  done
  (cd "$R/tools" && python3 graph_kernel_diff.py "/tmp/${TAG}_${m}_g0/run_results.db" "/tmp/${TAG}_${m}_g1/run_results.db" \
    --steps "$STEPS") > "$O/${TAG}_${m}.txt" 2>&1 || { tail -5 "$O/${TAG}_${m}.txt"; exit 1; }
  head -40 "$O/${TAG}_${m}.txt"
done
echo "[graph_diff] done"
