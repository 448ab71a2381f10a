#!/bin/bash
# ResNet-50 (bench default config) kernel profile: rocprofv3 --kernel-trace
# --stats over a short bench run; per-kernel and per-family summaries in
# gpurun_out/${TAG}_{stats,families}.txt (the trace database stays in /tmp).
set -o pipefail
TAG=${TAG:-r4_rn50}; STEPS=${STEPS:-10}; WARM=${WARM:-5}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "/tmp/${TAG}" -o run -- python3 "$R/bench.py" \
  --steps "$STEPS" --warmup "$WARM" $BENCH_ARGS > "$O/${TAG}.log" 2>&1 || { tail -20 "$O/${TAG}.log"; exit 1; }
python3 "$R/tools/kernel_stats.py" "/tmp/${TAG}/run_results.db" --top 40 > "$O/${TAG}_stats.txt"
python3 "$R/tools/kernel_stats.py" "/tmp/${TAG}/run_results.db" --top 60 --grid > "$O/${TAG}_grid.txt"
python3 "$R/tools/kernel_stats.py" "/tmp/${TAG}/run_results.db" --families --steps $((STEPS + WARM)) --top 30 \
  > "$O/${TAG}_families.txt"
python3 "$R/tools/kernel_stats.py" "/tmp/${TAG}/run_results.db" --busy 0 --window "${WIN:-mt_sgd}:${STEPS}" >> "$O/${TAG}_families.txt" || true
cat "$O/${TAG}_families.txt"
echo "[rn_prof] done"
