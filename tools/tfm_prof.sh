#!/bin/bash
# Transformer kernel profile: rocprofv3 --kernel-trace --stats over a short
# bench.py run of each listed model and a
# per-kernel summary (tools/kernel_stats.py) in gpurun_out/${TAG}_<model>_stats.txt
# (trace databases under /tmp on the box)
set -o pipefail
TAG=${TAG:-r4_prof}; MODELS=${MODELS:-"gpt2 bert"}; STEPS=${STEPS:-6}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for m in $MODELS; do
  # the trace database stays on the box (/tmp): gpurun_out/ must stay under 64 MiB
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "/tmp/${TAG}_$m" -o run -- python3 "$R/bench.py" --model "$m" \
    --steps "$STEPS" --warmup 4 > "$O/${TAG}_$m.log" 2>&1 || { tail -20 "$O/${TAG}_$m.log"; exit 1; }
  python3 "$R/tools/kernel_stats.py" "/tmp/${TAG}_$m/run_results.db" --top 40 > "$O/${TAG}_${m}_stats.txt" 2>&1 || {
    tail -5 "$O/${TAG}_${m}_stats.txt"; exit 1; }
  python3 "$R/tools/kernel_stats.py" "/tmp/${TAG}_$m/run_results.db" --families --steps $((STEPS + 4)) --top 30 \
    > "$O/${TAG}_${m}_families.txt" 2>&1 || { tail -5 "$O/${TAG}_${m}_families.txt"; exit 1; }
  python3 "$R/tools/kernel_stats.py" "/tmp/${TAG}_$m/run_results.db" --busy 0 --window "${WINDOW_KERNEL:-mt_adam}:${WINDOW_N:-20}" >> "$O/${TAG}_${m}_families.txt" 2>&1 || true
  tail -1 "$O/${TAG}_${m}_families.txt"
  head -25 "$O/${TAG}_${m}_stats.txt"
done
echo "[tfm_prof] done"
