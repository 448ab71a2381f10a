#!/bin/bash
# Idle-gap attribution of the transformer steps (tools/gap_stats.py) from a
# rocprofv3 kernel trace of a short bench run per model.
set -o pipefail
TAG=${TAG:-r5_gaps}; MODELS=${MODELS:-"gpt2 bert"}; STEPS=${STEPS:-12}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for m in $MODELS; do
  timeout -k 10 400 rocprofv3 --kernel-trace -d "/tmp/${TAG}_$m" -o run -- python3 "$R/bench.py" --model "$m" \
    --steps "$STEPS" --warmup 4 > "$O/${TAG}_$m.log" 2>&1 || { tail -20 "$O/${TAG}_$m.log"; exit 1; }
  if [ "$m" = gpt2 ]; then W="xent_fwd:$((4 * (STEPS - 2)))"; else W="xent_fwd:$((STEPS - 2))"; fi
  python3 "$R/tools/gap_stats.py" "/tmp/${TAG}_$m/run_results.db" --window "$W" --steps $((STEPS - 3)) --top 30 \
    > "$O/${TAG}_${m}_gaps.txt" 2>&1 || { tail -5 "$O/${TAG}_${m}_gaps.txt"; exit 1; }
  head -20 "$O/${TAG}_${m}_gaps.txt"
done
echo "[tfm_gaps] done"
