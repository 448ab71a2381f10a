#!/bin/bash
# HIP runtime trace (no counters) of a short bench run: long blocking API calls
set -o pipefail
M=${MODEL:-bert}; TAG=${TAG:-r5_stall}; STEPS=${STEPS:-12}
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --output-format csv -d "/tmp/${TAG}_$M" -o run -- \
  python3 "$R/bench.py" --model $M --steps $STEPS --warmup 4 > "$O/${TAG}_$M.log" 2>&1 || { tail -20 "$O/${TAG}_$M.log"; exit 1; }
if [ "$M" = gpt2 ]; then W="xent_fwd:$((4 * (STEPS - 2)))"; else W="xent_fwd:$((STEPS - 2))"; fi
python3 "$R/tools/hip_api_stalls.py" "/tmp/${TAG}_$M" --window "$W" --steps $((STEPS - 3)) > "$O/${TAG}_${M}_stalls.txt" 2>&1
head -40 "$O/${TAG}_${M}_stalls.txt"
