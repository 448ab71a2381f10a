#!/bin/bash
# Host-side (Python) profile of the bench's TIMED steps (DCP_BENCH_CPROFILE):
# top functions by own and cumulative time, and the host enqueue time per step
# next to the step time (host-bound when they are close).
set -o pipefail
M=${MODEL:-bert}; TAG=${TAG:-r5_host}; STEPS=${STEPS:-20}
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$O"
DCP_BENCH_CPROFILE=/tmp/${TAG}_$M.prof timeout -k 10 400 python3 bench.py --model $M --steps $STEPS --warmup 6 \
  ${BENCH_ARGS} > "$O/${TAG}_$M.log" 2>&1 || { tail -20 "$O/${TAG}_$M.log"; exit 1; }
grep "host enqueue" "$O/${TAG}_$M.log"
python3 - "$M" "$TAG" "$O" "$STEPS" <<'PY' > "$O/${TAG}_${M}_prof.txt"
import pstats, sys
m, tag, o, steps = sys.argv[1:]
st = pstats.Stats(f"/tmp/{tag}_{m}.prof")
print(f"# {steps} timed steps")
st.sort_stats("tottime").print_stats(40)
st.sort_stats("cumtime").print_stats(50)
PY
head -60 "$O/${TAG}_${M}_prof.txt"
