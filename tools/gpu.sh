#!/bin/bash
# One parametrised GPU-box runner (replaces the round-1 tools/gpu_runNN.sh
# scratch scripts; their history is in git). Every GPU step runs under its own
# `timeout -k`, steps chain with && semantics (set -e), and all output lands in
# gpurun_out/<tag>_*.
#
#   gpurun -- bash tools/gpu.sh TAG STEP [STEP ...]
#
# STEPs (run in order, the script stops at the first failure):
#   tests[=PYTEST_K]      pytest -m gpu (optionally -k PYTEST_K)
#   smoke                 __graft_entry__.smoke()
#   bench[=ARGS]          bench.py ARGS (commas -> spaces), JSON appended to TAG_bench.jsonl
#   prof[=ARGS]           rocprofv3 --kernel-trace --stats of bench.py ARGS
#   pmc=COUNTERS[:ARGS]   rocprofv3 --pmc COUNTERS (one pass) of bench.py ARGS
#   py=SCRIPT[:ARGS]      python3 SCRIPT ARGS
set -eo pipefail
TAG=${1:?tag}; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
args() { echo "${1//,/ }"; }
for step in "$@"; do
  name=${step%%=*}; val=""; [[ "$step" == *=* ]] && val=${step#*=}
  echo "[gpu.sh] $TAG: $step"
  case $name in
    tests)
      k=(); [[ -n "$val" ]] && k=(-k "${val//,/ }")
      timeout -k 10 900 python3 -u -m pytest -x -v -m gpu --timeout 240 --timeout-method thread "${k[@]}" tests \
        > "$O/${TAG}_tests.log" 2>&1 || { tail -40 "$O/${TAG}_tests.log"; exit 1; }
      tail -3 "$O/${TAG}_tests.log" ;;
    smoke)
      timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/${TAG}_smoke.log" 2>&1
      tail -1 "$O/${TAG}_smoke.log" ;;
    bench)
      timeout -k 10 600 python3 -u bench.py $(args "$val") > "$O/${TAG}_bench.log" 2>&1 || { tail -30 "$O/${TAG}_bench.log"; exit 1; }
      grep '^{' "$O/${TAG}_bench.log" | tee -a "$O/${TAG}_bench.jsonl" ;;
    prof)
      (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/${TAG}_prof" -o prof -- \
        python3 "$R/bench.py" $(args "$val") > "$O/${TAG}_prof.log" 2>&1) || { tail -30 "$O/${TAG}_prof.log"; exit 1; }
      grep '^{' "$O/${TAG}_prof.log" || true
      # keep the per-kernel summary, drop the (large) trace database
      ks="$O/${TAG}_kernel_stats.txt"; n=2
      while [[ -e "$ks" ]]; do ks="$O/${TAG}_kernel_stats_$n.txt"; n=$((n + 1)); done
      python3 "$R/tools/kernel_stats.py" "$O/${TAG}_prof/prof_results.db" --top 60 > "$ks" 2>&1 || true
      rm -rf "$O/${TAG}_prof" ;;
    pmc)
      ctr=${val%%:*}; rest=""; [[ "$val" == *:* ]] && rest=${val#*:}
      (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc $(args "$ctr") --kernel-trace --stats -d "$O/${TAG}_pmc" -o pmc -- \
        python3 "$R/bench.py" $(args "$rest") > "$O/${TAG}_pmc.log" 2>&1) || { tail -30 "$O/${TAG}_pmc.log"; exit 1; }
      ;;
    py)
      scr=${val%%:*}; rest=""; [[ "$val" == *:* ]] && rest=${val#*:}
      timeout -k 10 600 python3 -u "$scr" $(args "$rest") > "$O/${TAG}_$(basename "$scr" .py).log" 2>&1 || {
        tail -30 "$O/${TAG}_$(basename "$scr" .py).log"; exit 1; }
      tail -5 "$O/${TAG}_$(basename "$scr" .py).log" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "[gpu.sh] $TAG done"
