#!/bin/bash
# Same-box A/B of the attention kernels: tools/attn_bench.py under
# rocprofv3 --kernel-trace for the tree at $OLD (a built worktree of an
# earlier commit) and for this tree; kernel tables via tools/rocpd_stats.py.
#   OLD=ab_old bash tools/attn_ab.sh   → gpurun_out/attn_ab_{old,new}.txt
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for side in old new; do
  src=$R; [ $side = old ] && src=$R/${OLD:-ab_old}
  timeout -k 10 240 rocprofv3 --kernel-trace -d "$O/attn_ab_$side" -o run -- \
    python3 "$src/tools/attn_bench.py" --iters ${ITERS:-20} > "$O/attn_ab_${side}_bench.jsonl" 2> "$O/attn_ab_${side}.err" || { tail -5 "$O/attn_ab_${side}.err"; exit 1; }
  python3 "$R/tools/rocpd_stats.py" "$O/attn_ab_$side/run_results.db" 'dcp::kern.*attn_' --by-grid > "$O/attn_ab_$side.txt" || exit 1
  echo "== $side"; cat "$O/attn_ab_$side.txt"; grep -h '"case"' "$O/attn_ab_${side}_bench.jsonl"
done
