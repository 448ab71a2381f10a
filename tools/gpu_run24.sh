#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof24 -o prof -- python3 $R/tools/attn_bench.py --iters 3 > $R/gpurun_out/prof24.log 2>&1 || exit 1
python3 $R/tools/kernel_stats.py $(find /tmp/prof24 -name "*.db" | head -1) --grid --top 40 > $R/gpurun_out/attn_kstats24.txt 2>&1
echo done
