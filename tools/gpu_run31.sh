#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 500 rocprofv3 --kernel-trace -d /tmp/prof31 -o prof -- python3 $R/bench.py --steps 6 --warmup 3 > $R/gpurun_out/prof31.log 2>&1 || exit 1
DB=$(find /tmp/prof31 -name "*.db" | head -1)
python3 $R/tools/trace_summary.py $DB --steps 4 --marker mt_sgd --top 60 > $R/gpurun_out/prof31_resnet50.txt 2>&1
python3 $R/tools/kernel_stats.py $DB --grid --top 120 > $R/gpurun_out/prof31_grid.txt 2>&1
echo done
