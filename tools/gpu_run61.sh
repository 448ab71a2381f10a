#!/bin/bash
# ResNet-50 current state: bench, then a kernel trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 500 rocprofv3 --kernel-trace -d /tmp/prof61 -o prof -- python3 $R/bench.py --steps 6 --warmup 3 > $R/gpurun_out/prof61.log 2>&1 || exit 1
DB=$(find /tmp/prof61 -name "*.db" | head -1)
python3 $R/tools/trace_summary.py $DB --steps 4 --marker mt_sgd --top 70 > $R/gpurun_out/prof61_resnet50.txt 2>&1
echo done
