#!/bin/bash
# ResNet-50 after the GEMM issue/swizzle fixes: bench, then a kernel trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python3 bench.py --steps 30 --warmup 10 > gpurun_out/b42.log 2>&1 || exit 1
cd /tmp
timeout -k 10 500 rocprofv3 --kernel-trace -d /tmp/prof42 -o prof -- python3 $R/bench.py --steps 6 --warmup 3 > $R/gpurun_out/prof42.log 2>&1 || exit 1
DB=$(find /tmp/prof42 -name "*.db" | head -1)
python3 $R/tools/trace_summary.py $DB --steps 4 --marker mt_sgd --top 70 > $R/gpurun_out/prof42_resnet50.txt 2>&1
echo done
