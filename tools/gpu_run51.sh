#!/bin/bash
# ResNet-50 BK=64 GEMMs, ours 3x3 everywhere, strided downsample on the gathered GEMM: bench, then a kernel trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv1x1.py > gpurun_out/t51.log 2>&1 || exit 1
timeout -k 10 600 python3 bench.py --steps 30 --warmup 10 > gpurun_out/b51.log 2>&1 || exit 1
cd /tmp
timeout -k 10 500 rocprofv3 --kernel-trace -d /tmp/prof51 -o prof -- python3 $R/bench.py --steps 6 --warmup 3 > $R/gpurun_out/prof51.log 2>&1 || exit 1
DB=$(find /tmp/prof51 -name "*.db" | head -1)
python3 $R/tools/trace_summary.py $DB --steps 4 --marker mt_sgd --top 70 > $R/gpurun_out/prof51_resnet50.txt 2>&1
echo done
