#!/bin/bash
# GELU kernels (gelu.hip, bias grad fused into the backward): full GPU suite, benches, GPT-2 kernel stats
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_transformer_ops.py > gpurun_out/t70_ops.log 2>&1 || exit 1
timeout -k 10 600 python3 -u -m pytest -m gpu -q --timeout 120 --timeout-method thread tests > gpurun_out/t70_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/t70_gpu.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 500 python3 bench.py --model gpt2 --steps 20 --warmup 5 > gpurun_out/b70_gpt2.log 2>&1 || exit 1
timeout -k 10 500 python3 bench.py --model bert --steps 20 --warmup 5 > gpurun_out/b70_bert.log 2>&1 || exit 1
timeout -k 10 500 python3 bench.py --steps 30 --warmup 10 > gpurun_out/b70_resnet.log 2>&1 || exit 1
cd /tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d /tmp/p70 -o p -- python3 $R/bench.py --model gpt2 --steps 5 --warmup 3 > $R/gpurun_out/p70_gpt2.log 2>&1 || exit 1
find /tmp/p70 -name "*kernel_stats.csv" -exec cp {} $R/gpurun_out/ks70_gpt2.csv \;
echo done
