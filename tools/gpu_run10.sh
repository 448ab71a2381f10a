#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
PYTHONPATH=. timeout -k 10 300 python tools/grad_diag.py > gpurun_out/grad_diag.txt 2>&1
echo "grad_diag rc=$?" >> gpurun_out/grad_diag.txt
timeout -k 10 900 python -m pytest tests -m gpu -q --ignore=tests/test_gpu_graphs.py > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
timeout -k 10 300 python -m pytest tests/test_gpu_graphs.py -q > gpurun_out/pytest_graphs.log 2>&1
echo "pytest graphs rc=$?" >> gpurun_out/pytest_graphs.log
b() { tag=$1; shift; timeout -k 10 400 python bench.py "$@" > gpurun_out/b10_$tag.json 2> gpurun_out/b10_$tag.err; tail -1 gpurun_out/b10_$tag.json >> gpurun_out/b10_summary.jsonl; }
b convnet_ours --model convnet --steps 300 --warmup 30
b convnet_ours_graph --model convnet --steps 300 --warmup 30 --graph 1
b ours --steps 30 --warmup 10
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof10 -o prof -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/prof10.log 2>&1
echo "prof rc=$?" >> $GRAFT_REPO_ROOT/gpurun_out/prof10.log
echo done
