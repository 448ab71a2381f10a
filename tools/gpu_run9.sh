#!/bin/bash
# grad isolation, graph capture isolation, full GPU tests, ResNet/ConvNet bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
PYTHONPATH=. timeout -k 10 300 python tools/grad_diag.py > gpurun_out/grad_diag.txt 2>&1
echo "grad_diag rc=$?" >> gpurun_out/grad_diag.txt
true
true
timeout -k 10 900 python -m pytest tests -m gpu -q --ignore=tests/test_gpu_graphs.py > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
timeout -k 10 300 python -m pytest tests/test_gpu_graphs.py -q > gpurun_out/pytest_graphs.log 2>&1
echo "pytest graphs rc=$?" >> gpurun_out/pytest_graphs.log
b() { tag=$1; shift; timeout -k 10 400 python bench.py "$@" > gpurun_out/b9_$tag.json 2> gpurun_out/b9_$tag.err; tail -1 gpurun_out/b9_$tag.json >> gpurun_out/b9_summary.jsonl; }
b convnet_ours --model convnet --steps 200 --warmup 20
b convnet_torch --model convnet --steps 200 --warmup 20 --impl torch
b ours --steps 30 --warmup 10
b ours_graph --steps 30 --warmup 10 --graph 1
echo done
