#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TORCH_SHOW_CPP_STACKTRACES=1 timeout -k 10 400 python tools/graph_debug.py > gpurun_out/graph_debug.txt 2>&1
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
b() { tag=$1; shift; timeout -k 10 400 python bench.py "$@" > gpurun_out/b8_$tag.json 2> gpurun_out/b8_$tag.err; tail -1 gpurun_out/b8_$tag.json >> gpurun_out/b8_summary.jsonl; }
b ours --steps 30 --warmup 10
b ours_b384 --steps 20 --warmup 8 --batch 384
echo done
