#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
b() { tag=$1; shift; timeout -k 10 400 python bench.py "$@" > gpurun_out/b7_$tag.json 2> gpurun_out/b7_$tag.err; tail -1 gpurun_out/b7_$tag.json >> gpurun_out/b7_summary.jsonl; }
b ours --steps 30 --warmup 10
b ours_graph --steps 30 --warmup 10 --graph 1
b gpt2_ours --model gpt2 --steps 10 --warmup 4
b gpt2_torch --model gpt2 --impl torch --steps 10 --warmup 4
b bert_ours --model bert --steps 10 --warmup 4
b bert_torch --model bert --impl torch --steps 10 --warmup 4
cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof7 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/prof7.log 2>&1
echo done
