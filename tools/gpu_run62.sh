#!/bin/bash
# HIP-graph whole-step capture vs eager on the three workloads
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 bench.py --steps 30 --warmup 10 --graph 1 > gpurun_out/b62_resnet_graph.log 2>&1 || exit 1
timeout -k 10 500 python3 bench.py --model bert --steps 20 --warmup 5 --graph 1 > gpurun_out/b62_bert_graph.log 2>&1 || exit 1
timeout -k 10 500 python3 bench.py --model gpt2 --steps 20 --warmup 5 --graph 1 > gpurun_out/b62_gpt2_graph.log 2>&1 || exit 1
echo done
