#!/bin/bash
# BERT-base and GPT-2 eager kernel traces: per-kernel time, wall vs kernel sum
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/p64b -o prof -- python3 $R/bench.py --model bert --steps 6 --warmup 3 > $R/gpurun_out/p64b.log 2>&1 || exit 1
DB=$(find /tmp/p64b -name "*.db" | head -1)
python3 $R/tools/trace_summary.py $DB --steps 4 --marker mt_adam_kernel --top 45 > $R/gpurun_out/prof64_bert.txt 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/p64g -o prof -- python3 $R/bench.py --model gpt2 --steps 4 --warmup 2 > $R/gpurun_out/p64g.log 2>&1 || exit 1
DB=$(find /tmp/p64g -name "*.db" | head -1)
python3 $R/tools/trace_summary.py $DB --steps 3 --marker mt_adam_kernel --top 45 > $R/gpurun_out/prof64_gpt2.txt 2>&1
echo done
