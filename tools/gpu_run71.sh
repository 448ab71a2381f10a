#!/bin/bash
# GELU A/B on one box (DCP_FUSED_GELU=1/0) for BERT and GPT-2, then kernel traces with the fused GELU
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for m in bert gpt2; do
for g in 1 0 1; do
DCP_FUSED_GELU=$g timeout -k 10 400 python3 bench.py --model $m --steps 20 --warmup 5 > gpurun_out/b71_${m}_g$g.log 2>&1 || exit 1
grep '^{' gpurun_out/b71_${m}_g$g.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$m gelu=$g', d['value'], d['ms_per_step'])" >> gpurun_out/ab71.txt
done
done
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/p71b -o prof -- python3 $R/bench.py --model bert --steps 6 --warmup 3 > $R/gpurun_out/p71b.log 2>&1 || exit 1
DB=$(find /tmp/p71b -name "*.db" | head -1)
python3 $R/tools/trace_summary.py $DB --steps 4 --marker mt_adam_kernel --top 45 > $R/gpurun_out/prof71_bert.txt 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/p71g -o prof -- python3 $R/bench.py --model gpt2 --steps 4 --warmup 2 > $R/gpurun_out/p71g.log 2>&1 || exit 1
DB=$(find /tmp/p71g -name "*.db" | head -1)
python3 $R/tools/trace_summary.py $DB --steps 3 --marker mt_adam_kernel --top 45 > $R/gpurun_out/prof71_gpt2.txt 2>&1
echo done
