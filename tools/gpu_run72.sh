#!/bin/bash
# bf16 shadow weights written by the fused AdamW: tests, A/B (DCP_BF16_SHADOWS=1/0) BERT + GPT-2, BERT trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_transformer_ops.py tests/test_gpu_models.py tests/test_gpu_ddp.py tests/test_gpu_graphs.py tests/test_gpu_kernels.py > gpurun_out/t72.log 2>&1 || exit 1
for m in bert gpt2; do
for g in 1 0 1; do
DCP_BF16_SHADOWS=$g timeout -k 10 400 python3 bench.py --model $m --steps 20 --warmup 5 > gpurun_out/b72_${m}_s$g.log 2>&1 || exit 1
grep '^{' gpurun_out/b72_${m}_s$g.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$m shadows=$g', d['value'], d['ms_per_step'])" >> gpurun_out/ab72.txt
done
done
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/p72b -o prof -- python3 $R/bench.py --model bert --steps 6 --warmup 3 > $R/gpurun_out/p72b.log 2>&1 || exit 1
DB=$(find /tmp/p72b -name "*.db" | head -1)
python3 $R/tools/trace_summary.py $DB --steps 4 --marker mt_adam_kernel --top 45 > $R/gpurun_out/prof72_bert.txt 2>&1
echo done
