#!/bin/bash
# ResNet bench (wide conv3 materialised), graph test; BERT / GPT-2 kernel profiles
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_graphs.py tests/test_gpu_conv1x1.py -q --timeout 120 --timeout-method thread > gpurun_out/pytest_22.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_22.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 500 python bench.py --steps 30 --warmup 10 > gpurun_out/b22.json 2> gpurun_out/b22.err || exit 1
DCP_PRO_MAX_COUT=4096 timeout -k 10 500 python bench.py --steps 30 --warmup 10 > gpurun_out/b22_proall.json 2> gpurun_out/b22_proall.err || exit 1
cd /tmp
for m in bert gpt2; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof22_$m -o prof -- python3 $R/bench.py --model $m --steps 6 --warmup 3 > $R/gpurun_out/prof22_$m.log 2>&1 || exit 1
  python3 $R/tools/trace_summary.py $(ls /tmp/prof22_$m/*/prof_results.db /tmp/prof22_$m/prof_results.db 2>/dev/null | head -1) --steps 4 --marker mt_adam --top 45 > $R/gpurun_out/prof22_$m.txt 2>&1
done
echo done
