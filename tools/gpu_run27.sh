#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_transformer_ops.py tests/test_gpu_attention.py tests/test_gpu_models.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_27.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_27.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 tools/kernel_bench.py > gpurun_out/kbench27.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --model bert --steps 10 --warmup 4 > gpurun_out/b27_bert.json 2> gpurun_out/b27_bert.err || exit 1
timeout -k 10 400 python bench.py --model gpt2 --steps 10 --warmup 4 > gpurun_out/b27_gpt2.json 2> gpurun_out/b27_gpt2.err || exit 1
cd /tmp
for m in bert gpt2; do
  timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/prof27_$m -o prof -- python3 $R/bench.py --model $m --steps 6 --warmup 3 > $R/gpurun_out/prof27_$m.log 2>&1 || exit 1
  python3 $R/tools/trace_summary.py $(find /tmp/prof27_$m -name "*.db" | head -1) --steps 4 --marker mt_adam --top 40 > $R/gpurun_out/prof27_$m.txt 2>&1
done
echo done
