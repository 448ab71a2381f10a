#!/bin/bash
# tests, ResNet bench + kernel profile, GPT-2/BERT kernel profiles
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -m pytest tests -m gpu -q --ignore=tests/test_gpu_graphs.py > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
timeout -k 10 300 python -m pytest tests/test_gpu_graphs.py -q > gpurun_out/pytest_graphs.log 2>&1
echo "pytest graphs rc=$?" >> gpurun_out/pytest_graphs.log
timeout -k 10 400 python bench.py --steps 30 --warmup 10 > gpurun_out/b11_ours.json 2> gpurun_out/b11_ours.err || exit 1
tail -1 gpurun_out/b11_ours.json >> gpurun_out/b11_summary.jsonl
cd /tmp
for m in resnet50 gpt2 bert; do
  mk=mt_sgd; [ $m != resnet50 ] && mk=mt_adam
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof11_$m -o prof -- python3 $R/bench.py --model $m --steps 6 --warmup 3 > $R/gpurun_out/prof11_$m.log 2>&1 || exit 1
  python3 $R/tools/trace_summary.py $(ls /tmp/prof11_$m/*/prof_results.db /tmp/prof11_$m/prof_results.db 2>/dev/null | head -1) --steps 4 --marker $mk --top 45 > $R/gpurun_out/prof11_$m.txt 2>&1
done
timeout -k 10 300 python3 $R/tools/kernel_bench.py --json $R/gpurun_out/kbench11.json > $R/gpurun_out/kbench11.log 2>&1 || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $c --kernel-trace --output-format csv -d /tmp/pmc11_$c -o pmc -- python3 $R/tools/kernel_bench.py --iters 3 > $R/gpurun_out/pmc11_$c.log 2>&1 || exit 1
  python3 $R/tools/pmc_summary.py /tmp/pmc11_$c --top 40 > $R/gpurun_out/pmc11_$c.txt 2>&1
done
echo done
