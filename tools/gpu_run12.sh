#!/bin/bash
# Re-verify the tree after the container rebuild: GPU tests, ResNet-50 bench,
# kernel-trace profile of the ResNet step, PMC byte counters of our kernels.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu12.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu12.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python bench.py --steps 30 --warmup 10 > gpurun_out/b12_ours.json 2> gpurun_out/b12_ours.err || exit 1
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof12 -o prof -- python3 $R/bench.py --steps 6 --warmup 3 > $R/gpurun_out/prof12_resnet50.log 2>&1 || exit 1
python3 $R/tools/trace_summary.py $(ls /tmp/prof12/*/prof_results.db /tmp/prof12/prof_results.db 2>/dev/null | head -1) --steps 4 --marker mt_sgd --top 45 > $R/gpurun_out/prof12_resnet50.txt 2>&1
timeout -k 10 300 python3 $R/tools/kernel_bench.py --json $R/gpurun_out/kbench12.json > $R/gpurun_out/kbench12.log 2>&1 || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d /tmp/pmc12_$c -o pmc -- python3 $R/tools/kernel_bench.py --iters 3 > $R/gpurun_out/pmc12_$c.log 2>&1 || exit 1
  python3 $R/tools/pmc_summary.py /tmp/pmc12_$c --top 40 > $R/gpurun_out/pmc12_$c.txt 2>&1
done
echo done
