#!/bin/bash
# slab-reduce fix; GEMM bench; ResNet-50 bench with the GEMM path on/off; kernel profile.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv1x1.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_conv17.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_conv17.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u tools/gemm_bench.py --json gpurun_out/gemm17.json > gpurun_out/gemm17.log 2>&1 || exit 1
timeout -k 10 500 python bench.py --steps 30 --warmup 10 --gemm 1 > gpurun_out/b17_gemm1.json 2> gpurun_out/b17_gemm1.err || exit 1
timeout -k 10 500 python bench.py --steps 30 --warmup 10 --gemm 0 > gpurun_out/b17_gemm0.json 2> gpurun_out/b17_gemm0.err || exit 1
cd /tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d /tmp/prof17 -o prof -- python3 $R/bench.py --steps 6 --warmup 3 > $R/gpurun_out/prof17_resnet50.log 2>&1 || exit 1
python3 $R/tools/trace_summary.py $(ls /tmp/prof17/*/prof_results.db /tmp/prof17/prof_results.db 2>/dev/null | head -1) --steps 4 --marker mt_sgd --top 60 > $R/gpurun_out/prof17_resnet50.txt 2>&1
echo done
