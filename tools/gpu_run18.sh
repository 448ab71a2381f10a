#!/bin/bash
# dispatch by block intensity (layers 1-3 on our GEMMs); wgrad split cap relaxed
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv1x1.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_conv18.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_conv18.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u tools/gemm_bench.py --json gpurun_out/gemm18.json > gpurun_out/gemm18.log 2>&1 || exit 1
timeout -k 10 500 python bench.py --steps 30 --warmup 10 > gpurun_out/b18_l3.json 2> gpurun_out/b18_l3.err || exit 1
DCP_GEMM_MAX_INTENSITY=1000 timeout -k 10 500 python bench.py --steps 30 --warmup 10 > gpurun_out/b18_l4.json 2> gpurun_out/b18_l4.err || exit 1
DCP_GEMM_MAX_INTENSITY=150 timeout -k 10 500 python bench.py --steps 30 --warmup 10 > gpurun_out/b18_l2.json 2> gpurun_out/b18_l2.err || exit 1
echo done
