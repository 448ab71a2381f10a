#!/bin/bash
# gathered 3x3 wgrad tests + bench; graph capture test with the GEMM path on/off
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv1x1.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_conv20.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_conv20.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_graphs.py -q --timeout 120 --timeout-method thread > gpurun_out/pytest_graphs20.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_graphs20.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 500 python bench.py --steps 30 --warmup 10 > gpurun_out/b20.json 2> gpurun_out/b20.err || exit 1
echo done
