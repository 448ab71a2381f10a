#!/bin/bash
# v2 GEMMs (glds ring): numerics tests, kernel bench vs MIOpen.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv1x1.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_conv14.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_conv14.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u tools/gemm_bench.py --json gpurun_out/gemm14.json > gpurun_out/gemm14.log 2>&1 || exit 1
echo done
