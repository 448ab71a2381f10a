#!/bin/bash
# MFMA 1x1-conv GEMMs: numerics tests, kernel bench vs MIOpen, ResNet-50 bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv1x1.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_conv13.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_conv13.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u tools/gemm_bench.py --json gpurun_out/gemm13.json > gpurun_out/gemm13.log 2>&1 || exit 1
[ $rc -eq 0 ] || exit 1
timeout -k 10 500 python bench.py --steps 30 --warmup 10 > gpurun_out/b13_ours.json 2> gpurun_out/b13_ours.err || exit 1
echo done
