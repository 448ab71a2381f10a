#!/bin/bash
# full GPU test suite after the GEMM/BN changes
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu19.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu19.log
echo done
