#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_attention.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_attn23.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_attn23.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u tools/attn_bench.py > gpurun_out/attn23.log 2>&1 || exit 1
echo done
