#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_graphs.py -v --timeout 120 --timeout-method thread > gpurun_out/pytest_30.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_30.log
timeout -k 10 300 python -u tools/graph_numerics.py > gpurun_out/graph_num30.log 2>&1
echo done
