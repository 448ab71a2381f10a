#!/bin/bash
# full GPU suite + smoke + headline bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu28.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu28.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke28.log 2>&1 || exit 1
timeout -k 10 500 python bench.py > gpurun_out/b28.json 2> gpurun_out/b28.err || exit 1
echo done
