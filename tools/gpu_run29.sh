#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_graphs.py tests/test_gpu_attention.py -q --timeout 120 --timeout-method thread > gpurun_out/pytest_29.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_29.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u tools/attn_bench.py > gpurun_out/attn29.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --model bert --steps 10 --warmup 4 > gpurun_out/b29_bert.json 2> gpurun_out/b29_bert.err || exit 1
timeout -k 10 400 python bench.py --model gpt2 --steps 10 --warmup 4 > gpurun_out/b29_gpt2.json 2> gpurun_out/b29_gpt2.err || exit 1
echo done
