#!/bin/bash
# LayerNorm dγ/dβ accumulated in the finalize kernel under no_sync: tests, GPT-2 A/B (DCP_LN_ACCUM=1/0)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_transformer_ops.py tests/test_gpu_models.py tests/test_gpu_ddp.py > gpurun_out/t74.log 2>&1 || exit 1
tail -2 gpurun_out/t74.log
for g in 1 0 1 0; do
DCP_LN_ACCUM=$g timeout -k 10 400 python3 bench.py --model gpt2 --steps 20 --warmup 5 > gpurun_out/b74_s$g.log 2>&1 || exit 1
grep '^{' gpurun_out/b74_s$g.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('gpt2 ln_accum=$g', d['value'], d['ms_per_step'])" >> gpurun_out/ab74.txt
done
cat gpurun_out/ab74.txt
