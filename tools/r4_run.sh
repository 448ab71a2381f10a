#!/bin/bash
# Round-4 GPU check: selected GPU tests, then bench.py for the listed models
# (one JSON line each in gpurun_out/${TAG}_bench.jsonl). Stops at the first
# crash / hang (exit status other than 0 / 1 from pytest).
set -o pipefail
TAG=${TAG:-r4}; TESTS=${TESTS:-"tests/test_gpu_gemm_pp.py tests/test_gpu_transformer_ops.py"}
MODELS=${MODELS:-"gpt2 bert resnet50"}; STEPS=${STEPS:-20}
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$O"
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread > "$O/${TAG}_tests.log" 2>&1
  rc=$?
  tail -5 "$O/${TAG}_tests.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "[r4_run] tests rc=$rc: stopping"; exit $rc; fi
fi
for m in $MODELS; do
  timeout -k 10 400 python -u bench.py --model "$m" --steps "$STEPS" --warmup 8 $BENCH_ARGS > "$O/${TAG}_${m}.log" 2>&1 || {
    echo "[r4_run] bench $m failed"; tail -20 "$O/${TAG}_${m}.log"; exit 1; }
  grep '^{' "$O/${TAG}_${m}.log" | tail -1 | tee -a "$O/${TAG}_bench.jsonl" | cut -c1-300
  # the per-shape GEMM autotune table (us per candidate) of that run
  grep '^{' "$O/${TAG}_${m}.log" | tail -1 | python3 -c "
import json, sys
c = json.loads(sys.stdin.read())['config'].get('linear_gemm_us_by_candidate') or {}
for k, v in sorted(c.items()): print('  ', k, v)"
done
echo "[r4_run] done"
