#!/bin/bash
# Round-5 wgrad check: the ping-pong wgrad tests (+ the older wgrad users),
# the per-shape bench (pp vs ring vs hipBLASLt), then bench.py A/B of
# wg_pp = 1 / 0 on the models in MODELS. Stops at the first crash / hang.
set -o pipefail
TAG=${TAG:-r5w}; MODELS=${MODELS:-"resnet50 gpt2 bert"}; STEPS=${STEPS:-20}
TESTS=${TESTS:-"tests/test_gpu_wgrad_pp.py tests/test_gpu_conv1x1.py tests/test_gpu_lm_head.py"}
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$O"
if [ -n "$TESTS" ]; then
  timeout -k 10 500 python -u -m pytest $TESTS -x -v --timeout 120 --timeout-method thread > "$O/${TAG}_tests.log" 2>&1
  rc=$?
  grep -E "passed|failed|PASSED|FAILED|Error" "$O/${TAG}_tests.log" | tail -40
  if [ $rc -ne 0 ]; then echo "[r5_wgrad] tests rc=$rc: stopping"; exit $rc; fi
fi
if [ "${SHAPES:-1}" = 1 ]; then
  timeout -k 10 300 python -u tools/wgrad_pp_bench.py --rounds ${ROUNDS:-3} > "$O/${TAG}_shapes.jsonl" 2> "$O/${TAG}_shapes.err" || {
    echo "[r5_wgrad] shape bench failed"; tail -20 "$O/${TAG}_shapes.err"; exit 1; }
  cat "$O/${TAG}_shapes.jsonl"
fi
for m in $MODELS; do
  for v in 1 0; do
    timeout -k 10 300 python -u bench.py --model "$m" --steps "$STEPS" --warmup 8 --gemm-tune wg_pp=$v $BENCH_ARGS \
      > "$O/${TAG}_${m}_pp$v.log" 2>&1 || { echo "[r5_wgrad] bench $m pp=$v failed"; tail -20 "$O/${TAG}_${m}_pp$v.log"; exit 1; }
    grep '^{' "$O/${TAG}_${m}_pp$v.log" | tail -1 | python3 -c "
import json, sys
r = json.loads(sys.stdin.read()); r['wg_pp'] = $v
print(json.dumps(r))" | tee -a "$O/${TAG}_bench.jsonl" | cut -c1-200
  done
done
echo "[r5_wgrad] done"
