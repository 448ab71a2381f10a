#!/bin/bash
# gemm_pp numerics tests, then (only if they ran to completion without a
# crash / hang) the gemm_pp vs ring vs hipBLASLt bench.
set -o pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$O"
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm_pp.py -x -q --timeout 120 --timeout-method thread \
  > "$O/pp_test.log" 2>&1
rc=$?
tail -5 "$O/pp_test.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "[pp_run] tests ended with rc=$rc: stopping"; exit $rc; fi
timeout -k 10 420 python -u tools/gemm_pp_bench.py --rounds 3 --iters 10 --json "$O/pp_bench.jsonl" \
  > "$O/pp_bench.log" 2>&1 || { tail -20 "$O/pp_bench.log"; exit 1; }
cat "$O/pp_bench.log" | cut -c1-400
