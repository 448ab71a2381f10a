#!/bin/bash
# Generic round-6 GPU step runner: TESTS (pytest files, stop on failure),
# then each command of CMDS (';;'-separated, each under its own timeout),
# stopping at the first failure. Output under gpurun_out/${TAG}_*.
set -o pipefail
TAG=${TAG:-r6}
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$O"
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest $TESTS -x -v --timeout 120 --timeout-method thread > "$O/${TAG}_tests.log" 2>&1
  rc=$?
  grep -E "FAILED|Error|passed|failed" "$O/${TAG}_tests.log" | tail -15
  if [ $rc -ne 0 ]; then echo "[r6_gpu] tests rc=$rc: stopping"; exit $rc; fi
fi
i=0
IFS=$'\n'
for c in $(echo "$CMDS" | sed 's/;;/\n/g'); do
  i=$((i+1))
  echo "[r6_gpu] step $i: $c"
  timeout -k 10 ${STEP_TIMEOUT:-300} bash -c "$c" > "$O/${TAG}_s$i.log" 2>&1
  rc=$?
  tail -${TAILN:-25} "$O/${TAG}_s$i.log"
  if [ $rc -ne 0 ]; then echo "[r6_gpu] step $i rc=$rc: stopping"; exit $rc; fi
done
echo "[r6_gpu] done"
