#!/bin/bash
# xGMI bucket plan from the one-GPU contention emulator (VERDICT r3 Next #4,
# BASELINE config #4): every bucket all-reduce replaced by an
# N-rank ring all-reduce emulation on the comm stream (parallel/comm_hooks.py),
# per-bucket device time + exposed (un-overlapped) comm recorded.
#   * cap sweep 4..100 MiB at first-bucket 0.25 / 1 / 4 MiB, emulated world 8;
#   * tail split 0 / 2 / 8 MiB at the default cap;
#   * world 2 / 4 at two caps.
# One JSON line per timed run in gpurun_out/${TAG}.jsonl.
set -eo pipefail
TAG=${1:-bucket_sweep_emu}; STEPS=${STEPS:-12}; MODELS=${MODELS:-"resnet50 bert gpt2"}
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$O"
run() {  # label, bench args...
  local label=$1; shift
  timeout -k 10 420 python3 -u bench.py --steps "$STEPS" --warmup 6 --comm-timing 1 "$@" \
    > "$O/${TAG}_run.log" 2>&1 || { tail -30 "$O/${TAG}_run.log"; exit 1; }
  grep '^{' "$O/${TAG}_run.log" | python3 -c "
import json, sys
for l in sys.stdin:
    d = json.loads(l); d['label'] = '$label'; print(json.dumps(d))" | tee -a "$O/${TAG}.jsonl" | cut -c1-200
}
for m in $MODELS; do
  for f in 0.25 1 4; do
    run "$m w8 first$f" --model "$m" --emulate-world 8 --first-bucket-mb "$f" --tail-bucket-mb 2 \
      --bucket-sweep 4,8,16,25,50,100
  done
  for t in 0 8; do
    run "$m w8 tail$t" --model "$m" --emulate-world 8 --tail-bucket-mb "$t" --bucket-sweep 25,50
  done
  for w in 2 4; do
    run "$m w$w" --model "$m" --emulate-world "$w" --bucket-sweep 25,50
  done
done
echo "[bucket_sweep_emu] done"
