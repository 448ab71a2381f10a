#!/bin/bash
# Compute/communication overlap on ONE GPU (VERDICT r2 Next #2, NOTES §22):
# ResNet-50 b512 step time and exposed communication for
#   * the default single-process path (no comm stream: collectives are no-ops at N = 1),
#   * DCP_SINGLE_RANK_HOP=1: the real N > 1 code path (comm stream, event edges, RCCL calls),
#   * the contention emulation of an 8-rank ring all-reduce (comm_hooks.contention_emulation_hook)
#     at several CU reservations of the persistent GEMM grids.
# One JSON line per run in gpurun_out/${TAG}_overlap.jsonl.
set -eo pipefail
TAG=${1:-overlap}; STEPS=${2:-20}
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$O"
run() {  # label, env..., -- bench args
  local label=$1; shift
  local envs=()
  while [[ $1 != -- ]]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python3 -u bench.py --steps "$STEPS" --warmup 8 "$@" > "$O/${TAG}_run.log" 2>&1 || {
    tail -20 "$O/${TAG}_run.log"; exit 1; }
  grep '^{' "$O/${TAG}_run.log" | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); d['label']='$label'; print(json.dumps(d))" | tee -a "$O/${TAG}_overlap.jsonl"
}
run default X=1 --
run hop DCP_SINGLE_RANK_HOP=1 -- --comm-timing 1
for r in 0 8 16 32; do
  run "emu8_reserve$r" X=1 -- --comm-timing 1 --emulate-world 8 --reserve-cus $r
done
run "emu8_reserve0_prio" DCP_COMM_STREAM_PRIORITY=high -- --comm-timing 1 --emulate-world 8 --reserve-cus 0
echo "[overlap_sweep] done"
