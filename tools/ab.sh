#!/bin/bash
# A/B the headline bench under environment variants on ONE box (box-to-box
# spread is a few %, so compare arms of one call only).
#   gpurun -- bash tools/ab.sh TAG "BENCH_ARGS" "ENV_A" "ENV_B" ...
# ENV_x: space-separated VAR=value list ("-" = no extra env). Each arm runs
# bench.py once; the JSON lines go to gpurun_out/TAG_ab.jsonl with the arm name.
set -eo pipefail
TAG=${1:?tag}; ARGS=${2:-"--steps 20 --warmup 8"}; shift 2
mkdir -p gpurun_out
for arm in "$@"; do
  envs=(); [[ "$arm" != "-" ]] && read -r -a envs <<< "$arm"
  echo "[ab] $TAG arm: $arm"
  env "${envs[@]}" timeout -k 10 400 python3 -u bench.py $ARGS > gpurun_out/${TAG}_arm.log 2>&1 || {
    tail -20 gpurun_out/${TAG}_arm.log; exit 1; }
  line=$(grep '^{' gpurun_out/${TAG}_arm.log | tail -1)
  python3 -c "import json,sys; d=json.loads(sys.argv[1]); d['arm']=sys.argv[2]; print(json.dumps(d))" "$line" "$arm" \
    >> gpurun_out/${TAG}_ab.jsonl
  python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(f\"  {sys.argv[2]:50s} {d['value']:10.1f} samples/s  {d['ms_per_step']:.3f} ms\")" "$line" "$arm"
done
