#!/bin/bash
# Sensitivity of the xGMI bucket-cap choice to the emulator's assumed bus
# bandwidth (VERDICT r4 Next 9): ResNet-50 / GPT-2 / BERT at emulated world 8,
# busbw 150 / 300 / 450 GB/s (the 300 GB/s of the r4 sweep +-50 %), caps
# 4 / 16 / 50 MiB (--bucket-sweep: one timed run per cap in one process),
# first 1 MiB, tail 2 MiB. One JSON line per run in gpurun_out/${TAG}.jsonl,
# each with exposed comm ms and the device-timed bucket readiness.
set -eo pipefail
TAG=${1:-r5_bucket_sensitivity}; STEPS=${STEPS:-10}; MODELS=${MODELS:-"resnet50 gpt2 bert"}
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$O"
for m in $MODELS; do
  for bw in 150 300 450; do
    timeout -k 10 400 python3 -u bench.py --model "$m" --steps "$STEPS" --warmup 5 --comm-timing 1 \
      --emulate-world 8 --emulate-busbw "$bw" --first-bucket-mb 1 --tail-bucket-mb 2 --bucket-sweep 4,16,50 \
      > "$O/${TAG}_run.log" 2>&1 || { tail -30 "$O/${TAG}_run.log"; exit 1; }
    grep '^{' "$O/${TAG}_run.log" | python3 -c "
import json, sys
for l in sys.stdin:
    d = json.loads(l); d['label'] = '$m w8 busbw$bw'; print(json.dumps(d))" | tee -a "$O/${TAG}.jsonl" | \
      python3 -c "
import json, sys
for l in sys.stdin:
    d = json.loads(l); c = d.get('comm', {})
    print(d['label'], 'cap', d['config'].get('bucket_cap_mb'), 'ms/step', d['ms_per_step'], 'exposed', c.get('exposed_comm_ms'),
          'ready_dev', c.get('bucket_ready_dev_ms'))"
  done
done
echo "[sensitivity] done"
