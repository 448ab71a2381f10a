#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { tag=$1; shift; timeout -k 10 300 "$@" --tag $tag > gpurun_out/sb5_$tag.txt 2>&1; grep '^{' gpurun_out/sb5_$tag.txt >> gpurun_out/sb5_summary.jsonl; }
run ours_default python tools/step_breakdown.py --variant ours --profile 0
DCP_SINGLE_RANK_HOP=1 run ours_hop_normal python tools/step_breakdown.py --variant ours --profile 0
DCP_SINGLE_RANK_HOP=1 DCP_COMM_STREAM_PRIORITY=high run ours_hop_high python tools/step_breakdown.py --variant ours --profile 0
run torch_fusedmodel python tools/step_breakdown.py --variant torch --fused-model 1 --profile 0
run torch_plain python tools/step_breakdown.py --variant torch --profile 0
run ours_nofuse python tools/step_breakdown.py --variant ours --fused 0 --profile 0
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
echo done
