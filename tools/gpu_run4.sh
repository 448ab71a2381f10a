#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in ours torch ours_ddp_torch_opt torch_ddp_ours_opt noddp_ours_opt; do
  timeout -k 10 300 python tools/step_breakdown.py --variant $v > gpurun_out/sb_$v.txt 2>&1 || exit 1
done
timeout -k 10 300 python tools/step_breakdown.py --variant ours --fused 0 --profile 0 > gpurun_out/sb_ours_nofuse.txt 2>&1
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
timeout -k 10 600 python tools/conv_vs_gemm.py > gpurun_out/conv_vs_gemm.txt 2>&1
echo done
