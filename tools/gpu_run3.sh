#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
for tag in a b; do
  timeout -k 10 400 python bench.py --impl torch --steps 30 --warmup 10 > gpurun_out/b_torch_$tag.json 2> gpurun_out/b_torch_$tag.err || exit 1
  timeout -k 10 400 python bench.py --fused-bn 1 --steps 30 --warmup 10 > gpurun_out/b_ours_fbn_$tag.json 2> gpurun_out/b_ours_fbn_$tag.err || exit 1
  timeout -k 10 400 python bench.py --fused-bn 0 --steps 30 --warmup 10 > gpurun_out/b_ours_$tag.json 2> gpurun_out/b_ours_$tag.err || exit 1
done
timeout -k 10 400 python bench.py --impl torch --benchmark-cudnn 0 --steps 30 --warmup 10 > gpurun_out/b_torch_nobench.json 2> gpurun_out/b_torch_nobench.err
timeout -k 10 400 python bench.py --fused-bn 1 --benchmark-cudnn 0 --steps 30 --warmup 10 > gpurun_out/b_ours_nobench.json 2> gpurun_out/b_ours_nobench.err
mkdir -p gpurun_out/miopen_db && cp -r ~/.config/miopen/* gpurun_out/miopen_db/ 2>/dev/null; ls -la ~/.config/miopen ~/.cache/miopen > gpurun_out/miopen_ls.txt 2>&1
echo done
