#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
timeout -k 10 400 python bench.py --fused-bn 1 --steps 20 --warmup 10 > gpurun_out/bench_ours_fbn.json 2> gpurun_out/bench_ours_fbn.err &&
timeout -k 10 400 python bench.py --fused-bn 0 --steps 20 --warmup 10 > gpurun_out/bench_ours.json 2> gpurun_out/bench_ours.err &&
timeout -k 10 400 python bench.py --impl torch --steps 20 --warmup 10 > gpurun_out/bench_torch.json 2> gpurun_out/bench_torch.err &&
cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_ours -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --fused-bn 1 --steps 10 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/prof_ours.log 2>&1
echo "exit=$?"
