#!/bin/bash
# First GPU validation: build check, GPU tests, bench (ours vs stock torch), rocprof stats.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
timeout -k 10 300 python -c "import distributed_compute_pytorch_amd as d; print('import ok')" > gpurun_out/import.log 2>&1 &&
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 400 python bench.py --fused-bn 0 --steps 20 --warmup 10 > gpurun_out/bench_ours.json 2> gpurun_out/bench_ours.err &&
timeout -k 10 400 python bench.py --impl torch --steps 20 --warmup 10 > gpurun_out/bench_torch.json 2> gpurun_out/bench_torch.err &&
timeout -k 10 400 python bench.py --impl torch --channels-last 0 --steps 20 --warmup 10 > gpurun_out/bench_torch_nchw.json 2> gpurun_out/bench_torch_nchw.err &&
cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_ours -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --fused-bn 0 --steps 10 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/prof_ours.log 2>&1
echo "exit=$?"
