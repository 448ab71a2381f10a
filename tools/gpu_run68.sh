#!/bin/bash
# LayerNorm backward workgroup cap: kernel trace of the LN shapes at 1024 vs 256 blocks, tests, BERT bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_transformer_ops.py > gpurun_out/t68.log 2>&1 || exit 1
cd /tmp
for cap in 1024 256 128; do
DCP_LN_BWD_BLOCKS=$cap timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d /tmp/p68_$cap -o p -- python3 $R/tools/kernel_bench.py --iters 10 > $R/gpurun_out/kb68_$cap.log 2>&1 || exit 1
find /tmp/p68_$cap -name "*kernel_stats.csv" -exec cp {} $R/gpurun_out/ks68_$cap.csv \;
done
cd $R
timeout -k 10 500 python3 bench.py --model bert --steps 20 --warmup 5 > gpurun_out/b68_bert.log 2>&1 || exit 1
echo done
