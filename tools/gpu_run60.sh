#!/bin/bash
# A/B: parity stride-2 dgrad (view-based weight subsets) on/off, interleaved twice
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv1x1.py > gpurun_out/t60.log 2>&1 || exit 1
for r in 1 2; do
DCP_S2_DGRAD_PARITY=1 timeout -k 10 600 python3 bench.py --steps 30 --warmup 10 > gpurun_out/b60_par$r.log 2>&1 || exit 1
timeout -k 10 600 python3 bench.py --steps 30 --warmup 10 > gpurun_out/b60_off$r.log 2>&1 || exit 1
done
echo done
