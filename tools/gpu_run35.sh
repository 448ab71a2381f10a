#!/bin/bash
# BN reduce kernels after the unroll: sweep the row-slab cap
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/bn_sweep35.log
: > $O
for cfg in "DCP_BN_RED_ROWBLK=512" "DCP_BN_RED_ROWBLK=256" "DCP_BN_RED_ROWBLK=1024" "DCP_BN_RED_ROWBLK=128"; do
  echo "== $cfg" >> $O
  env $cfg timeout -k 10 120 python3 tools/bn_sweep.py --iters 20 >> $O 2>&1 || exit 1
done
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_batchnorm.py > gpurun_out/t35.log 2>&1 || exit 1
echo done
