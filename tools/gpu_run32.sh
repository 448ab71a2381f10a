#!/bin/bash
# BN geometry sweep on every ResNet-50 BN shape (one process per setting: the knobs are read once)
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/bn_sweep32.log
: > $O
for cfg in "" "DCP_BN_RED_BLOCKS=1024" "DCP_BN_RED_BLOCKS=512" "DCP_BN_RED_BLOCKS=4096 DCP_BN_RED_ATOMICS=524288" "DCP_BN_RED_ATOMICS=32768" "DCP_BN_RED_BLOCKS=1024 DCP_BN_RED_ATOMICS=32768"; do
  echo "== $cfg" >> $O
  env $cfg timeout -k 10 120 python3 tools/bn_sweep.py --iters 20 >> $O 2>&1 || exit 1
done
echo done
