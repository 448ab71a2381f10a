#!/bin/bash
# stride-2 3x3 dgrad as four parity-class implicit GEMMs: tests + ResNet bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_conv1x1.py tests/test_gpu_models.py > gpurun_out/t58.log 2>&1 || exit 1
timeout -k 10 600 python3 bench.py --steps 30 --warmup 10 > gpurun_out/b58.log 2>&1 || exit 1
echo done
