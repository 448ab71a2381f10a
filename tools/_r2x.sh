set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 200 python3 -u -m pytest -x -v -m gpu --timeout 120 --timeout-method thread -k "conv3x3_c64_direct" tests/test_gpu_conv1x1.py > gpurun_out/r2x_t1.log 2>&1 || { grep -v "^  File" gpurun_out/r2x_t1.log | tail -40; exit 1; }
tail -1 gpurun_out/r2x_t1.log
timeout -k 10 300 python3 -u -m pytest -x -q -m gpu --timeout 240 --timeout-method thread -k "conv or gemm or stem or fusions or resnet or graph" tests > gpurun_out/r2x_tests.log 2>&1 || { tail -30 gpurun_out/r2x_tests.log; exit 1; }
tail -1 gpurun_out/r2x_tests.log
for arm in 0 1; do
  DCP_CONV3_DIRECT=$arm timeout -k 10 300 python3 -u tools/gemm_bench.py --batch 512 --iters 10 --only3x3 > gpurun_out/r2x_g$arm.log 2>&1
done
grep -h '56x56 c=64' gpurun_out/r2x_g0.log gpurun_out/r2x_g1.log | cut -c1-260
bash tools/ab.sh r2x "--steps 20 --warmup 8" "DCP_CONV3_DIRECT=0" "-" "DCP_CONV3_DIRECT=0" "-"
