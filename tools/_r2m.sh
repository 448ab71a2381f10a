set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q -m gpu --timeout 240 --timeout-method thread -k "conv or gemm or stem or fusions or wgrad or resnet" tests > gpurun_out/r2m_tests.log 2>&1 || { tail -30 gpurun_out/r2m_tests.log; exit 1; }
tail -1 gpurun_out/r2m_tests.log
DCP_WGRAD_ORDER=0 timeout -k 10 300 python3 -u tools/gemm_bench.py --batch 512 --iters 10 > gpurun_out/r2m_gemm_o0.log 2>&1
DCP_WGRAD_ORDER=1 timeout -k 10 300 python3 -u tools/gemm_bench.py --batch 512 --iters 10 > gpurun_out/r2m_gemm_o1.log 2>&1
bash tools/ab.sh r2m "--steps 20 --warmup 8" "DCP_WGRAD_ORDER=0" "DCP_WGRAD_ORDER=1" "DCP_WGRAD_ORDER=0" "DCP_WGRAD_ORDER=1"
