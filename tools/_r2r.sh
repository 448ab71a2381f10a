set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q -m gpu --timeout 240 --timeout-method thread -k "stem or fusions or graph" tests > gpurun_out/r2r_tests.log 2>&1 || { tail -30 gpurun_out/r2r_tests.log; exit 1; }
tail -1 gpurun_out/r2r_tests.log
bash tools/ab.sh r2r "--steps 20 --warmup 8" "-" "-"
bash tools/gpu.sh r2r "prof=--steps,10,--warmup,5"
