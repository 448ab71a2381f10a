#!/bin/bash
# ConvNet (the reference model): GPU tests, bench (HIP graph by default), and a
# rocprofv3 --kernel-trace --stats profile -> gpurun_out/convnet_prof/*
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O/convnet_prof"
timeout -k 10 300 python -u -m pytest tests/test_gpu_convnet.py -x -q --timeout 120 --timeout-method thread > "$O/convnet_tests.log" 2>&1
rc=$?; tail -3 "$O/convnet_tests.log"
if [ $rc -ne 0 ]; then echo "[convnet_prof] tests rc=$rc: stopping"; exit 1; fi
for g in 1 0; do
  timeout -k 10 300 python -u bench.py --model convnet --steps 200 --warmup 30 --graph $g > "$O/convnet_bench_g$g.log" 2>&1 || { tail -20 "$O/convnet_bench_g$g.log"; exit 1; }
  grep '^{' "$O/convnet_bench_g$g.log" | tail -1 | tee -a "$O/convnet_bench.jsonl" | cut -c1-250
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/convnet_prof" -o run -- python3 "$R/bench.py" --model convnet --steps 60 --warmup 10 --graph 0 > "$O/convnet_prof.log" 2>&1 || { tail -20 "$O/convnet_prof.log"; exit 1; }
echo "[convnet_prof] done"
