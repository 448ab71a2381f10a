#!/bin/bash
# GPU clock / power while a bench runs: rocm-smi samples every second next to
# `python bench.py $BENCH_ARGS` (read-only queries). Output:
# gpurun_out/${TAG}_clk.txt (samples) and ${TAG}_bench.log.
TAG=${TAG:-clk}; BENCH_ARGS=${BENCH_ARGS:-"--steps 300 --warmup 10"}
mkdir -p gpurun_out
timeout -k 10 300 python3 -u bench.py $BENCH_ARGS > gpurun_out/${TAG}_bench.log 2>&1 &
BP=$!
for i in $(seq 1 120); do
  kill -0 $BP 2>/dev/null || break
  echo "t=$i $(date +%s.%N)" >> gpurun_out/${TAG}_clk.txt
  timeout 10 rocm-smi --showclocks --showpower >> gpurun_out/${TAG}_clk.txt 2>&1
  sleep 1
done
wait $BP; rc=$?
tail -1 gpurun_out/${TAG}_bench.log
exit $rc
