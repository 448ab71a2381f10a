R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/hw; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/hw_auto -o run -- python3 $R/bench.py --model gpt2 --steps 3 --warmup 2 --graph 0 > $O/auto.log 2>&1 || { tail -20 $O/auto.log; exit 1; }
python3 $R/tools/long_kernel_trace.py /tmp/hw_auto/run_results.db --min-us 300 --window 120 --match wgrad > $O/auto_trace.txt 2>&1
echo '{"head_wgrad 8192 50304 768": "ring"}' > /tmp/pin.json
DCP_LINEAR_CHOICES=/tmp/pin.json timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/hw_ring -o run -- python3 $R/bench.py --model gpt2 --steps 3 --warmup 2 --graph 0 > $O/ring.log 2>&1 || { tail -20 $O/ring.log; exit 1; }
python3 $R/tools/long_kernel_trace.py /tmp/hw_ring/run_results.db --min-us 300 > $O/ring_trace.txt 2>&1
tail -1 $O/auto.log; tail -1 $O/ring.log
