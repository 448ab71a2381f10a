set -o pipefail
mkdir -p gpurun_out
bash tools/gpu.sh r2b prof=--steps,6,--warmup,3 || exit 1
python3 tools/step_timeline.py $(ls gpurun_out/r2b_prof/*/*.db 2>/dev/null | head -1 || true) > gpurun_out/r2b_timeline.txt 2>&1
python3 tools/step_timeline.py $(ls gpurun_out/r2b_prof/*/*.db 2>/dev/null | head -1 || true) --group > gpurun_out/r2b_group.txt 2>&1
ls -R gpurun_out/r2b_prof | head -20
timeout -k 10 300 python3 -u -m pytest -x -v -m gpu --timeout 240 --timeout-method thread --runxfail -k "captured_step_matches_eager" tests > gpurun_out/r2b_graph.log 2>&1
tail -30 gpurun_out/r2b_graph.log
exit 0
