#!/bin/bash
# full GPU suite + smoke + the three workload benches (ResNet-50 default, BERT-base, GPT-2-small)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu56.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu56.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke56.log 2>&1 || exit 1
timeout -k 10 500 python bench.py > gpurun_out/b56_resnet.json 2> gpurun_out/b56_resnet.err || exit 1
timeout -k 10 500 python bench.py --model bert --steps 20 --warmup 5 > gpurun_out/b56_bert.json 2> gpurun_out/b56_bert.err || exit 1
timeout -k 10 500 python bench.py --model gpt2 --steps 20 --warmup 5 > gpurun_out/b56_gpt2.json 2> gpurun_out/b56_gpt2.err || exit 1
echo done
