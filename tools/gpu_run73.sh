#!/bin/bash
# round-end evidence on the committed tree: full GPU suite, smoke(), the three
# GPU benches (default bench.py = ResNet-50), a rocprofv3 --stats of ResNet-50
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest -x -v -m gpu --timeout 120 --timeout-method thread tests > gpurun_out/t73.log 2>&1 || exit 1
tail -3 gpurun_out/t73.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke73.log 2>&1 || exit 1
timeout -k 10 400 python3 bench.py > gpurun_out/b73_resnet50.log 2>&1 || exit 1
grep '^{' gpurun_out/b73_resnet50.log
for m in bert gpt2; do
timeout -k 10 400 python3 bench.py --model $m --steps 20 --warmup 5 > gpurun_out/b73_$m.log 2>&1 || exit 1
grep '^{' gpurun_out/b73_$m.log
done
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/p73 -o prof -- python3 $R/bench.py --steps 6 --warmup 3 > $R/gpurun_out/p73.log 2>&1 || exit 1
echo done
