#!/bin/bash
# FETCH_SIZE and WRITE_SIZE (separate passes: TCC slot limits) over a short
# ResNet-50 bench run, csv out under gpurun_out/pmc_bytes_{fetch,write}.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  tag=$(echo $c | tr 'A-Z' 'a-z' | cut -d_ -f1)
  timeout -s KILL 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$R/gpurun_out/pmc_bytes_$tag" -o pmc -- \
    python3 "$R/bench.py" --steps 3 --warmup 2 > "$R/gpurun_out/pmc_bytes_$tag.log" 2>&1
done
echo done
