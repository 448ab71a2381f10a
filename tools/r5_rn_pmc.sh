#!/bin/bash
# ResNet-50 bench (3 steps) under rocprofv3 PMC: FETCH_SIZE, WRITE_SIZE and the
# MFMA-busy group in separate passes; per (kernel, grid) summaries in
# gpurun_out/${TAG}_*.txt (tools/pmc_by_dispatch.py).
set -o pipefail
TAG=${TAG:-r5_rn_pmc}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "/tmp/${TAG}_p$i" -o run -- \
    python3 "$R/bench.py" --steps 3 --warmup 2 $BENCH_ARGS > "$O/${TAG}_p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$O/${TAG}_p$i.log"; exit 1; }
done
python3 "$R/tools/pmc_by_dispatch.py" /tmp/${TAG}_p1 /tmp/${TAG}_p2 /tmp/${TAG}_p3 --top 45 > "$O/${TAG}.txt"
head -45 "$O/${TAG}.txt" | cut -c1-260
echo "[r5_rn_pmc] done"
