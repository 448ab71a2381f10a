#!/bin/bash
# Two rocprofv3 PMC passes (tools/pmc_gemm.sh counter groups) over each
# tools/gemm_one.py case of CASES ('|'-separated arg strings), then the
# tools/pmc_mfma.py summary of each -> gpurun_out/${TAG}_summary.txt
set -o pipefail
TAG=${TAG:-r6pmc}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
export TMPDIR=/tmp
IFS='|' read -ra CS <<< "$CASES"
n=0
for args in "${CS[@]}"; do
  n=$((n + 1))
  i=0
  for ctr in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
             "SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i + 1))
    (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d "$O/${TAG}_c${n}_$i" -o pmc -- \
      python3 "$R/tools/gemm_one.py" $args > "$O/${TAG}_c${n}_$i.log" 2>&1) || { echo "[r6_pmc] case $n pass $i failed"; tail -5 "$O/${TAG}_c${n}_$i.log"; exit 1; }
  done
  { echo "== case $n: $args"; python3 "$R/tools/pmc_mfma.py" "$O/${TAG}_c${n}_1" "$O/${TAG}_c${n}_2"; } >> "$O/${TAG}_summary.txt"
done
cat "$O/${TAG}_summary.txt"
