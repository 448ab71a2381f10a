#!/bin/bash
# Two PMC passes (gfx950 slot limits: ≤ 8 SQ counters each) over one GEMM
# shape of tools/gemm_one.py, csv out under gpurun_out/TAG_{1,2}/.
#   bash tools/pmc_gemm.sh TAG "GEMM_ONE_ARGS"
set -eo pipefail
TAG=${1:?tag}; ARGS=${2:?args}
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd /tmp
i=0
for ctr in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d "$R/gpurun_out/${TAG}_$i" -o pmc -- \
    python3 "$R/tools/gemm_one.py" $ARGS > "$R/gpurun_out/${TAG}_$i.log" 2>&1
done
echo "[pmc_gemm] $TAG done"
