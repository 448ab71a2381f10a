#!/bin/bash
# Extra PMC passes (memory-pipe pressure) over one tools/gemm_one.py shape:
#   bash tools/pmc_gemm2.sh TAG "GEMM_ONE_ARGS"
set -eo pipefail
TAG=${1:?tag}; ARGS=${2:?args}
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd /tmp
i=0
for ctr in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES" \
           "SQ_INSTS_VMEM SQ_INST_LEVEL_VMEM SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_INST_LEVEL_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d "$R/gpurun_out/${TAG}_$i" -o pmc -- \
    python3 "$R/tools/gemm_one.py" $ARGS > "$R/gpurun_out/${TAG}_$i.log" 2>&1
done
echo "[pmc_gemm2] $TAG done"
