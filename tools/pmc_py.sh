#!/bin/bash
# Two PMC passes (issue / wait breakdown, memory-pipe pressure) over a python
# script: bash tools/pmc_py.sh TAG SCRIPT [ARGS...]   (csv under gpurun_out/TAG_{1,2}/)
set -eo pipefail
TAG=${1:?tag}; SCRIPT=${2:?script}; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd /tmp
i=0
for ctr in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i + 1))
  timeout -s KILL 180 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d "$R/gpurun_out/${TAG}_$i" -o pmc -- \
    python3 "$R/$SCRIPT" "$@" > "$R/gpurun_out/${TAG}_$i.log" 2>&1
done
echo "[pmc_py] $TAG done"
