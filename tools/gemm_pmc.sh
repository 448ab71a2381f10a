#!/bin/bash
# PMC passes (one counter group per run, kernel trace only) over
# ${PROBE:-tools/gemm_pmc_probe.py}, then tools/pmc_mfma.py -> gpurun_out/${PTAG:-gemm_pmc}/summary.txt
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/${PTAG:-gemm_pmc}
mkdir -p "$O"
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_SALU" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE GRBM_COUNT" \
           ${EXTRA_GROUP:+"$EXTRA_GROUP"}; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "/tmp/gemm_pmc_p$i" -o run -- \
    python3 "$R/${PROBE:-tools/gemm_pmc_probe.py}" > "$O/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$O/p$i.log"; exit 1; }
done
python3 "$R/tools/pmc_mfma.py" /tmp/gemm_pmc_p1 /tmp/gemm_pmc_p2 > "$O/summary.txt" && cat "$O/summary.txt"
python3 "$R/tools/pmc_by_dispatch.py" /tmp/gemm_pmc_p* --top 20 > "$O/by_dispatch.txt" && cut -c1-400 "$O/by_dispatch.txt"
echo "[gemm_pmc] done"
