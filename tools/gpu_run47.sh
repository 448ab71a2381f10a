#!/bin/bash
# SQ counters of gemm_nt after the SALU/swizzle fix (layer-4 1x1 shape) and of the gathered 3x3 fwd
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU --kernel-trace --output-format csv -d /tmp/p47 -o p -- python3 $R/tools/gemm_one.py --op fwd > $R/gpurun_out/g47.log 2>&1 || exit 1
python3 $R/tools/pmc_summary.py /tmp/p47 --top 40 > $R/gpurun_out/pmc47.txt 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d /tmp/p47b -o p -- python3 $R/tools/gemm_one.py --op fwd > $R/gpurun_out/g47b.log 2>&1 || exit 1
python3 $R/tools/pmc_summary.py /tmp/p47b --top 40 > $R/gpurun_out/pmc47b.txt 2>&1 || exit 1
echo done
