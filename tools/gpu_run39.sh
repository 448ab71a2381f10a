#!/bin/bash
# PMC counters of gemm_nt on the layer-4 shape (M=12544, 2048->512), plain and with the BN prologue
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 120 python3 $R/tools/gemm_one.py --op fwd --iters 2 > $R/gpurun_out/g39_smoke.log 2>&1 || exit 1
for op in fwd fwd_pro; do
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS --kernel-trace --output-format csv -d /tmp/p39_$op -o p -- python3 $R/tools/gemm_one.py --op $op > $R/gpurun_out/g39_$op.log 2>&1 || exit 1
python3 $R/tools/pmc_summary.py /tmp/p39_$op --top 20 > $R/gpurun_out/pmc39_$op.txt 2>&1 || exit 1
done
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d /tmp/p39_i -o p -- python3 $R/tools/gemm_one.py --op fwd > $R/gpurun_out/g39_i.log 2>&1 || exit 1
python3 $R/tools/pmc_summary.py /tmp/p39_i --top 20 > $R/gpurun_out/pmc39_i.txt 2>&1
echo done
