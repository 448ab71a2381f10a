#!/bin/bash
# SQ counters after the GEMM core fixes (NOTES §14): layer-4 1x1 fwd, 14x14 c=256 3x3 implicit GEMM, 1x1 wgrad
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
C1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU"
timeout -s KILL 90 rocprofv3 --pmc $C1 --kernel-trace --output-format csv -d /tmp/p77a -o p -- python3 $R/tools/gemm_one.py --op fwd > $R/gpurun_out/g77a.log 2>&1 || exit 1
python3 $R/tools/pmc_summary.py /tmp/p77a --top 40 > $R/gpurun_out/pmc77a.txt 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc $C1 --kernel-trace --output-format csv -d /tmp/p77b -o p -- python3 $R/tools/gemm_one.py --op conv3 --m 50176 --cin 256 --cout 256 --hw 14 > $R/gpurun_out/g77b.log 2>&1 || exit 1
python3 $R/tools/pmc_summary.py /tmp/p77b --top 40 > $R/gpurun_out/pmc77b.txt 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc $C1 --kernel-trace --output-format csv -d /tmp/p77c -o p -- python3 $R/tools/gemm_one.py --op wgrad --m 50176 --cin 1024 --cout 256 > $R/gpurun_out/g77c.log 2>&1 || exit 1
python3 $R/tools/pmc_summary.py /tmp/p77c --top 40 > $R/gpurun_out/pmc77c.txt 2>&1 || exit 1
echo done
