#!/bin/bash
# wgrad GEMM: kernel split (MFMA kernel vs slab reduce) and SQ counters, layer-4 and layer-3 shapes
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
for sh in "12544 2048 512" "50176 1024 256" "200704 128 512"; do
set -- $sh
tag=w$1
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/p41_$tag -o p -- python3 $R/tools/gemm_one.py --op wgrad --m $1 --cin $2 --cout $3 > $R/gpurun_out/g41_$tag.log 2>&1 || exit 1
find /tmp/p41_$tag -name "*kernel_stats.csv" -exec cp {} $R/gpurun_out/ks41_$tag.csv \;
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU --kernel-trace --output-format csv -d /tmp/p41p_$tag -o p -- python3 $R/tools/gemm_one.py --op wgrad --m $1 --cin $2 --cout $3 > $R/gpurun_out/g41p_$tag.log 2>&1 || exit 1
python3 $R/tools/pmc_summary.py /tmp/p41p_$tag --top 12 > $R/gpurun_out/pmc41_$tag.txt 2>&1 || exit 1
done
echo done
