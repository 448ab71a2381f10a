#!/bin/bash
# PMC passes over the 64-channel direct 3x3 forward (tools/gemm_one.py conv3),
# one rocprofv3 run per counter group (gfx950 slot limits), csv out.
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd /tmp
i=0
for ctr in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d "$R/gpurun_out/pmc_c3_$i" -o pmc -- \
    python3 "$R/tools/gemm_one.py" --m 1605632 --cin 64 --cout 64 --op conv3 --hw 56 --iters 5 > "$R/gpurun_out/pmc_c3_$i.log" 2>&1
done
echo done
