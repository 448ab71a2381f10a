set -eo pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 200 python3 -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread -k "conv3x3_c64_direct or conv_kxk" tests/test_gpu_conv1x1.py > gpurun_out/r2y_t1.log 2>&1 || { grep -v "^  File" gpurun_out/r2y_t1.log | tail -40; exit 1; }
tail -1 gpurun_out/r2y_t1.log
C1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_ANY"
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $C1 --kernel-trace --output-format csv -d $R/gpurun_out/r2y_d3b -o p -- python3 $R/tools/gemm_one.py --op conv3 --hw 56 --cin 64 --cout 64 --m 1605632 --iters 5 > $R/gpurun_out/r2y.log 2>&1) || { tail -20 gpurun_out/r2y.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/r2y_d3b --top 8 | cut -c1-120
timeout -k 10 300 python3 -u tools/gemm_bench.py --batch 512 --iters 10 --only3x3 > gpurun_out/r2y_g.log 2>&1
grep -h '56x56 c=64' gpurun_out/r2y_g.log | cut -c1-260
