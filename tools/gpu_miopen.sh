#!/bin/bash
# MIOpen solver selection experiments for the ResNet-50 step:
#  A: default find mode (baseline)      B: MIOPEN_FIND_MODE=NORMAL (full find)
#  C: NORMAL + FIND_ENFORCE=SEARCH (tune tunable solvers; perf db -> gpurun_out/miopen_db)
#  D: NORMAL with the tuned db
set -o pipefail
mkdir -p gpurun_out/miopen_db
export TMPDIR=/tmp
S=gpurun_out/miopen_summary.jsonl
b() { tag=$1; shift; timeout -k 10 ${T:-400} python bench.py --steps 20 --warmup 5 "$@" > gpurun_out/mi_$tag.json 2> gpurun_out/mi_$tag.err; rc=$?; echo "{\"tag\": \"$tag\", \"rc\": $rc}" >> $S; tail -1 gpurun_out/mi_$tag.json >> $S; return $rc; }
b A_default
MIOPEN_FIND_MODE=1 b B_normal
MIOPEN_USER_DB_PATH=$PWD/gpurun_out/miopen_db MIOPEN_FIND_MODE=1 MIOPEN_FIND_ENFORCE=3 MIOPEN_LOG_LEVEL=4 T=1000 b C_search
MIOPEN_USER_DB_PATH=$PWD/gpurun_out/miopen_db MIOPEN_FIND_MODE=1 b D_tuned
ls -la gpurun_out/miopen_db >> $S
echo done
