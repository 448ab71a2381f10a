#!/bin/bash
# per-kernel times (by grid) of the BN sweep: default geometry vs row-block cap 512 (grid-first listing)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d /tmp/p34a -o prof -- python3 $R/tools/bn_sweep.py --iters 10 > $R/gpurun_out/p34a.log 2>&1 || exit 1
DB=$(find /tmp/p34a -name "*.db" | head -1)
python3 -c "import sqlite3;c=sqlite3.connect('$DB');print([r[1] for r in c.execute('pragma table_info(kernels)')])" > $R/gpurun_out/p34_cols.txt
python3 $R/tools/kernel_stats.py $DB --grid --top 80 > $R/gpurun_out/p34a_grid.txt 2>&1
DCP_BN_RED_BLOCKS=512 timeout -k 10 200 rocprofv3 --kernel-trace -d /tmp/p34b -o prof -- python3 $R/tools/bn_sweep.py --iters 10 > $R/gpurun_out/p34b.log 2>&1 || exit 1
DB=$(find /tmp/p34b -name "*.db" | head -1)
python3 $R/tools/kernel_stats.py $DB --grid --top 80 > $R/gpurun_out/p34b_grid.txt 2>&1
echo done
