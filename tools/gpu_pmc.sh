#!/bin/bash
# HBM traffic per kernel: separate rocprofv3 --pmc passes for FETCH_SIZE and WRITE_SIZE
# (MI355X_MICROARCH.md: TCC FETCH_SIZE and WRITE_SIZE do not fit one pass), kernel-trace only.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $R/gpurun_out/pmc/$C -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e --no-alt > $R/gpurun_out/pmc/$C.log 2>&1 || { tail -20 $R/gpurun_out/pmc/$C.log; exit 1; }
done
ls $R/gpurun_out/pmc/*/
