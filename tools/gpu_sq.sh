#!/bin/bash
# SQ (shader) counters for the named kernels: two --pmc passes, kernel-trace only.
# usage: gpu_sq.sh <out name> <kernel regex>
set -o pipefail
R=$GRAFT_REPO_ROOT
NAME=${1:-sq}
RE=${2:-k_tile_parse|k_insert_round|k_row_max}
mkdir -p $R/gpurun_out/$NAME
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > $R/gpurun_out/$NAME/counters.txt 2>&1 || true
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -k 10 600 rocprofv3 --pmc $P --kernel-trace --kernel-include-regex "$RE" --output-format csv -d $R/gpurun_out/$NAME/p$i -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e --no-alt > $R/gpurun_out/$NAME/p$i.log 2>&1 || { tail -20 $R/gpurun_out/$NAME/p$i.log; exit 1; }
done
ls $R/gpurun_out/$NAME/*/
