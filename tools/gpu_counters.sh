#!/bin/bash
# Counters for the kernels matching $2 on a 1-step C4 bench: FETCH_SIZE, WRITE_SIZE (own passes,
# MI355X_MICROARCH.md) and two SQ passes; each rocprofv3 pass under its own kill-limit.
# usage: gpu_counters.sh <out name> <kernel regex>
set -o pipefail
R=$GRAFT_REPO_ROOT; NAME=${1:-ctr}; RE=${2:-k_}
mkdir -p $R/gpurun_out/$NAME
cd /tmp && export TMPDIR=/tmp
i=0
for P in "FETCH_SIZE" "WRITE_SIZE" \
         "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
         "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $P --kernel-trace --kernel-include-regex "$RE" --output-format csv -d $R/gpurun_out/$NAME/p$i -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e --no-alt ${BENCH_ARGS:-} > $R/gpurun_out/$NAME/p$i.log 2>&1 || { tail -20 $R/gpurun_out/$NAME/p$i.log; exit 1; }
done
python3 $R/tools/counter_table.py $R/gpurun_out/$NAME ${OUT_JSON:-} ${COMMIT:-}
