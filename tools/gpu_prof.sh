#!/bin/bash
# rocprofv3 kernel stats of a short C4 bench (or $BENCH_ARGS); prints the top kernels
set -o pipefail
R=$GRAFT_REPO_ROOT; NAME=${1:-prof}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$NAME -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-alt ${BENCH_ARGS:-} > $R/gpurun_out/$NAME.log 2>&1 || { tail -30 $R/gpurun_out/$NAME.log; exit 1; }
python3 $R/tools/prof_summary.py $R/gpurun_out/$NAME/run_kernel_stats.csv 3
