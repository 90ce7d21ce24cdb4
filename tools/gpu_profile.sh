#!/bin/bash
# rocprofv3 kernel-trace + stats of the bench (C4), summary to gpurun_out/$1
set -o pipefail
R=$GRAFT_REPO_ROOT
NAME=${1:-prof}
shift
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$NAME -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-alt "$@" > $R/gpurun_out/$NAME.log 2>&1 || { tail -30 $R/gpurun_out/$NAME.log; exit 1; }
tail -1 $R/gpurun_out/$NAME.log
