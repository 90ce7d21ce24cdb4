#!/bin/bash
# kernel stats of the forced general protocol at N = 1 (C4, hashed names): where the owner dedup goes
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_shx1 -o run -- python3 $R/bench.py --shard --workload C4 --names hashed --force-protocol --steps 2 --warmup 1 > $R/gpurun_out/shx1_prof.log 2>&1 || { tail -30 $R/gpurun_out/shx1_prof.log; exit 1; }
f=$(ls $R/gpurun_out/prof_shx1/*/run_kernel_stats.csv | head -1); head -40 "$f"
