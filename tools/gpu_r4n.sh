#!/bin/bash
# kernel stats after the pair words: C4 (default bench) and C3
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c4n -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-e2e --no-alt --no-cpu-baseline > $R/gpurun_out/r4n_c4.log 2>&1 || { tail -30 $R/gpurun_out/r4n_c4.log; exit 1; }
python3 $R/tools/rocpd_stats.py $R/gpurun_out/prof_c4n/run_results.db 22
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c3n -o run -- python3 $R/bench.py --workload C3 --steps 5 --warmup 1 --no-e2e --no-alt --no-cpu-baseline > $R/gpurun_out/r4n_c3.log 2>&1 || { tail -30 $R/gpurun_out/r4n_c3.log; exit 1; }
python3 $R/tools/rocpd_stats.py $R/gpurun_out/prof_c3n/run_results.db 16
