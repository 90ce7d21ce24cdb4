#!/bin/bash
# first bench + profile session
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python tools/gpu_check_synth.py > gpurun_out/s1_synth.log 2>&1 || { echo synth failed; tail gpurun_out/s1_synth.log; exit 1; }
timeout -k 10 300 python bench.py --workload C4 --scale 0.05 --steps 3 --warmup 1 --no-cpu-baseline --phases > gpurun_out/s1_small.log 2>&1 || { echo small failed; tail -30 gpurun_out/s1_small.log; exit 1; }
tail -3 gpurun_out/s1_small.log
timeout -k 10 600 python bench.py --workload C4 --steps 3 --warmup 1 --phases > gpurun_out/s1_c4.log 2>&1 || { echo c4 failed; tail -30 gpurun_out/s1_c4.log; exit 1; }
tail -30 gpurun_out/s1_c4.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof1 -o c4 -- python3 $R/bench.py --workload C4 --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/s1_prof.log 2>&1 || { echo prof failed; tail -30 $R/gpurun_out/s1_prof.log; exit 1; }
ls -R $R/gpurun_out/prof1 | head -20
