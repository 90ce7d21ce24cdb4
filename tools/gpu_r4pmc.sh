#!/bin/bash
# C4 PMC passes (FETCH_SIZE, WRITE_SIZE, two SQ passes; each its own rocprofv3 run) -> per-kernel
# traffic summary (gpurun_out/pmc_c4.json, tagged $COMMIT) + kernel stats of C3 and C2
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -X faulthandler -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_gpu_shard.py > gpurun_out/pmc_shard_tests.log 2>&1 || { tail -40 gpurun_out/pmc_shard_tests.log; exit 1; }
tail -1 gpurun_out/pmc_shard_tests.log
bash tools/gpu_shard_x1.sh || exit 1
OUT_JSON=$R/gpurun_out/pmc_c4.json COMMIT=${COMMIT:-unknown} bash tools/gpu_counters.sh ctr_c4f "g2n::" || exit 1
cd /tmp && export TMPDIR=/tmp
for w in C3 C2; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${w}f -o run -- python3 $R/bench.py --workload $w --steps 5 --warmup 1 --no-e2e --no-alt --no-cpu-baseline > $R/gpurun_out/prof_${w}f.log 2>&1 || { tail -30 $R/gpurun_out/prof_${w}f.log; exit 1; }
python3 $R/tools/rocpd_stats.py $R/gpurun_out/prof_${w}f/run_results.db 12
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_C4f -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-e2e --no-alt --no-cpu-baseline > $R/gpurun_out/prof_C4f.log 2>&1 || { tail -30 $R/gpurun_out/prof_C4f.log; exit 1; }
python3 $R/tools/rocpd_stats.py $R/gpurun_out/prof_C4f/run_results.db 12
