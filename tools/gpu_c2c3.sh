#!/bin/bash
# C2 / C3 device-resident bench lines + rocprofv3 kernel stats, and the GPU tests added this round.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_cli.py::test_single_gpu_path_without_torch tests/test_verbose_golden.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_misc.log 2>&1 || { tail -30 gpurun_out/t_misc.log; exit 1; }
tail -2 gpurun_out/t_misc.log
for W in C3 C2; do
  timeout -k 10 300 python bench.py --workload $W --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > gpurun_out/bench_$W.json 2> gpurun_out/bench_$W.err || { tail -30 gpurun_out/bench_$W.err; exit 1; }
  BENCH_ARGS="--workload $W" bash tools/gpu_prof.sh prof_$W || exit 1
done
