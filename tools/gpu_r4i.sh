#!/bin/bash
# round-4 profiles at HEAD: rocprofv3 kernel stats of the C4 / C2 / C3 benches and the C4 PMC passes
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
bash tools/gpu_prof.sh c4 || exit 1
BENCH_ARGS="--workload C2" bash tools/gpu_prof.sh c2 || exit 1
BENCH_ARGS="--workload C3" bash tools/gpu_prof.sh c3 || exit 1
OUT_JSON=$R/gpurun_out/pmc_c4.json COMMIT=f436ec4 bash tools/gpu_counters.sh ctr "k_" || exit 1
