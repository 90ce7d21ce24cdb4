#!/bin/bash
# One GPU session: the GPU test suite, the C4 bench (no e2e), rocprof kernel stats, and the PMC /
# SQ counter passes whose summary bench.py reads (profiles/r02/pmc_c4.json, tagged with $COMMIT).
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 --no-e2e > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
bash tools/gpu_prof.sh prof_c4 && OUT_JSON=$R/gpurun_out/pmc_c4.json bash tools/gpu_counters.sh ctr_c4 "g2n::"
