#!/bin/bash
# K2 A/B: parity tests of the tile-local parse, then C4 bench phases for base vs experiment libs, then stamps
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_diff.py tests/test_gpu_golden.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -k "tile_local or decimal or c4_full or golden or fuzz or maxsym or csr_output or synthetic or deterministic or float_duplicate" > gpurun_out/k2_tests.log 2>&1 || { tail -30 gpurun_out/k2_tests.log; exit 1; }
tail -2 gpurun_out/k2_tests.log
bash tools/gpu_exp.sh "$@" || exit 1
bash tools/gpu_k2_stamps.sh stamps || exit 1
