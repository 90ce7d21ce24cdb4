#!/bin/bash
# the GPU test suite in one process, with its own limit
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 ${1:-900} python -m pytest tests -m gpu -q -x ${@:2} > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -40 gpurun_out/gpu_tests.log
exit $rc
