#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u tools/chunked_probe2.py hashed > gpurun_out/chunked_probe2.log 2>&1 || { tail -30 gpurun_out/chunked_probe2.log; exit 1; }
cat gpurun_out/chunked_probe2.log
