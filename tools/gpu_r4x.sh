#!/bin/bash
# chunked single-GPU build vs one piece on a quarter-C4 file on disk
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u tools/chunked_probe.py > gpurun_out/chunked_probe.jsonl 2> gpurun_out/chunked_probe.err || { tail -30 gpurun_out/chunked_probe.err; exit 1; }
cat gpurun_out/chunked_probe.jsonl
