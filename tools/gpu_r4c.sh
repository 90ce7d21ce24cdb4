#!/bin/bash
# K2 A/B first (tools/gpu_r4b.sh), then the round-4 parity tests + C5 line (tools/gpu_r4a.sh)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
bash tools/gpu_r4b.sh "$@" || exit 1
bash tools/gpu_r4a.sh
