#!/bin/bash
# K2 variants A/B (tests + bench phases) and the K2 stamps, then the round-4 parity (tools/gpu_r4a.sh)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
bash tools/gpu_r4b.sh "$@" || exit 1
bash tools/gpu_k2_stamps.sh stamps && python -c "import json; d=json.load(open('gpurun_out/k2_stamps.json')); print({k: v for k, v in d.items() if k != 'per_cu'})"
bash tools/gpu_r4a.sh
