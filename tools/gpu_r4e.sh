#!/bin/bash
# round-4 parity (tools/gpu_r4a.sh), then experiment libraries A/B (tests + C4 phases) and the F1 stamps
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
bash tools/gpu_r4a.sh || exit 1
bash tools/gpu_r4b.sh "$@" || exit 1
bash tools/gpu_f1_stamps.sh f1st && python -c "import json; d=json.load(open('gpurun_out/f1_stamps.json')); print({k: v for k, v in d.items() if k != 'per_cu'})"
