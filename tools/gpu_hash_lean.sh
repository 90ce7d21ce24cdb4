#!/bin/bash
# the lean S-first hash pass: parity tests, then the C4 bench line with its hash-dictionary leg
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_hash_lean.py tests/test_gpu_diff.py -m gpu -x -q --timeout 300 --timeout-method thread -k "hash_lean or hash_dictionary or s_first or general or tile_local or decimal" > gpurun_out/hl_tests.log 2>&1 || { tail -40 gpurun_out/hl_tests.log; exit 1; }
tail -2 gpurun_out/hl_tests.log
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/hl_bench.json 2> gpurun_out/hl_bench.err || { tail -30 gpurun_out/hl_bench.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/hl_bench.json').read().strip().splitlines()[-1])
print(d['ms_per_step'], d['phase_ms']); print(json.dumps(d.get('alt_paths', {}).get('hash_dictionary')))
print(json.dumps(d.get('other_configs')))"
