#!/bin/bash
# round-4 closing run: the whole -m gpu suite, the driver's default bench command, kernel stats of
# C4 / C3 / C2, the C4 PMC passes (traffic per kernel, tagged with $COMMIT)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/final_tests.log 2>&1 || { tail -40 gpurun_out/final_tests.log; exit 1; }
tail -2 gpurun_out/final_tests.log
timeout -k 10 900 python -u bench.py > gpurun_out/final_bench.json 2> gpurun_out/final_bench.err || { tail -30 gpurun_out/final_bench.err; exit 1; }
tail -1 gpurun_out/final_bench.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'], d['phase_ms'], d['roofline']['frac'], d.get('alt_paths',{}).get('hash_dictionary',{}).get('ms_per_step'), [ (k, v.get('ms_per_step'), v.get('device_ms_per_step')) for k, v in d.get('other_configs', {}).items()])"
