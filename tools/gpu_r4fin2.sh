#!/bin/bash
# F1 at 8 waves by default: the partition / finish parity tests, full-size digests, the C4 bench
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -m gpu -x -q --timeout 400 --timeout-method thread \
  tests/test_gpu_diff.py -k "maxsym or csr_output or synthetic or int64_index or fuzz_gpu or convert_format or failed_build or weighted_sum" \
  tests/test_gpu_fullsize.py tests/test_gpu_golden.py tests/test_gpu_shard.py > gpurun_out/r4fin2_tests.log 2>&1 || { tail -40 gpurun_out/r4fin2_tests.log; exit 1; }
tail -1 gpurun_out/r4fin2_tests.log
timeout -k 10 900 python -u bench.py > gpurun_out/final_bench2.json 2> gpurun_out/final_bench2.err || { tail -30 gpurun_out/final_bench2.err; exit 1; }
tail -1 gpurun_out/final_bench2.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value'], d['phase_ms'], d['roofline']['frac'], d.get('alt_paths',{}).get('hash_dictionary',{}).get('ms_per_step'), [ (k, v.get('ms_per_step'), v.get('device_ms_per_step')) for k, v in d.get('other_configs', {}).items()])"
