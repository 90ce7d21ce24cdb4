#!/bin/bash
# the dictionary size estimate for S-poor inputs: dictionary / hash-tier parity tests, the goldens,
# then the chunked probe (hashed names) and the forced protocol line
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -X faulthandler -m pytest -m gpu -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_diff.py -k "dictionary or s_first or fuzz_gpu or synthetic or deterministic" tests/test_gpu_golden.py \
  tests/test_gpu_shard.py > gpurun_out/r4z_tests.log 2>&1 || { tail -60 gpurun_out/r4z_tests.log; exit 1; }
tail -2 gpurun_out/r4z_tests.log
timeout -k 10 600 python -u tools/chunked_probe2.py hashed > gpurun_out/chunked_probe2.log 2>&1 || { tail -30 gpurun_out/chunked_probe2.log; exit 1; }
grep total_s gpurun_out/chunked_probe2.log
timeout -k 10 600 python -u tools/chunked_probe.py > gpurun_out/chunked_probe.jsonl 2> gpurun_out/chunked_probe.err || { tail -30 gpurun_out/chunked_probe.err; exit 1; }
cat gpurun_out/chunked_probe.jsonl
