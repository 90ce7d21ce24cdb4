#!/bin/bash
# weighted SUM CSR through the value-carrying bucket partition: its parity tests (new + the weighted
# goldens / fuzz / synthetic / C3 digest), then the C3 bench leg and its kernel stats
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -X faulthandler -m pytest -m gpu -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_diff.py -k "weighted_sum or csr_output or convert_format or float_duplicate or synthetic or fuzz_gpu" \
  tests/test_gpu_fullsize.py::test_c3_full_size_equals_oracle tests/test_gpu_golden.py \
  > gpurun_out/r4k_tests.log 2>&1 || { tail -80 gpurun_out/r4k_tests.log; exit 1; }
tail -3 gpurun_out/r4k_tests.log
timeout -k 10 300 python -u bench.py --workload C3 --steps 20 --warmup 3 > gpurun_out/r4k_c3.json 2> gpurun_out/r4k_c3.err || { tail -30 gpurun_out/r4k_c3.err; exit 1; }
cat gpurun_out/r4k_c3.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c3k -o run -- python3 $R/bench.py --workload C3 --steps 5 --warmup 1 > $R/gpurun_out/r4k_prof.log 2>&1 || { tail -30 $R/gpurun_out/r4k_prof.log; exit 1; }
f=$(ls $R/gpurun_out/prof_c3k/*/run_kernel_stats.csv 2>/dev/null | head -1); [ -n "$f" ] && head -25 "$f"
bash $R/tools/gpu_shard_prof.sh
exit 0
