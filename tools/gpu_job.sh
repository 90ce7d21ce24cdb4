#!/bin/bash
# One gpurun job made of steps, run in order, each under its own time limit; the job stops at the
# first failing step and prints the tail of its log.  Replaces the one-off launch scripts.
#
# usage (on the box):  bash tools/gpu_job.sh <tag> <step> [<step> ...]
#   tests:<pytest args>     python -m pytest -m gpu <args>            -> gpurun_out/<tag>_s<i>.log
#   bench:<bench.py args>   python bench.py <args>                    -> gpurun_out/<tag>_s<i>.json (+ .err)
#   prof:<bench.py args>    rocprofv3 --kernel-trace --stats of bench.py <args>; top kernels printed,
#                           database under gpurun_out/<tag>_s<i>/
#   pmc:<bench.py args>     tools/gpu_counters.sh passes on bench.py <args> -> gpurun_out/<tag>_pmc.json
#   py:<script + args>      python -u <script + args>                 -> gpurun_out/<tag>_s<i>.log
#   ab:<libs> <bench args>  bench.py per library (main, or exp_<x>.so from tools/exp_build.sh), twice
# step arguments are word-split by the shell (eval): quote inside them, e.g. "tests:f.py -k 'a or b'".
# limits (seconds): T_TESTS (900), T_BENCH (600), T_PROF (300), T_PY (600); COMMIT tags the pmc summary.
# example:
#   gpurun --timeout 1200 -- 'bash tools/gpu_job.sh r5a "tests:tests/test_gpu_diff.py -k int64" "bench:--steps 5"'
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${1:?tag}; shift
i=0
for step in "$@"; do
  i=$((i + 1))
  kind=${step%%:*}; args=${step#*:}
  base=gpurun_out/${TAG}_s$i
  echo "== step $i: $kind $args"
  case $kind in
    tests)
      eval "timeout -k 10 ${T_TESTS:-900} python -u -X faulthandler -m pytest -m gpu -x -q --timeout 300 \
        --timeout-method thread $args" > $base.log 2>&1 || { tail -60 $base.log; exit 1; }
      tail -2 $base.log ;;
    bench)
      timeout -k 10 ${T_BENCH:-600} python -u bench.py $args > $base.json 2> $base.err || { tail -40 $base.err; exit 1; }
      tail -1 $base.json | cut -c1-3000 ;;
    prof)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 ${T_PROF:-300} rocprofv3 --kernel-trace --stats \
        -d "$R/$base" -o run -- python3 "$R/bench.py" $args > "$R/$base.log" 2>&1) || { tail -30 $base.log; exit 1; }
      python3 tools/rocpd_stats.py $base/run_results.db 16 | tee $base.txt ;;
    pmc)
      OUT_JSON=$R/gpurun_out/${TAG}_pmc.json COMMIT=${COMMIT:-unknown} BENCH_ARGS="$args" \
        bash tools/gpu_counters.sh ${TAG}_ctr "g2n::" || exit 1 ;;
    ab)  # ab:<lib,lib,...> <bench.py args>: each library in turn (main = libg2n.so, x = exp_x.so; lib@F runs
         # it with G2N_TEST_FLAGS=F), twice
      libs=${args%% *}; bargs=${args#* }
      for rep in 1 2; do for l in ${libs//,/ }; do
        ln=${l%@*}; fl=0; [ "$ln" != "$l" ] && fl=${l#*@}
        lp=$R/gfa2network_amd/_lib/$([ "$ln" = main ] && echo libg2n.so || echo exp_$ln.so)
        G2N_TEST_FLAGS=$fl G2N_LIB=$lp timeout -k 10 ${T_BENCH:-600} python -u bench.py $bargs > ${base}_${l}_$rep.json 2>> $base.err ||
          { tail -20 $base.err; exit 1; }
        python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d.get('device_ms_per_step'), d.get('phase_ms'))" ${base}_${l}_$rep.json $l
      done; done ;;
    py)
      timeout -k 10 ${T_PY:-600} python -u $args > $base.log 2>&1 || { tail -40 $base.log; exit 1; }
      tail -5 $base.log ;;
    *) echo "unknown step kind: $kind"; exit 2 ;;
  esac
done
