#!/bin/bash
# GPU box runner (round 4): bash scripts/gpu_run.sh OUT STEP [STEP ...]
# Steps run in order, each under its own time limit; the first failure ends
# the call.  Output under gpurun_out/OUT/.
#   suite        the whole -m gpu suite in one process (suite.log)
#   tests:EXPR   pytest -m gpu -k EXPR (tests.log)
#   smoke        __graft_entry__.smoke() (smoke.log)
#   bench        the driver's bench command (bench.json)
#   prof         the same bench command under rocprofv3 --kernel-trace --stats,
#                then the trace split by grid size (kernel_by_grid.txt)
#   c3           scripts/bench_c3.py (c3.json)
#   py:SCRIPT    python SCRIPT (SCRIPT.log), e.g. py:scripts/bench_cook.py
#   kt:SCRIPT[,ARG...]  SCRIPT under rocprofv3 --kernel-trace --memory-copy-trace
#                --stats (kt_<script>/: kernel and copy stats, script log)
set -o pipefail
R=$PWD
O=$R/gpurun_out/$1
shift
mkdir -p $O
for step in "$@"; do
  echo "== $step $(date +%T)"
  case $step in
    suite)
      s=$(date +%s)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
          --durations=12 > $O/suite.log 2>&1; rc=$?
      echo "pytest rc=$rc process_wall_s=$(( $(date +%s) - s ))" | tee -a $O/suite.log
      tail -4 $O/suite.log
      [ $rc -eq 0 ] || exit $rc ;;
    tests:*)
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
          -k "${step#tests:}" > $O/tests.log 2>&1; rc=$?
      tail -5 $O/tests.log
      [ $rc -eq 0 ] || exit $rc ;;
    smoke)
      timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
      grep -v amdgpu.ids $O/smoke.log | tail -2 ;;
    bench)
      timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
      cut -c1-600 $O/bench.json ;;
    prof)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv \
          -d $O/prof -o run -- python3 $R/bench.py --steps 20 --warmup 5 > $O/prof.log 2>&1) || { tail $O/prof.log; exit 1; }
      python scripts/kstats_grid.py $O/prof/run_kernel_trace.csv > $O/kernel_by_grid.txt
      head -30 $O/kernel_by_grid.txt
      rm -f $O/prof/run_kernel_trace.csv ;;
    c3)
      timeout -k 10 300 python -u scripts/bench_c3.py > $O/c3.json 2> $O/c3.err || { tail $O/c3.err; exit 1; }
      cat $O/c3.json ;;
    py:*)
      f=${step#py:}
      timeout -k 10 400 python -u $f > $O/$(basename $f).log 2>&1 || { tail $O/$(basename $f).log; exit 1; }
      tail -20 $O/$(basename $f).log ;;
    kt:*)
      IFS=',' read -ra A <<< "${step#kt:}"
      d=$O/kt_$(basename ${A[0]} .py)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats \
          --output-format csv -d $d -o run -- python3 $R/${A[0]} "${A[@]:1}" > $d.log 2>&1) || { tail $d.log; exit 1; }
      python scripts/kstats.py $d/run_kernel_stats.csv | head -25
      python scripts/ktimeline.py $d/run_kernel_trace.csv 40 $d/run_memory_copy_trace.csv > $d/timeline.txt
      head -3 $d/run_memory_copy_trace.csv > $d/copy_trace_head.csv
      rm -f $d/run_kernel_trace.csv $d/run_memory_copy_trace.csv
      tail -5 $d.log ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
