#!/bin/bash
# GPU box, one build-measure iteration: selected GPU tests (-k expression in $1),
# then optional extra commands ($2...) each under its own time limit.
mkdir -p gpurun_out/iter
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "$1" > gpurun_out/iter/tests.log 2>&1; rc=$?
tail -5 gpurun_out/iter/tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/iter/tests.log | head -30; exit $rc; }
shift
i=0
for cmd in "$@"; do
  i=$((i+1))
  timeout -k 10 300 bash -c "$cmd" > gpurun_out/iter/x$i.log 2>&1; rc=$?
  tail -40 gpurun_out/iter/x$i.log
  [ $rc -eq 0 ] || exit $rc
done
