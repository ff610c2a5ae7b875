#!/bin/bash
# GPU box: the whole -m gpu suite once (one process), then smoke(); logs in gpurun_out/.
# The pytest process's wall time is logged next to pytest's own time, so a
# slow or hung interpreter exit shows as the difference.
mkdir -p gpurun_out
s=$(date +%s)
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    --durations=12 > gpurun_out/suite.log 2>&1; rc=$?
e=$(date +%s)
echo "pytest rc=$rc process_wall_s=$((e - s))" | tee -a gpurun_out/suite.log
tail -4 gpurun_out/suite.log
[ $rc -eq 0 ] || exit $rc
s=$(date +%s)
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc wall_s=$(( $(date +%s) - s ))" | tee -a gpurun_out/smoke.log
grep -v amdgpu.ids gpurun_out/smoke.log | tail -3
exit $rc
