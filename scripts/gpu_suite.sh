#!/bin/bash
# GPU box: the whole -m gpu suite once (one process), then smoke(); logs in gpurun_out/.
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/suite.log 2>&1; rc=$?
tail -3 gpurun_out/suite.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" 2>&1 | grep -v amdgpu.ids
