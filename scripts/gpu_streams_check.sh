#!/bin/bash
# GPU box: the two-stream scenario (fused and two-kernel decode), then the full
# GPU test suite twice; one summary line each.
timeout -k 10 300 python -u scripts/dbg_streams.py 64 two both | grep -v ": ok$"; echo "fused done"
DBG_NOFUSED=1 timeout -k 10 300 python -u scripts/dbg_streams.py 48 two both | grep -v ": ok$"; echo "nofused done"
for rep in 1 2; do
  timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
      > gpurun_out/suite_$rep.log 2>&1
  echo "suite $rep: $(tail -1 gpurun_out/suite_$rep.log)"
done
