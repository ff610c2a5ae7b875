#!/bin/bash
# GPU box: cook GPU tests on the default library, then scripts/bench_cook.py
# (no CPU baseline) for the default library and every udpspeeder_amd/ab/*.so, twice.
timeout -k 10 300 python -u -m pytest tests/test_gpu_cook.py -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/cook_t.log 2>&1 || { tail -30 gpurun_out/cook_t.log; exit 1; }
tail -1 gpurun_out/cook_t.log
for i in 1 2; do
  for lib in default udpspeeder_amd/ab/*.so; do
    if [ $lib != default ]; then export RSMI_LIB=$PWD/$lib; else unset RSMI_LIB; fi
    echo -n "$(basename $lib): "
    timeout -k 10 200 python -u scripts/bench_cook.py --cpu-sample 0 2>/dev/null | python3 -c "
import json,sys
d=json.loads([l for l in sys.stdin if l.startswith('{')][-1])
print({k: v for k, v in d.items() if 'ms' in k or 'frac' in k})" || exit 1
  done
done
