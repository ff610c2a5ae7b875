#!/bin/bash
# GPU box: cook parity tests (default library), bench_cook.py for the default
# library and every non-trace ab/*.so (twice), then the k_cook phase trace.
mkdir -p gpurun_out/ck
timeout -k 10 300 python -u -m pytest tests/test_gpu_cook.py tests/test_fec_frame.py -m gpu -x -q -k "cook or cooked" \
    --timeout 120 --timeout-method thread > gpurun_out/ck/tests.log 2>&1; rc=$?
tail -1 gpurun_out/ck/tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/ck/tests.log | head; exit $rc; }
for i in 1 2; do
  echo "default $(timeout -k 10 120 python -u scripts/bench_cook.py --cpu-sample 0 2>&1 | grep -v amdgpu.ids | tail -1 | cut -c1-220)" || exit 1
  for l in udpspeeder_amd/ab/*.so; do case $l in *trace*) continue;; esac
    echo "$l $(RSMI_LIB=$PWD/$l timeout -k 10 120 python -u scripts/bench_cook.py --cpu-sample 0 2>&1 | grep -v amdgpu.ids | tail -1 | cut -c1-220)" || exit 1
  done
done
RSMI_LIB=$PWD/udpspeeder_amd/ab/librsmi_ctrace.so timeout -k 10 200 python -u scripts/cook_trace.py 2>&1 | grep -v amdgpu.ids
