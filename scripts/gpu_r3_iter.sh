#!/bin/bash
# GPU box, round-3 iteration: C3 class-kernel A/B (gpu_c3_ab.sh), the fused
# cook tests, then bench_frame.py in plain / fused / unfused cook modes.
mkdir -p gpurun_out/c3ab gpurun_out/fc
bash scripts/gpu_c3_ab.sh > gpurun_out/c3ab/ab.log 2>&1; rc=$?
grep -E "passed|failed|rror|c3_decode|W=|per group|entry->" gpurun_out/c3ab/ab.log | cut -c1-200
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_cook.py tests/test_fec_frame.py -m gpu -x -q \
    -k "out_of_place or cooked" --timeout 120 --timeout-method thread > gpurun_out/fc/tests.log 2>&1; rc=$?
tail -3 gpurun_out/fc/tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/fc/tests.log | head -20; exit $rc; }
for m in "" sep dev host; do
  timeout -k 10 180 python -u scripts/bench_frame.py --cpu-sample 0 ${m:+--cook $m} 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/fc/bench_frame.jsonl || exit 1
done
