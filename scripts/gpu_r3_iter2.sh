#!/bin/bash
# GPU box: the FEC framing / cook / tunnel / ragged GPU tests, then
# bench_frame.py in plain / unfused / fused-device / fused-host cook modes.
mkdir -p gpurun_out/fc
timeout -k 10 400 python -u -m pytest tests/test_gpu_cook.py tests/test_fec_frame.py tests/test_tunnel.py \
    tests/test_gpu_parity.py -m gpu -x -q -k "cook or frame or tunnel or ragged or plan" \
    --timeout 120 --timeout-method thread > gpurun_out/fc/tests.log 2>&1; rc=$?
tail -3 gpurun_out/fc/tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/fc/tests.log | head -20; exit $rc; }
rm -f gpurun_out/fc/bench_frame.jsonl
for m in "" sep dev host; do
  timeout -k 10 180 python -u scripts/bench_frame.py --cpu-sample 0 ${m:+--cook $m} 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/fc/bench_frame.jsonl | cut -c1-150 || exit 1
done
for i in 1 2; do timeout -k 10 120 python -u scripts/bench_c3.py 2>&1 | grep c3_ || exit 1; done
