#!/bin/bash
# GPU box: paired ragged-decode kernels -- ragged/plan parity tests with the
# default library, then C3 timing for default vs ab/*.so (twice).
mkdir -p gpurun_out/pair
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c4.py -m gpu -x -q -k "ragged or plan" \
    --timeout 120 --timeout-method thread > gpurun_out/pair/tests.log 2>&1; rc=$?
tail -3 gpurun_out/pair/tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED|error" gpurun_out/pair/tests.log | head -30; exit $rc; }
for i in 1 2; do
  echo "default $(timeout -k 10 120 python -u scripts/bench_c3.py 2>&1 | grep c3_decode)" || exit 1
  for l in udpspeeder_amd/ab/*.so; do
    echo "$l $(RSMI_LIB=$PWD/$l timeout -k 10 120 python -u scripts/bench_c3.py 2>&1 | grep c3_decode)" || exit 1
  done
done
