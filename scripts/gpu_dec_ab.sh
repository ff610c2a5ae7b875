#!/bin/bash
# GPU box: RS parity tests on the default build, then the RS(20,10) encode/decode
# A/B over the default library and every udpspeeder_amd/ab/*.so.
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_fec_decode.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > gpurun_out/dec_tests.log 2>&1 || { tail -30 gpurun_out/dec_tests.log; exit 1; }
tail -1 gpurun_out/dec_tests.log
for i in 1 2; do
  timeout -k 10 120 python -u scripts/ab_encode.py 2>&1 | grep -v amdgpu.ids || exit 1
  for lib in udpspeeder_amd/ab/*.so; do
    RSMI_LIB=$PWD/$lib timeout -k 10 120 python -u scripts/ab_encode.py 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
