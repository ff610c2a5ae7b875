#!/bin/bash
# GPU box: bpermute-MAC decode iteration -- the ds_bpermute probe, the decode
# parity tests on the default library, then decode timing (dec_timing.py) for
# the default library and every udpspeeder_amd/ab/*.so.  Logs in gpurun_out/bp/.
mkdir -p gpurun_out/bp
timeout -k 10 120 ./scripts/probes/bperm_probe > gpurun_out/bp/probe.txt 2>&1; rc=$?
cat gpurun_out/bp/probe.txt | grep -v amdgpu.ids
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest ${BP_TESTS:-tests/test_gpu_parity.py tests/test_gpu_c4.py} -m gpu -x -q \
    --timeout 120 --timeout-method thread > gpurun_out/bp/tests.log 2>&1; rc=$?
tail -5 gpurun_out/bp/tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/bp/tests.log | head -30; exit $rc; }
pat=${BP_PATTERNS:-b2b,dec_only,worst}
for i in 1 2; do
  timeout -k 10 120 python -u scripts/dec_timing.py $pat 2>&1 | grep -v amdgpu.ids || exit 1
  for lib in udpspeeder_amd/ab/*.so; do
    RSMI_LIB=$PWD/$lib timeout -k 10 120 python -u scripts/dec_timing.py $pat 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
