#!/bin/bash
# GPU box: fused decode A/B -- decode parity tests on each ab/*.so, then
# dec_timing.py (b2b, dec_only, worst) for the default library and each ab/*.so, twice.
mkdir -p gpurun_out/dab
for l in udpspeeder_amd/ab/*.so; do
  RSMI_LIB=$PWD/$l timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "decode and not ragged" \
      --timeout 120 --timeout-method thread > gpurun_out/dab/tests_$(basename $l).log 2>&1; rc=$?
  echo "$l: $(tail -1 gpurun_out/dab/tests_$(basename $l).log)"
  [ $rc -eq 0 ] || exit $rc
done
for i in 1 2; do
  timeout -k 10 120 python -u scripts/dec_timing.py b2b,dec_only,worst 2>&1 | grep -v amdgpu.ids || exit 1
  for l in udpspeeder_amd/ab/*.so; do
    RSMI_LIB=$PWD/$l timeout -k 10 120 python -u scripts/dec_timing.py b2b,dec_only,worst 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
