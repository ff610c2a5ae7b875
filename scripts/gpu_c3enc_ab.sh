#!/bin/bash
# GPU box: C3 ragged encode A/B -- ragged/plan/rtc parity tests on the default
# library and every ab/*.so, then the C3 encode timing (bench_c3.py)
# alternating between the libraries three times.
mkdir -p gpurun_out/c3enc
libs="default"
for l in udpspeeder_amd/ab/*.so; do libs="$libs $l"; done
for lib in $libs; do
  [ $lib = default ] && unset RSMI_LIB || export RSMI_LIB=$PWD/$lib
  timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_bitslice_rtc.py -m gpu -x -q -k "ragged or plan or rtc" \
      --timeout 120 --timeout-method thread > gpurun_out/c3enc/tests_$(basename $lib).log 2>&1; rc=$?
  echo "$lib: $(tail -1 gpurun_out/c3enc/tests_$(basename $lib).log)"
  [ $rc -eq 0 ] || exit $rc
done
for i in 1 2 3; do
  for lib in $libs; do
    [ $lib = default ] && unset RSMI_LIB || export RSMI_LIB=$PWD/$lib
    echo "$lib $(timeout -k 10 120 python -u scripts/bench_c3.py 2>&1 | grep c3_encode)" || exit 1
  done
done
