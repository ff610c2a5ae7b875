#!/bin/bash
# GPU box: C3 ragged decode A/B -- ragged parity tests on the default library
# and every ab/*.so that is not a trace build, C3 timing (bench_c3.py) per
# library twice, then the phase trace (c3_trace.py) for each trace build.
mkdir -p gpurun_out/c3ab
libs="default"
for l in udpspeeder_amd/ab/*.so; do case $l in *trace*) ;; *) libs="$libs $l";; esac; done
for lib in $libs; do
  [ $lib = default ] && unset RSMI_LIB || export RSMI_LIB=$PWD/$lib
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "ragged or plan" \
      --timeout 120 --timeout-method thread > gpurun_out/c3ab/tests_$(basename $lib).log 2>&1; rc=$?
  echo "$lib: $(tail -1 gpurun_out/c3ab/tests_$(basename $lib).log)"
  [ $rc -eq 0 ] || exit $rc
done
for i in 1 2; do
  for lib in $libs; do
    [ $lib = default ] && unset RSMI_LIB || export RSMI_LIB=$PWD/$lib
    echo "$lib $(timeout -k 10 120 python -u scripts/bench_c3.py 2>&1 | grep c3_decode)" || exit 1
  done
done
for l in udpspeeder_amd/ab/*trace*.so; do
  echo "== $l"
  RSMI_LIB=$PWD/$l timeout -k 10 200 python -u scripts/c3_trace.py 2>&1 | grep -v amdgpu.ids || exit 1
done
