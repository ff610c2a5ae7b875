#!/bin/bash
# GPU box, round 3 A/B: cook with slicing-by-16 (default) against slicing-by-8
# (ab/librsmi_s8.so) and nt packet loads/stores (ab/librsmi_cooknt.so); ragged
# decode survivor loads without nt (ab/librsmi_ragld0.so) on C3 decode.
# Parity tests for each library first, then timings alternating.
mkdir -p gpurun_out/aux
AB=$PWD/udpspeeder_amd/ab
run_tests() {  # name lib tests -k
  [ $2 = default ] && unset RSMI_LIB || export RSMI_LIB=$2
  timeout -k 10 300 python -u -m pytest $3 -m gpu -x -q -k "$4" --timeout 120 --timeout-method thread \
      > gpurun_out/aux/tests_$1.log 2>&1 || { tail -5 gpurun_out/aux/tests_$1.log; exit 1; }
  echo "$1: $(tail -1 gpurun_out/aux/tests_$1.log)"
}
COOKT="tests/test_gpu_cook.py tests/test_fec_frame.py"
run_tests default_cook default "$COOKT" "cook or cooked"
run_tests cooknt $AB/librsmi_cooknt.so "$COOKT" "cook or cooked"
run_tests ragld0 $AB/librsmi_ragld0.so tests/test_gpu_parity.py "ragged or plan"
for i in 1 2 3; do
  for l in default $AB/librsmi_s8.so $AB/librsmi_cooknt.so; do
    [ $l = default ] && unset RSMI_LIB || export RSMI_LIB=$l
    echo "$(basename $l) $(timeout -k 10 120 python -u scripts/bench_cook.py --cpu-sample 0 2>&1 | grep -v amdgpu.ids | tail -1 | cut -c1-200)" || exit 1
  done
done
for i in 1 2 3; do
  for l in default $AB/librsmi_ragld0.so; do
    [ $l = default ] && unset RSMI_LIB || export RSMI_LIB=$l
    echo "$(basename $l) $(timeout -k 10 120 python -u scripts/bench_c3.py 2>&1 | grep c3_decode)" || exit 1
  done
done
