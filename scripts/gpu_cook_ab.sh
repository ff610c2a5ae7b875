#!/bin/bash
# GPU box: cook tests + bench_cook for the default library and every
# udpspeeder_amd/ab/*.so (RSMI_LIB).
timeout -k 10 300 python -u -m pytest tests/test_gpu_cook.py -m gpu -x -q --timeout 120 \
    --timeout-method thread > gpurun_out/cook_tests.log 2>&1 || { tail -30 gpurun_out/cook_tests.log; exit 1; }
tail -1 gpurun_out/cook_tests.log
for lib in udpspeeder_amd/ab/*.so; do
  [ -e "$lib" ] || continue
  RSMI_LIB=$PWD/$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_cook.py -m gpu -x -q --timeout 120 \
      --timeout-method thread > gpurun_out/cook_tests_ab.log 2>&1 || { tail -30 gpurun_out/cook_tests_ab.log; exit 1; }
  echo "$(basename $lib): $(tail -1 gpurun_out/cook_tests_ab.log)"
done
for i in 1 2; do
  echo -n "default: "
  timeout -k 10 120 python -u scripts/bench_cook.py --cpu-sample 0 --iters 10 2>&1 | grep '^{' || exit 1
  for lib in udpspeeder_amd/ab/*.so; do
    [ -e "$lib" ] || continue
    echo -n "$(basename $lib): "
    RSMI_LIB=$PWD/$lib timeout -k 10 120 python -u scripts/bench_cook.py --cpu-sample 0 --iters 10 2>&1 | grep '^{' || exit 1
  done
done
