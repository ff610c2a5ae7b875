#!/bin/bash
# GPU box, round 3: k_cook two-chain CRC fold (default) against one chain
# (ab/librsmi_onech.so): cook parity tests on the default library, then
# bench_cook.py alternating three times.
mkdir -p gpurun_out/ck3
timeout -k 10 300 python -u -m pytest tests/test_gpu_cook.py tests/test_fec_frame.py -m gpu -x -q -k "cook or cooked" \
    --timeout 120 --timeout-method thread > gpurun_out/ck3/tests.log 2>&1 || { tail -5 gpurun_out/ck3/tests.log; exit 1; }
tail -1 gpurun_out/ck3/tests.log
for i in 1 2 3; do
  for l in default $PWD/udpspeeder_amd/ab/librsmi_onech.so; do
    [ $l = default ] && unset RSMI_LIB || export RSMI_LIB=$l
    echo "$(basename $l) $(timeout -k 10 120 python -u scripts/bench_cook.py --cpu-sample 0 2>&1 | grep -v amdgpu.ids | tail -1 | cut -c1-200)" || exit 1
  done
done
