#!/bin/bash
# GPU box: tests/test_gpu_parity.py twice for the default library and for every
# udpspeeder_amd/ab/*.so (RSMI_LIB); one summary line per run.
for rep in 1 2; do
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 120 --timeout-method thread \
      > gpurun_out/parity_default_$rep.log 2>&1
  echo "default $rep: $(tail -1 gpurun_out/parity_default_$rep.log)"
  for lib in udpspeeder_amd/ab/*.so; do
    [ -e "$lib" ] || continue
    b=$(basename $lib .so)
    RSMI_LIB=$PWD/$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 120 \
        --timeout-method thread > gpurun_out/parity_${b}_$rep.log 2>&1
    echo "$b $rep: $(tail -1 gpurun_out/parity_${b}_$rep.log)"
  done
done
