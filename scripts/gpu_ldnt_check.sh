#!/bin/bash
# GPU box: nt decode loads (ab/librsmi_ldnt.so) under the two-stream scenario and
# the full GPU suite, then the encode/decode A/B against the default library.
L=$PWD/udpspeeder_amd/ab/librsmi_ldnt.so
RSMI_LIB=$L timeout -k 10 300 python -u scripts/dbg_streams.py 64 two both | grep -v ": ok$"; echo "streams done"
RSMI_LIB=$L timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
    > gpurun_out/suite_ldnt.log 2>&1; echo "suite: $(tail -1 gpurun_out/suite_ldnt.log)"
for i in 1 2; do
  timeout -k 10 120 python -u scripts/ab_encode.py 2>&1 | grep -v amdgpu.ids
  RSMI_LIB=$L timeout -k 10 120 python -u scripts/ab_encode.py 2>&1 | grep -v amdgpu.ids
done
