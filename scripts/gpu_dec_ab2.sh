#!/bin/bash
# GPU box: scripts/dec_timing.py for the default library and every udpspeeder_amd/ab/*.so.
for lib in default udpspeeder_amd/ab/*.so; do
  if [ $lib != default ]; then export RSMI_LIB=$PWD/$lib; else unset RSMI_LIB; fi
  timeout -k 10 100 python -u scripts/dec_timing.py 2>&1 | grep -v amdgpu.ids | grep "b2b\|worst" || exit 1
done
