#!/bin/bash
# GPU box: scripts/ab_encode.py (C1 encode + C2 decode, 40 reps) for the default
# library and every udpspeeder_amd/ab/*.so, twice.
for i in 1 2; do
  timeout -k 10 120 python -u scripts/ab_encode.py 2>&1 | grep -v amdgpu.ids || exit 1
  for lib in udpspeeder_amd/ab/*.so; do
    RSMI_LIB=$PWD/$lib timeout -k 10 120 python -u scripts/ab_encode.py 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
