#!/bin/bash
# GPU box: the two-stream encode/erase/decode scenario (scripts/dbg_streams.py)
# for the default library and every udpspeeder_amd/ab/*.so, then the codec A/B.
N=${1:-64}
timeout -k 10 300 python -u scripts/dbg_streams.py $N two both | grep -v ": ok$"
echo "default done"
for lib in udpspeeder_amd/ab/*.so; do
  RSMI_LIB=$PWD/$lib timeout -k 10 300 python -u scripts/dbg_streams.py $N two both | grep -v ": ok$"
  echo "$(basename $lib) done"
done
timeout -k 10 120 python -u scripts/ab_encode.py 2>&1 | grep -v amdgpu.ids
for lib in udpspeeder_amd/ab/*.so; do
  RSMI_LIB=$PWD/$lib timeout -k 10 120 python -u scripts/ab_encode.py 2>&1 | grep -v amdgpu.ids
done
