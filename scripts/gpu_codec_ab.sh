#!/bin/bash
# GPU box: RS(20,10) encode/decode A/B (scripts/ab_encode.py) for the default
# library and every udpspeeder_amd/ab/*.so, twice, plus bench.py for each.
for i in 1 2; do
  timeout -k 10 120 python -u scripts/ab_encode.py 2>&1 | grep -v amdgpu.ids || exit 1
  for lib in udpspeeder_amd/ab/*.so; do
    RSMI_LIB=$PWD/$lib timeout -k 10 120 python -u scripts/ab_encode.py 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
echo -n "bench default: "; timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-extras 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['encode_ms'], d['decode_ms'])"
for lib in udpspeeder_amd/ab/*.so; do
  echo -n "bench $(basename $lib): "; RSMI_LIB=$PWD/$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-extras 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['encode_ms'], d['decode_ms'])"
done
