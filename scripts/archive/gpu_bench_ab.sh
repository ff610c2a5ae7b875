#!/bin/bash
# GPU box: bench.py (no CPU baseline, no extras) alternating the default library
# and every udpspeeder_amd/ab/*.so, three rounds; then one full bench.py line.
for i in 1 2 3; do
  echo -n "bench default: "; timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-extras 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['encode_ms'], d['decode_ms'])" || exit 1
  for lib in udpspeeder_amd/ab/*.so; do
    echo -n "bench $(basename $lib): "; RSMI_LIB=$PWD/$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-extras 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['encode_ms'], d['decode_ms'])" || exit 1
  done
done
