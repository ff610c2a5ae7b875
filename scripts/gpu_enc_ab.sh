#!/bin/bash
# GPU box: encode/decode A/B (scripts/ab_encode.py) alternating the default
# library and every udpspeeder_amd/ab/*.so, three rounds.
for i in 1 2 3; do
  timeout -k 10 120 python -u scripts/ab_encode.py || exit 1
  for lib in udpspeeder_amd/ab/*.so; do
    RSMI_LIB=$PWD/$lib timeout -k 10 120 python -u scripts/ab_encode.py || exit 1
  done
done
