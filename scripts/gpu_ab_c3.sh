#!/bin/bash
# GPU box: scripts/bench_c3.py (C3 ragged encode + decode) alternating the default
# library and every udpspeeder_amd/ab/*.so, three rounds.
for i in ${ROUNDS:-1 2 3}; do
  for lib in "" udpspeeder_amd/ab/*.so; do
    echo -n "${lib:-default}: "
    env ${lib:+RSMI_LIB=$PWD/$lib} timeout -k 10 200 python -u scripts/bench_c3.py 2>/dev/null | tr '\n' ' ' || exit 1
    echo
  done
done
