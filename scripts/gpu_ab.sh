#!/bin/bash
# GPU box: kernel A/B, the default library against every udpspeeder_amd/ab/*.so,
# alternating, three rounds.  $1: benches to run (c2, c3 or "c2 c3"; default c2);
# $2: optional pytest -k filter run first on the default library.
set -o pipefail
mkdir -p gpurun_out
benches=${1:-c2}
if [ -n "$2" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$2" > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
  tail -2 gpurun_out/ab_tests.log
fi
for i in 1 2 3; do
  for lib in default udpspeeder_amd/ab/*.so; do
    for b in $benches; do
      args=""
      [ "$b" = cook ] && args="--cpu-sample 0 --iters 20"
      [ "$b" = frame ] && args="--cook dev --cpu-sample 0"
      if [ "$lib" = default ]; then
        echo -n "default $b: "; timeout -k 10 150 python -u scripts/bench_$b.py $args | tr '\n' ' ' || exit 1
      else
        echo -n "$(basename $lib) $b: "; RSMI_LIB=$PWD/$lib timeout -k 10 150 python -u scripts/bench_$b.py $args | tr '\n' ' ' || exit 1
      fi
      echo
    done
  done
done
