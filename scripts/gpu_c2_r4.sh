#!/bin/bash
# GPU box, round 4: C2 fused decode -- Lagrange-form variant's parity (decode
# tests through RSMI_LIB), phase traces of both forms, then per-kernel A/B.
set -o pipefail
O=gpurun_out/r4i
mkdir -p $O
RSMI_LIB=$PWD/udpspeeder_amd/ab/librsmi_lag.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 \
    --timeout-method thread -k "decode or c4 or fec or tunnel" > $O/tests_lag.log 2>&1 || { tail -20 $O/tests_lag.log; exit 1; }
tail -2 $O/tests_lag.log
for v in trace tracelag; do
  RSMI_LIB=$PWD/udpspeeder_amd/ab/librsmi_$v.so timeout -k 10 200 python -u scripts/c2_trace.py > $O/c2_$v.txt 2>&1 || { tail $O/c2_$v.txt; exit 1; }
  echo "== $v"; grep -v amdgpu.ids $O/c2_$v.txt
done
bash scripts/gpu_ab_kernels.sh r4i 2 scripts/bench_c2.py main lag lag6
