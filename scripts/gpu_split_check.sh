#!/bin/bash
# GPU box: encode parity tests (split-k networks included), then the bench A/B.
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
    -k "encode or c1 or roundtrip or concurrent or hipgraph" > gpurun_out/split_tests.log 2>&1 || { tail -30 gpurun_out/split_tests.log; exit 1; }
tail -2 gpurun_out/split_tests.log
bash scripts/gpu_bench_ab.sh
