#!/bin/bash
# GPU box: FEC decoder tests, then bench_fdec (steady state, no CPU baseline).
timeout -k 10 300 python -u -m pytest tests/test_fec_decode.py -m gpu -q --timeout 120 \
    --timeout-method thread > gpurun_out/fdec_tests.log 2>&1 || { tail -30 gpurun_out/fdec_tests.log; exit 1; }
tail -1 gpurun_out/fdec_tests.log
timeout -k 10 300 python -u scripts/bench_fdec.py --cpu-sample 0 2>&1 | grep '^{' || exit 1
RSMI_HOST_THREADS=1 timeout -k 10 300 python -u scripts/bench_fdec.py --cpu-sample 0 2>&1 | grep '^{' || exit 1
