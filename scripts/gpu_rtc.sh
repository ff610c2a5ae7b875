#!/bin/bash
# GPU box: run-time bit-sliced encoders -- parity tests, then one bench line
# (extras include rtc_f10_5_encode).  Logs under gpurun_out/.
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_bitslice_rtc.py -m gpu -x -v --timeout 200 \
    --timeout-method thread > gpurun_out/rtc_tests.log 2>&1; rc=$?
tail -15 gpurun_out/rtc_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py --no-cpu-baseline > gpurun_out/rtc_bench.json 2> gpurun_out/rtc_bench.err; rc=$?
tail -c 3000 gpurun_out/rtc_bench.json
exit $rc
