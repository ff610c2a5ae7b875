#!/bin/bash
# GPU box: framing + decode-manager tests (one pytest process).
timeout -k 10 500 python -u -m pytest tests/test_fec_frame.py tests/test_fec_decode.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > gpurun_out/fec_tests.log 2>&1
rc=$?
tail -40 gpurun_out/fec_tests.log
exit $rc
