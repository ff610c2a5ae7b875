#!/bin/bash
# GPU box: framing tests, framing bench (both modes) and a rocprofv3 kernel-stats pass.
R=$PWD
timeout -k 10 400 python -u -m pytest tests/test_fec_frame.py -m gpu -x -q --timeout 120 \
    --timeout-method thread > gpurun_out/fec_tests.log 2>&1 || { tail -30 gpurun_out/fec_tests.log; exit 1; }
tail -2 gpurun_out/fec_tests.log
timeout -k 10 200 python -u scripts/bench_frame.py > gpurun_out/frame0.json 2>&1 || exit 1
timeout -k 10 200 python -u scripts/bench_frame.py --mode 1 > gpurun_out/frame1.json 2>&1 || exit 1
grep -h '^{' gpurun_out/frame0.json gpurun_out/frame1.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_frame \
    -o run -- python3 $R/scripts/bench_frame.py --reps 2 > $R/gpurun_out/prof_frame.log 2>&1 || exit 1
cd $R
python scripts/kstats.py gpurun_out/prof_frame/run_kernel_stats.csv
