#!/bin/bash
# GPU box (round 6): the parity cook in the encoder's epilogue -- its tests,
# the A/B on the f1_f2 workload, and the A/B under rocprofv3 (kernel stats).
# Output: gpurun_out/r06_pcook/.
set -o pipefail
R=$PWD
O=gpurun_out/r06_pcook
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity_cook.py tests/test_gpu_copy_peak.py tests/test_gpu_ref_placement.py tests/test_fec_frame.py tests/test_gpu_cook.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python scripts/ab_parity_cook.py > $O/ab.json 2> $O/ab.err || { tail $O/ab.err; exit 1; }
cat $O/ab.json
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- \
    python3 $R/scripts/ab_parity_cook.py > $R/$O/prof_ab.json 2> $R/$O/prof_ab.err) || { tail $O/prof_ab.err; exit 1; }
python scripts/kstats_grid.py $O/prof/run_kernel_trace.csv > $O/kernel_by_grid.txt
rm -f $O/prof/run_kernel_trace.csv
head -30 $O/kernel_by_grid.txt
