#!/bin/bash
# GPU box (round 6): the split-k ragged encode (BS_RAG_SPLIT) -- the ragged
# encode tests, then C3 encode with the default build and a BS_RAG_SPLIT=0
# build (udpspeeder_amd/ab/librsmi_ragnosplit.so) alternating, 3 runs each,
# then the default under rocprofv3.  Output: gpurun_out/r06_ragsplit/.
set -o pipefail
R=$PWD
O=gpurun_out/r06_ragsplit
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_bitslice_rtc.py tests/test_multidev.py -m gpu -x -q -k "ragged" \
    --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2 3; do
  timeout -k 10 200 python scripts/bench_c3.py > $O/split_$i.json 2>> $O/err.log || { tail $O/err.log; exit 1; }
  RSMI_LIB=$R/udpspeeder_amd/ab/librsmi_ragnosplit.so timeout -k 10 200 python scripts/bench_c3.py > $O/nosplit_$i.json 2>> $O/err.log || { tail $O/err.log; exit 1; }
done
head -1 $O/split_*.json $O/nosplit_*.json
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- \
    python3 $R/scripts/bench_c3.py > $R/$O/prof_c3.json 2> $R/$O/prof_c3.err) || { tail $O/prof_c3.err; exit 1; }
python scripts/kstats_grid.py $O/prof/run_kernel_trace.csv > $O/kernel_by_grid.txt
rm -f $O/prof/run_kernel_trace.csv
head -12 $O/kernel_by_grid.txt
