#!/bin/bash
# GPU box: receive-side bench + rocprofv3 kernel stats of it.
R=$PWD
timeout -k 10 300 python -u scripts/bench_fdec.py > gpurun_out/fdec0.json 2>&1 || { tail -20 gpurun_out/fdec0.json; exit 1; }
grep -h '^{' gpurun_out/fdec0.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_fdec \
    -o run -- python3 $R/scripts/bench_fdec.py --reps 1 > $R/gpurun_out/prof_fdec.log 2>&1 || exit 1
cd $R
python scripts/kstats.py gpurun_out/prof_fdec/run_kernel_stats.csv
