#!/bin/bash
# GPU box: the widened rows' benches (with their reference CPU baselines) and
# rocprofv3 kernel stats of each, written under gpurun_out/rows/.
R=$PWD
O=$R/gpurun_out/rows
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_cook.py tests/test_fec_frame.py tests/test_fec_decode.py \
    -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -u scripts/bench_cook.py > $O/cook.json 2>&1 || exit 1
timeout -k 10 200 python -u scripts/bench_frame.py > $O/frame0.json 2>&1 || exit 1
timeout -k 10 200 python -u scripts/bench_frame.py --mode 1 > $O/frame1.json 2>&1 || exit 1
timeout -k 10 300 python -u scripts/bench_fdec.py > $O/fdec0.json 2>&1 || exit 1
grep -h '^{' $O/cook.json $O/frame0.json $O/frame1.json $O/fdec0.json
cd /tmp && export TMPDIR=/tmp
for b in cook frame fdec; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$b -o run -- \
      python3 $R/scripts/bench_$b.py --cpu-sample 0 > $O/prof_$b.log 2>&1 || exit 1
done
cd $R
for b in cook frame fdec; do python scripts/kstats.py $O/prof_$b/run_kernel_stats.csv | grep rsmi; done
