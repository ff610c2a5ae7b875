#!/bin/bash
# GPU box: the round-end sequence -- every GPU test, smoke(), the bench line and
# a rocprofv3 kernel-stats pass over the same bench command.
R=$PWD
O=$R/gpurun_out/final
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
grep smoke $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
    python3 $R/bench.py --no-cpu-baseline > $O/prof.log 2>&1 || exit 1
cd $R
python scripts/kstats.py $O/prof/run_kernel_stats.csv | grep rsmi
timeout -k 10 300 python -u scripts/e2e_host.py > $O/e2e.json 2> $O/e2e.err || { tail $O/e2e.err; exit 1; }
tail -5 $O/e2e.json
