#!/bin/bash
# GPU box (round 6, final): the whole -m gpu suite and smoke, the plain bench
# command, the same command under rocprofv3 (kernel trace + stats), and the
# FETCH_SIZE / WRITE_SIZE passes behind bench.py's roofline.traffic.
# Output: gpurun_out/r06_final/ (copied into profiles/r06/final/).
set -o pipefail
R=$PWD
O=gpurun_out/r06_final
mkdir -p $O
s=$(date +%s)
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
echo "pytest process_wall_s=$(( $(date +%s) - s ))" | tee -a $O/gpu_tests.log
tail -2 $O/gpu_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
timeout -k 10 240 python bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- \
    python3 $R/bench.py > $R/$O/prof_bench.json 2> $R/$O/prof_bench.err) || { tail $O/prof_bench.err; exit 1; }
python scripts/kstats.py $O/prof/run_kernel_stats.csv > $O/kernel_stats.txt
python scripts/kstats_grid.py $O/prof/run_kernel_trace.csv > $O/kernel_by_grid.txt
rm -f $O/prof/run_kernel_trace.csv
bash scripts/gpu_traffic.sh > $O/traffic.txt 2>&1 || { tail $O/traffic.txt; exit 1; }
cp gpurun_out/traffic/traffic_encode.json gpurun_out/traffic/traffic_decode.json $O/
cp gpurun_out/traffic/p1/run_counter_collection.csv $O/traffic_fetch_counters.csv
cp gpurun_out/traffic/p2/run_counter_collection.csv $O/traffic_write_counters.csv
# the counters behind DESIGN's C3 and cook paragraphs (one set per pass)
bash scripts/pmc_passes.sh pmc6_c3 k_bs_ragged k_decode_ragged_mix -- scripts/bench_c3.py > $O/pmc6_c3.txt 2>&1 || { tail $O/pmc6_c3.txt; exit 1; }
PMC_SETS="FETCH_SIZE;WRITE_SIZE;SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVES;SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU" \
    bash scripts/pmc_passes.sh pmc6_cook k_cook k_decook -- scripts/bench_cook.py > $O/pmc6_cook.txt 2>&1 || { tail $O/pmc6_cook.txt; exit 1; }
cat $O/pmc6_c3.txt $O/pmc6_cook.txt
head -30 $O/kernel_by_grid.txt
