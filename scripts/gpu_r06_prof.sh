#!/bin/bash
# GPU box (round 6): C3 encode/decode (own and reference placement), the fused
# send path's kernel times (rocprofv3 kernel trace of bench_frame --cook dev)
# and k_cook_frame's FETCH_SIZE / WRITE_SIZE.  Output: gpurun_out/r06_prof/.
set -e
set -o pipefail
R=$PWD
O=$R/gpurun_out/r06_prof
mkdir -p $O
timeout -k 10 200 python -u scripts/bench_c3.py > $O/c3.txt 2>&1
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/frame -o run -- \
    python3 $R/scripts/bench_frame.py --cook dev --cpu-sample 0 --reps 3 > $O/frame.log 2>&1)
python scripts/kstats.py $O/frame/run_kernel_stats.csv > $O/frame_kernels.txt
rm -f $O/frame/run_kernel_trace.csv
PMC_SETS="FETCH_SIZE;WRITE_SIZE" bash scripts/pmc_passes.sh r06_prof/pmc_cookf k_cook_frame k_cook k_bs2 -- \
    scripts/bench_frame.py --cook dev --cpu-sample 0 --reps 2 > /dev/null
cat $O/c3.txt $O/frame_kernels.txt $O/pmc_cookf/summary.txt
# end to end (host memory) on the current device, [0] and [0, 0]
for d in "" "0" "0,0"; do
  E2E_DEVICES=$d timeout -k 10 300 python -u scripts/e2e_host.py > $O/e2e_devs_${d:-current}.json 2>&1
done
