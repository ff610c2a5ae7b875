#!/bin/bash
# GPU box: k_cook_frame's time per launch (rocprofv3 kernel trace of
# scripts/bench_frame.py --cook dev) for the measurement builds in
# udpspeeder_amd/ab/ (COOKF_PROBE: stores or loads removed; wrong output).
set -o pipefail
R=$PWD
mkdir -p gpurun_out/cookf_probe
for v in default $(ls udpspeeder_amd/ab/ | sed 's/librsmi_//; s/.so//'); do
  d=$R/gpurun_out/cookf_probe/$v
  if [ $v = default ]; then e=""; else e="RSMI_LIB=$R/udpspeeder_amd/ab/librsmi_$v.so"; fi
  (cd /tmp && export TMPDIR=/tmp && env $e timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- \
      python3 $R/scripts/bench_frame.py --cook dev --cpu-sample 0 --reps 3 > $d.log 2>&1) || { tail $d.log; exit 1; }
  echo "== $v"; python scripts/kstats.py $d/run_kernel_stats.csv | grep -i "cook\|bs2" | cut -c1-120
  rm -f $d/run_kernel_trace.csv
done
