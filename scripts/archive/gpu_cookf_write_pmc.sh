#!/bin/bash
# GPU box: FETCH_SIZE / WRITE_SIZE of k_cook_frame per store stream -- the
# shipped kernel, and the measurement builds without its plain slot stores
# (ab/librsmi_ns.so) or without its cooked stores (ab/librsmi_no.so) -- over
# scripts/bench_frame.py --cook dev.  Output: gpurun_out/pmc_cookf_<v>/.
set -e
export PMC_SETS="FETCH_SIZE;WRITE_SIZE"
R=$PWD
bash scripts/pmc_passes.sh pmc_cookf_default k_cook_frame k_cook k_bs2 -- scripts/bench_frame.py --cook dev --cpu-sample 0 --reps 2
for v in ns no; do
  RSMI_LIB=$R/udpspeeder_amd/ab/librsmi_$v.so bash scripts/pmc_passes.sh pmc_cookf_$v k_cook_frame k_cook k_bs2 -- \
      scripts/bench_frame.py --cook dev --cpu-sample 0 --reps 2
done
