#!/bin/bash
# GPU box: k_cook_frame without the plain header piece (the 16 B its grid
# starts with, 112 B into a 128-B line; measurement build ab/librsmi_h0.so):
# WRITE_SIZE and kernel time against the shipped kernel.
set -e
export PMC_SETS="WRITE_SIZE"
R=$PWD
bash scripts/pmc_passes.sh pmc_cookf_h0def k_cook_frame -- scripts/bench_frame.py --cook dev --cpu-sample 0 --reps 2
RSMI_LIB=$R/udpspeeder_amd/ab/librsmi_h0.so bash scripts/pmc_passes.sh pmc_cookf_h0 k_cook_frame -- \
    scripts/bench_frame.py --cook dev --cpu-sample 0 --reps 2
bash scripts/gpu_cookf_probe.sh
