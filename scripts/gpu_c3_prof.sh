#!/bin/bash
# GPU box: C3 ragged encode/decode (scripts/bench_c3.py) under a rocprofv3 kernel
# trace, then one SQ counter pass over the class decode kernels.
R=$PWD
O=$R/gpurun_out/${1:-c3prof}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- \
    python3 $R/scripts/bench_c3.py > $O/kt.log 2>&1 || { tail $O/kt.log; exit 1; }
cd $R
python scripts/kstats_grid.py $O/kt/run_kernel_trace.csv > $O/kernel_by_grid.txt
head -12 $O/kernel_by_grid.txt
grep c3_ $O/kt.log
PMC_SETS="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS" \
  bash scripts/pmc_passes.sh $(basename $O)/pmc k_decode_ragged_cls k_decode_ragged_big k_bs_ragged -- scripts/bench_c3.py
