#!/bin/bash
# GPU box, round 3: the driver's bench command, then a rocprofv3 kernel trace of
# the SAME command (so every bench number can be recomputed from the trace of
# one box), then PMC passes over the C3 kernels (scripts/bench_c3.py).
set -o pipefail
R=$PWD
O=$R/gpurun_out/${1:-r03prof}
mkdir -p $O
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
cut -c1-400 $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
    python3 $R/bench.py --steps 20 --warmup 5 > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
cd $R
python scripts/kstats_grid.py $O/prof/run_kernel_trace.csv > $O/kernel_by_grid.txt
head -30 $O/kernel_by_grid.txt
[ -n "$NO_PMC" ] && exit 0
PMC_SETS="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD;SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_WR" \
  bash scripts/pmc_passes.sh $(basename $O)/pmc_c3 k_bs_ragged k_decode_ragged_cls k_decode_ragged_big -- scripts/bench_c3.py
