#!/bin/bash
# PMC passes over the cook/de_cook bench (one counter set per rocprofv3 run).
# Run on the GPU box from the repo root; writes gpurun_out/pmc_cook/<pass>/...
# Usage: bash scripts/pmc_cook.sh [bench_cook.py args]; PMC_SETS overrides the sets
# (';'-separated).
set -e
R=$PWD
cd /tmp && export TMPDIR=/tmp
SETS=${PMC_SETS:-"FETCH_SIZE;WRITE_SIZE;SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT;SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES;SQ_BUSY_CYCLES SQ_WAVE_CYCLES"}
mkdir -p $R/gpurun_out/pmc_cook
IFS=';' read -ra ARR <<< "$SETS"
i=0
for set in "${ARR[@]}"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $set --output-format csv -d $R/gpurun_out/pmc_cook/p$i -o run -- \
      python3 $R/scripts/bench_cook.py --groups 16384 --iters 2 "$@" > $R/gpurun_out/pmc_cook/p$i.log 2>&1
done
