#!/bin/bash
# PMC passes (one counter set per rocprofv3 run) over a short command, then a
# per-kernel average summary.  Run on the GPU box from the repo root:
#   bash scripts/pmc_passes.sh <out-name> <kernel-substring...> -- <python script + args>
# e.g. bash scripts/pmc_passes.sh pmc_frame k_frame -- scripts/bench_frame.py --reps 1
# PMC_SETS overrides the counter sets (';'-separated).
set -e
R=$PWD
NAME=$1; shift
KERNELS=()
while [ "$1" != "--" ]; do KERNELS+=("$1"); shift; done
shift
SETS=${PMC_SETS:-"FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU;SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"}
mkdir -p $R/gpurun_out/$NAME
cd /tmp && export TMPDIR=/tmp
IFS=';' read -ra ARR <<< "$SETS"
i=0
for set in "${ARR[@]}"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $set --output-format csv -d $R/gpurun_out/$NAME/p$i -o run -- \
      python3 $R/"$@" > $R/gpurun_out/$NAME/p$i.log 2>&1
done
cd $R
python scripts/pmc_summary.py gpurun_out/$NAME "${KERNELS[@]}" | tee gpurun_out/$NAME/summary.txt
