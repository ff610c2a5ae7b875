#!/bin/bash
# GPU box: decode timing (scripts/dec_timing.py) and one SQ counter pass over
# scripts/ab_encode.py for the default library and every udpspeeder_amd/ab/*.so.
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD"
for lib in default udpspeeder_amd/ab/*.so; do
  name=$(basename $lib .so)
  if [ $lib != default ]; then export RSMI_LIB=$PWD/$lib; else unset RSMI_LIB; fi
  timeout -k 10 100 python -u scripts/dec_timing.py 2>&1 | grep -v amdgpu.ids || exit 1
  PMC_SETS="$SQ" bash scripts/pmc_passes.sh pmc_$name k_decode_fused k_decode_lean -- scripts/ab_encode.py > /dev/null 2>&1 || exit 1
  echo "$name: $(cat gpurun_out/pmc_$name/summary.txt)"
done
