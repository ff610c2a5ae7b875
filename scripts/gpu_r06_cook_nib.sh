#!/bin/bash
# GPU box (round 6): the conflict-free nibble-table CRC (ab/librsmi_nib.so,
# COOK_NIB=1) against the shipped slicing-by-16 tables: cook tests on the nib
# build, three alternating bench_cook rounds, and an LDS counter pass of each
# (SQ_LDS_BANK_CONFLICT vs SQ_LDS_IDX_ACTIVE).  Output: gpurun_out/r06_nib/.
set -e
set -o pipefail
R=$PWD
O=$R/gpurun_out/r06_nib
mkdir -p $O
RSMI_LIB=$R/udpspeeder_amd/ab/librsmi_nib.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 \
    --timeout-method thread tests/test_gpu_cook.py > $O/nib_tests.log 2>&1
tail -1 $O/nib_tests.log
bash scripts/gpu_ab.sh cook > $O/ab.txt 2>&1
for v in default nib; do
  if [ $v = default ]; then unset RSMI_LIB; else export RSMI_LIB=$R/udpspeeder_amd/ab/librsmi_nib.so; fi
  PMC_SETS="SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU;SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY" \
      bash scripts/pmc_passes.sh r06_nib/pmc_$v k_cook k_decook -- scripts/bench_cook.py --groups 16384 --iters 2 --cpu-sample 0 > /dev/null
done
unset RSMI_LIB
grep -v amdgpu.ids $O/ab.txt
cat $O/pmc_default/summary.txt $O/pmc_nib/summary.txt
