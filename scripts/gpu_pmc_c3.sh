#!/bin/bash
# GPU box: PMC passes over scripts/bench_c3.py (C3 ragged encode k_bs_ragged and
# decode k_decode_ragged): traffic, instruction mix and wait cycles.
PMC_SETS="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD;SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_WR" \
  bash scripts/pmc_passes.sh ${1:-pmc_c3} k_bs_ragged k_decode_ragged -- scripts/bench_c3.py
