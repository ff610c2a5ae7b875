#!/bin/bash
# GPU box: PMC passes over the C1 encode + decode A/B script (k_bs_20_30, k_decode_fused).
PMC_SETS="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU;SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM" \
  bash scripts/pmc_passes.sh pmc_dec k_bs_20_30 k_decode_fused -- scripts/ab_encode.py
