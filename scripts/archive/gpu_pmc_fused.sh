#!/bin/bash
# GPU box: counter passes over the fused run (scripts/ab_frame_cook.py):
# FETCH_SIZE, WRITE_SIZE and two SQ sets for k_cook_frame and the parity
# k_cook; then per-launch HBM bytes of k_cook_frame against its algorithmic
# bytes (payload read + plain packet written + cooked packet written).
set -e
export PMC_SETS="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD;SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_WR"
bash scripts/pmc_passes.sh pmc4_fused k_cook_frame "k_cook(" -- scripts/ab_frame_cook.py
O=gpurun_out/pmc4_fused
# 1,310,720 data packets: 1200-B payload read, 8 + 1203 B written plain,
# 1211 + 4 + 19 (mean iv + iv_len) B written cooked
python scripts/pmc_traffic.py $O/p1/run_counter_collection.csv $O/p2/run_counter_collection.csv \
    k_cook_frame 65536 $((1310720 * (1200 + 1211 + 1234))) > $O/traffic_cook_frame.json
cat $O/traffic_cook_frame.json
