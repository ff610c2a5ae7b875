set -o pipefail
mkdir -p gpurun_out/r4b
RSMI_LIB=udpspeeder_amd/ab/librsmi_trace.so timeout -k 10 200 python -u scripts/c3_trace.py > gpurun_out/r4b/c3_trace.txt 2>&1 || { tail gpurun_out/r4b/c3_trace.txt; exit 1; }
cat gpurun_out/r4b/c3_trace.txt
PMC_SETS="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD;SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_WR" \
  bash scripts/pmc_passes.sh r4b/pmc_c3 k_bs_ragged k_decode_ragged_cls k_decode_ragged_big -- scripts/bench_c3.py
