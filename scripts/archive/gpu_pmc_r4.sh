#!/bin/bash
# GPU box, round 4: counter passes (FETCH_SIZE, WRITE_SIZE and two sets of 8 SQ
# counters, one rocprofv3 run each) over the shipped kernels -- the C1 encode
# and C2 decode (scripts/ab_encode.py), cook / de_cook (scripts/bench_cook.py)
# and the C3 kernels (scripts/bench_c3.py) -- then per-kernel summaries and
# the per-launch HBM bytes bench.py reports as roofline traffic
# (scripts/pmc_traffic.py).  Output: gpurun_out/pmc4_*/.
set -e
export PMC_SETS="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD;SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_WR"
bash scripts/pmc_passes.sh pmc4_codec k_bs2_20_30 k_decode_fused -- scripts/ab_encode.py
O=gpurun_out/pmc4_codec
python scripts/pmc_traffic.py $O/p1/run_counter_collection.csv $O/p2/run_counter_collection.csv \
    k_bs2_20_30 65536 2457600000 > $O/traffic.json
python - <<'PY' > $O/alg_decode.txt
import sys; sys.path.insert(0, ".")
from udpspeeder_amd import synth
p = synth.erasure_present(synth.ERASE_SEED, 0, 65536, 30, 5)
e = (p[:, :20] == 0).sum(1)
print(int(((e > 0) * 20 * 1250).sum() + (e * 1250).sum()))
PY
python scripts/pmc_traffic.py $O/p1/run_counter_collection.csv $O/p2/run_counter_collection.csv \
    k_decode_fused 65536 $(cat $O/alg_decode.txt) > $O/traffic_decode.json
cat $O/traffic.json $O/traffic_decode.json
bash scripts/pmc_passes.sh pmc4_cook k_cook k_decook -- scripts/bench_cook.py
bash scripts/pmc_passes.sh pmc4_c3 k_bs_ragged k_decode_ragged_mix -- scripts/bench_c3.py
