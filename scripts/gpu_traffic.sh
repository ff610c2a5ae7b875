#!/bin/bash
# GPU box: separate FETCH_SIZE / WRITE_SIZE passes over scripts/ab_encode.py (C1
# encode + C2 decode), turned into per-launch HBM bytes for k_bs2_20_30 and
# k_decode_fused (scripts/pmc_traffic.py) in gpurun_out/traffic/.
set -e
R=$PWD
O=$R/gpurun_out/traffic
PMC_SETS="FETCH_SIZE;WRITE_SIZE" bash scripts/pmc_passes.sh traffic k_bs2_20_30 k_decode_fused -- scripts/ab_encode.py > /dev/null
python scripts/pmc_traffic.py $O/p1/run_counter_collection.csv $O/p2/run_counter_collection.csv \
    k_bs2_20_30 65536 2457600000 encode > $O/traffic_encode.json
python - <<'PY' > $O/alg_decode.txt
import sys; sys.path.insert(0, ".")
from udpspeeder_amd import synth
p = synth.erasure_present(synth.ERASE_SEED, 0, 65536, 30, 5)
e = (p[:, :20] == 0).sum(1)
print(int(((e > 0) * 20 * 1250).sum() + (e * 1250).sum()))
PY
python scripts/pmc_traffic.py $O/p1/run_counter_collection.csv $O/p2/run_counter_collection.csv \
    k_decode_fused 65536 $(cat $O/alg_decode.txt) decode > $O/traffic_decode.json
cat $O/traffic_encode.json $O/traffic_decode.json
