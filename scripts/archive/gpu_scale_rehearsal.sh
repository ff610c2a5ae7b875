#!/bin/bash
# GPU box (1 GPU): the N > 1 bench paths rehearsed with every rank on cuda:0
# (gloo), plus the C3 workload line at N = 1.  Lines go to gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --workload c3 --steps 10 --warmup 2 > gpurun_out/c3_n1.json 2> gpurun_out/c3_n1.err || { tail -20 gpurun_out/c3_n1.err; exit 1; }
cat gpurun_out/c3_n1.json
timeout -k 10 400 python -u bench.py --gpus 2 --share-device --backend gloo --steps 5 --warmup 1 --no-extras > gpurun_out/c4_n2_rehearsal.json 2> gpurun_out/c4_n2_rehearsal.err || { tail -20 gpurun_out/c4_n2_rehearsal.err; exit 1; }
cat gpurun_out/c4_n2_rehearsal.json
timeout -k 10 400 python -u bench.py --gpus 2 --share-device --backend gloo --workload c3 --steps 5 --warmup 1 --total-groups 262144 > gpurun_out/c3_n2_rehearsal.json 2> gpurun_out/c3_n2_rehearsal.err || { tail -20 gpurun_out/c3_n2_rehearsal.err; exit 1; }
cat gpurun_out/c3_n2_rehearsal.json
