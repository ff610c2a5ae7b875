#!/bin/bash
# GPU box: the decoder's copy back on its own stream (RSMI_FDEC_COPY_STREAM=1)
# or on the caller's (0), scripts/bench_pipeline.py --conns 1,2,4, alternating, two rounds.
set -o pipefail
mkdir -p gpurun_out/copy_stream_ab
for i in 1 2; do
  for v in 1 0; do
    RSMI_FDEC_COPY_STREAM=$v timeout -k 10 300 python -u scripts/bench_pipeline.py --conns 1,2,4 \
        > gpurun_out/copy_stream_ab/cs${v}_$i.json 2>/dev/null || exit 1
    python3 -c "
import json; d=json.load(open('gpurun_out/copy_stream_ab/cs${v}_$i.json'))['decode']
print('copy_stream=$v', ' '.join(f'{k}:{v[\"Mpps_in\"]}' for k, v in d.items()))"
  done
done
