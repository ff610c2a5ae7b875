#!/bin/bash
# GPU box: scripts/diag_streams.py without the cross-stream ordering, for the
# default library and the udpspeeder_amd/ab variants; output in gpurun_out/.
export RSMI_STREAM_ORDER=0
REPS=${1:-200}; G=${2:-2048}
timeout -k 10 240 python -u scripts/diag_streams.py $REPS $G > gpurun_out/diag_default.log 2>&1 || exit 1
tail -1 gpurun_out/diag_default.log
for lib in udpspeeder_amd/ab/*.so; do
  b=$(basename $lib .so)
  RSMI_LIB=$PWD/$lib timeout -k 10 240 python -u scripts/diag_streams.py $REPS $G > gpurun_out/diag_$b.log 2>&1 || exit 1
  tail -1 gpurun_out/diag_$b.log
done
