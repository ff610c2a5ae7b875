#!/bin/bash
# GPU box: level-1 drop-in latency A/B (scripts/dropin_trace.py), alternating,
# three rounds: the default library with the one-group path's pinned memory
# default / coherent / uncached (RSMI_ONE_HOSTMEM 0/1/2), and the server's poll spacing
# (udpspeeder_amd/ab/librsmi_g<N>.so, SRV_GAP=N).  Parity first:
# tests/test_dropin_server.py on every variant.
set -o pipefail
mkdir -p gpurun_out
AB=$PWD/udpspeeder_amd/ab
run_t() {  # $1 label, then env assignments
  local lab=$1; shift
  env "$@" timeout -k 10 120 python -u -m pytest tests/test_dropin_server.py tests/test_dropin_link.py -m gpu -x -q \
      --timeout 60 --timeout-method thread > gpurun_out/dropin_ab_t_$lab.log 2>&1 || { tail -20 gpurun_out/dropin_ab_t_$lab.log; exit 1; }
  echo "tests $lab: $(tail -1 gpurun_out/dropin_ab_t_$lab.log)"
}
run_t mem1 RSMI_ONE_HOSTMEM=1
run_t mem2 RSMI_ONE_HOSTMEM=2
for g in g1 g16 g64; do run_t $g RSMI_LIB=$AB/librsmi_$g.so; done
for i in 1 2 3; do
  for v in mem0 mem1 mem2 g1 g16 g64; do
    case $v in
      mem0) e="RSMI_ONE_HOSTMEM=0" ;;
      mem1) e="RSMI_ONE_HOSTMEM=1" ;;
      mem2) e="RSMI_ONE_HOSTMEM=2" ;;
      g*) e="RSMI_LIB=$AB/librsmi_$v.so" ;;
    esac
    echo -n "$v: "
    env $e timeout -k 10 120 python -u scripts/dropin_trace.py 2>/dev/null | tail -1 || exit 1
  done
done
