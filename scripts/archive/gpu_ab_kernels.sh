#!/bin/bash
# GPU box: per-kernel times of A/B library builds (scripts/build_ab.sh) under
# rocprofv3 --kernel-trace --stats, variants alternated to spread box drift.
#   bash scripts/gpu_ab_kernels.sh OUT ROUNDS SCRIPT VARIANT [VARIANT ...]
# VARIANT "main" is udpspeeder_amd/librsmi.so, anything else ab/librsmi_<v>.so.
# Per run: gpurun_out/OUT/<variant>_<round>.txt (name / calls / average ns).
set -o pipefail
R=$PWD
O=$R/gpurun_out/$1
ROUNDS=$2
SCRIPT=$3
shift 3
mkdir -p $O
for r in $(seq 1 $ROUNDS); do
  for v in "$@"; do
    lib=$R/udpspeeder_amd/librsmi.so
    [ "$v" != main ] && lib=$R/udpspeeder_amd/ab/librsmi_$v.so
    (cd /tmp && export TMPDIR=/tmp && RSMI_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats \
        --output-format csv -d $O/p_${v}_$r -o run -- python3 $R/$SCRIPT > $O/${v}_$r.log 2>&1) || { tail $O/${v}_$r.log; exit 1; }
    python scripts/kstats.py $O/p_${v}_$r/run_kernel_stats.csv > $O/${v}_$r.txt
    rm -rf $O/p_${v}_$r
    echo "== $v round $r"; grep -E "${KPAT:-decode|bs_ragged}" $O/${v}_$r.txt; grep -h "ms" $O/${v}_$r.log | tail -2 | cut -c1-200
  done
done
