#!/bin/bash
# Build A/B variants of librsmi.so (compile-time knobs) into udpspeeder_amd/ab/.
# Usage: bash scripts/build_ab.sh name "EXTRA flags" [name "flags" ...]
set -e
cd "$(dirname "$0")/../udpspeeder_amd/csrc"
mkdir -p ../ab
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  make -j8 EXTRA="$flags" OUT=../ab/librsmi_$name.so BUILD=../../build/ab_$name > /dev/null
  echo "built ab/librsmi_$name.so ($flags)"
done
