#!/bin/bash
# Build eval_check variants (generator env knobs) into risc0_amd/lib_variants/libr0hip_tune_<name>.so
#   bash tools/rehearsal/ec_variants.sh NAME "ENV=VAL ..." [NAME "ENV=..."]...
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p $ROOT/risc0_amd/lib_variants
while [ $# -ge 2 ]; do
  rm -rf $ROOT/risc0_amd/csrc/gen/rv32im
  env $2 make -C $ROOT/risc0_amd/csrc -j8 > /dev/null
  cp $ROOT/risc0_amd/lib/libr0hip.so $ROOT/risc0_amd/lib_variants/libr0hip_tune_$1.so
  echo built $1
  shift 2
done
rm -rf $ROOT/risc0_amd/csrc/gen/rv32im
make -C $ROOT/risc0_amd/csrc -j8 > /dev/null
