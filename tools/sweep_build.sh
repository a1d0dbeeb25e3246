#!/usr/bin/env bash
# Build library variants for a GPU sweep: tools/sweep_build.sh name "-DFLAG=.." [name "-D.."]...
# -> starch_amd/_sweep/<name>/libstarch_amd.so (select with STARCH_AMD_LIB=...)
set -e
cd "$(dirname "$0")/.."
while [ $# -ge 2 ]; do
  make -s -j8 BUILD=starch_amd/_sweep/$1 EXTRA="$2" starch_amd/_sweep/$1/libstarch_amd.so
  rm -f starch_amd/_sweep/$1/*.o
  shift 2
done
ls starch_amd/_sweep
