#!/usr/bin/env bash
# register / LDS / spill summary of the kernels in a built object (dev tool):
#   tools/kregs.sh starch_amd/_build/bz2_bwt3.o [name-regex]
set -e
T=$(mktemp -d)
/opt/rocm/lib/llvm/bin/llvm-objcopy --dump-section=.hip_fatbin=$T/fat.bin "$1"
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input=$T/fat.bin \
  --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$T/k.co
/opt/rocm/lib/llvm/bin/llvm-readelf --notes $T/k.co | python3 -c '
import sys, re
txt = sys.stdin.read()
pat = re.compile(sys.argv[1] if len(sys.argv) > 1 else ".")
for blk in txt.split("- .agpr_count")[1:]:
    g = lambda k: (re.search(r"\.%s:\s+(\S+)" % k, blk) or [None, "?"])[1]
    name = g("name")
    if not pat.search(name): continue
    print("%-5s vgpr %4s agpr %3s sgpr %3s spill %3s lds %6s  %s" % ("", g("vgpr_count"), (re.match(r"\s*:\s*(\d+)", blk) or [None,"?"])[1], g("sgpr_count"), g("vgpr_spill_count"), g("group_segment_fixed_size"), name[:110]))
' "${2:-.}"
rm -rf $T
