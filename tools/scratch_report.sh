#!/bin/bash
# Scratch (private segment) and VGPRs of every kernel in a built object or library:
#   bash tools/scratch_report.sh rustnetworkstack_amd/build/rns_checksum.o [only-nonzero]
# (the gfx950 code object is unbundled from the .hip_fatbin section and its AMDGPU
# metadata notes read with llvm-readelf; names demangled).
set -eu
OBJ=$1; ONLY=${2:-}
T=$(mktemp -d); trap 'rm -rf "$T"' EXIT
LLVM=/opt/rocm/lib/llvm/bin
$LLVM/llvm-objcopy --dump-section=.hip_fatbin="$T/fat.bin" "$OBJ" "$T/dummy.o"
$LLVM/clang-offload-bundler --unbundle --type=o --input="$T/fat.bin" --targets=hipv4-amdgcn-amd-amdhsa--gfx950 \
    --output="$T/k.co"
$LLVM/llvm-readelf --notes "$T/k.co" | awk '
  /^ *- \.agpr_count:/ { if (name != "") emit(); name=""; scr=""; vg="" }
  /^ *\.name: / { name=$2 }
  /\.private_segment_fixed_size:/ { scr=$2 }
  /^ *\.vgpr_count:/ { vg=$2 }
  function emit() { print scr "\t" vg "\t" name }
  END { if (name != "") emit() }' | sort -k3 | c++filt | sed 's/(anonymous namespace):://' |
  { if [ -n "$ONLY" ]; then awk -F'\t' '$1 != 0'; else cat; fi; } |
  awk -F'\t' 'BEGIN { print "scratch_B_per_lane\tvgprs\tkernel" } { print }'
