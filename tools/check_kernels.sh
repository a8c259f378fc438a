#!/bin/bash
# check_kernels.sh OBJ -- every kernel the host half of a hipcc object
# registers must exist in its gfx950 code object.  The two halves are
# compiled by separate passes; a header edited while one of them runs leaves a
# host stub whose kernel is missing, and launching it aborts the process on
# the GPU (seen in round 5: pair_kernel<24, false, 2>).  Used by
# libssa_amd/Makefile after each .hip compile.
set -euo pipefail
obj=$1
arch=${ARCH:-gfx950}
llvm=/opt/rocm/lib/llvm/bin
tmp=$(mktemp -d)
trap 'rm -rf "$tmp"' EXIT
objcopy --dump-section .hip_fatbin="$tmp/fatbin" "$obj"
"$llvm/clang-offload-bundler" --unbundle --type=o --input="$tmp/fatbin" \
    --targets="hipv4-amdgcn-amd-amdhsa--$arch" --output="$tmp/co"
"$llvm/llvm-readelf" -s --wide "$tmp/co" | awk '{print $8}' | sed 's/\.kd$//' | sort -u > "$tmp/dev"
# the registration strings (__hipRegisterFunction / __hipRegisterVar device names)
objcopy --dump-section .rodata.str1.1="$tmp/str" "$obj"
tr '\0' '\n' < "$tmp/str" | grep '^_Z' | sort -u > "$tmp/host" || true
missing=$(comm -23 "$tmp/host" "$tmp/dev")
if [ -n "$missing" ]; then
    echo "check_kernels: $obj registers kernels its $arch code object lacks:" >&2
    echo "$missing" | c++filt >&2
    exit 1
fi
