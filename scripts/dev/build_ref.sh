#!/bin/bash
# Dev-only: build libcapnp_packed.so from the kernel source at git ref REF into
# capnp-zig_amd/lib_exp/NAME.so (same-box A/B timings with CPK_LIB=...).
# usage: scripts/dev/build_ref.sh REF NAME
set -euo pipefail
cd "$(dirname "$0")/../../capnp-zig_amd"
ref=$1; name=$2
tmp=$(mktemp -d)
git show "$ref:capnp-zig_amd/csrc/packed_kernels.hip" > $tmp/packed_kernels.hip
cp csrc/kernels.h $tmp/
HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result"
mkdir -p lib_exp
/opt/rocm/bin/hipcc $HIPFLAGS -I../include -I$tmp -c -o $tmp/k.o $tmp/packed_kernels.hip
/opt/rocm/bin/hipcc $HIPFLAGS -I../include -Icsrc -c -o $tmp/a.o csrc/capnp_packed_abi.cpp
/opt/rocm/bin/hipcc $HIPFLAGS -shared -o lib_exp/$name.so $tmp/k.o $tmp/a.o
rm -rf $tmp
echo built lib_exp/$name.so
