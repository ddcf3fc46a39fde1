#!/bin/bash
# Dev-only: build the codec library with extra -D flags into capnp-zig_amd/lib_exp/NAME.so
# usage: bash scripts/dev/build_variant.sh NAME "-DFOO -DBAR=1"
set -eu
cd "$(dirname "$0")/../../capnp-zig_amd"
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -I../include -Icsrc"
mkdir -p lib_exp
T=$(mktemp -d)
/opt/rocm/bin/hipcc $F $2 -c -o "$T/k.o" csrc/packed_kernels.hip
/opt/rocm/bin/hipcc $F $2 -c -o "$T/a.o" csrc/capnp_packed_abi.cpp
/opt/rocm/bin/hipcc $F -shared -o "lib_exp/$1.so" "$T/k.o" "$T/a.o"
rm -rf "$T"
