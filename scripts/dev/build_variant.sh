#!/bin/bash
# Dev-only: build libcapnp_packed.so with extra -D flags into capnp-zig_amd/lib_exp/NAME.so
# (selected at run time with CPK_LIB=...; never the shipped library).
# usage: scripts/dev/build_variant.sh NAME "-DFOO=1 -DBAR=2"
set -euo pipefail
cd "$(dirname "$0")/../../capnp-zig_amd"
name=$1; defs=${2:-}
mkdir -p lib_exp/$name
HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result"
/opt/rocm/bin/hipcc $HIPFLAGS -I../include -Icsrc $defs -c -o lib_exp/$name/k.o csrc/packed_kernels.hip
/opt/rocm/bin/hipcc $HIPFLAGS -I../include -Icsrc $defs -c -o lib_exp/$name/a.o csrc/capnp_packed_abi.cpp
/opt/rocm/bin/hipcc $HIPFLAGS -shared -o lib_exp/$name.so lib_exp/$name/k.o lib_exp/$name/a.o
rm -rf lib_exp/$name
echo built lib_exp/$name.so
