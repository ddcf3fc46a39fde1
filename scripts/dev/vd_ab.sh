#!/bin/bash
# Dev A/B: the validate leg (bench.py --only validate) for lib_exp builds and the shipped library.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/vd
mkdir -p $O
for r in 1 2; do
  for lib in "$@" capnp-zig_amd/lib/libcapnp_packed.so; do
    CPK_LIB=$lib timeout -k 10 300 python3 bench.py --only validate > $O/v.json 2>$O/v.err || { tail -5 $O/v.err; exit 1; }
    echo "validate lib=$(basename $lib) $(python3 -c "import json;d=json.load(open('$O/v.json'))['validate'];t=d['trees'];print(t['ms'],t['frac'],t['all_valid'],d['c1']['ms'])")"
  done
done
