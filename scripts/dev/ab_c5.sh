#!/bin/bash
# Dev-only same-box A/B: the C5 skewed leg (bench.py --only c5) and the headline
# encode/decode microbench, for lib_exp/NAME.so and the shipped library, alternating.
# usage (on the GPU box): bash scripts/dev/ab_c5.sh NAME [NAME2 ...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/ab
mkdir -p $O
libs=""
for b in "$@"; do libs="$libs capnp-zig_amd/lib_exp/$b.so"; done
libs="$libs capnp-zig_amd/lib/libcapnp_packed.so"
for r in 1 2; do
  for lib in $libs; do
    CPK_LIB=$lib timeout -k 10 180 python3 bench.py --only c5 --steps 20 --warmup 3 > $O/c5.json 2>$O/c5.err || { tail -5 $O/c5.err; exit 1; }
    echo "c5 lib=$(basename $lib) $(python3 -c "import json;d=json.load(open('$O/c5.json'))['c5'];print(d['encode_ms'],d['decode_ms'],d['GiB_s'],d['bit_exact_roundtrip'])")"
    if [ -z "${NOHEAD:-}" ]; then
      CPK_LIB=$lib timeout -k 10 120 python3 scripts/microbench.py --reps 9 --only encode,decode > $O/x.json 2>&1 || { cat $O/x.json; exit 1; }
      echo "head lib=$(basename $lib) $(tail -1 $O/x.json)"
    fi
  done
done
