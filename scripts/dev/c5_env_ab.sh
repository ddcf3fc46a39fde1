#!/bin/bash
# Dev A/B: the C5 leg under environment combinations (one per argument, e.g. "CPK_DECODE=fused
# CPK_SM_FRAC=0.75"), alternating, twice; CPK_LIB may name a lib_exp build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/c5env
mkdir -p $O
for r in 1 2; do
  for combo in "$@"; do
    env $combo timeout -k 10 180 python3 bench.py --only c5 --steps 20 --warmup 3 > $O/c5.json 2>$O/c5.err || { tail -5 $O/c5.err; exit 1; }
    echo "c5 [$combo] $(python3 -c "import json;d=json.load(open('$O/c5.json'))['c5'];print(d['encode_ms'],d['decode_ms'],d['GiB_s'],d['bit_exact_roundtrip'])")"
    if [ -n "${HEAD:-}" ]; then  # the headline encode / decode microbench too
      env $combo timeout -k 10 120 python3 scripts/microbench.py --reps 9 --only ${HEAD} > $O/x.json 2>&1 || { cat $O/x.json; exit 1; }
      echo "head [$combo] $(tail -1 $O/x.json)"
    fi
  done
done
