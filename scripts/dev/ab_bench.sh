#!/bin/bash
# Dev-only same-box A/B of the bench step itself (encode then decode, headline only) for
# lib_exp/{NAME…}.so and the shipped library, alternating, $REPS rounds (default 2).
# usage: bash scripts/dev/ab_bench.sh NAME...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/ab; mkdir -p $O
libs=(); for n in "$@"; do libs+=("capnp-zig_amd/lib_exp/$n.so"); done; libs+=("capnp-zig_amd/lib/libcapnp_packed.so")
for r in $(seq ${REPS:-2}); do
  for lib in "${libs[@]}"; do
    CPK_LIB=$lib timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-host-path --no-read-message \
        --no-skewed --no-sweep --no-dense --no-c1 --no-validate > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
    echo "$(basename $lib) $(python3 -c "import json;d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]);print(d['value'],d['encode_ms'],d['decode_ms'],d['bit_exact_roundtrip'])")"
  done
done
