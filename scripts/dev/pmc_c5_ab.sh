#!/bin/bash
# Dev-only: C5 HBM traffic (FETCH_SIZE / WRITE_SIZE passes, kernel trace only) and C5 timings,
# shipped library against lib_exp/${ESLIB:-es_old}.so (the streaming small-unit encoder, CPK_ES_STREAM=1,
# from the commit before its removal). Usage: bash scripts/dev/pmc_c5_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/pmc_c5_ab
mkdir -p $O
for name in ship ${ESLIB:-es_old}; do
  lib=capnp-zig_amd/lib/libcapnp_packed.so
  [ $name != ship ] && lib=capnp-zig_amd/lib_exp/${ESLIB:-es_old}.so
  mkdir -p $O/$name
  for c in FETCH_SIZE WRITE_SIZE; do
    CPK_LIB=$lib timeout -k 10 240 rocprofv3 --pmc $c --output-format csv -d "$O/$name/$c" -o run -- \
        python3 bench.py --only c5 --steps 2 --warmup 1 > "$O/$name/$c.log" 2>&1
    rc=$?; echo "$name $c rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
done
for r in 1 2; do
  for name in ship ${ESLIB:-es_old}; do
    lib=capnp-zig_amd/lib/libcapnp_packed.so
    [ $name != ship ] && lib=capnp-zig_amd/lib_exp/${ESLIB:-es_old}.so
    CPK_LIB=$lib timeout -k 10 200 python3 bench.py --only c5 > $O/c5.json 2>&1
    rc=$?; [ $rc -ne 0 ] && { tail -3 $O/c5.json; exit $rc; }
    echo "$name $(grep '^{' $O/c5.json | tail -1 | cut -c1-330)"
  done
done
