#!/bin/bash
# Dev: GPU tests against lib_exp/NAME.so (CPK_LIB), then the C5/headline A/B vs the shipped library.
# usage: bash scripts/dev/test_variant.sh NAME TAG pytest-args...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
name=$1; OUT=gpurun_out/$2; shift 2
mkdir -p "$OUT"
CPK_LIB=capnp-zig_amd/lib_exp/$name.so timeout -k 10 600 python3 -u -m pytest "$@" -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 "$OUT/pytest.log"
[ $rc -ne 0 ] && exit $rc
bash scripts/dev/ab_c5.sh $name
