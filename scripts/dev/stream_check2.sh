#!/bin/bash
# Dev-only, second half of the round-4 checks: the fused framing leg, the streaming small-unit
# encoder (lib_exp/es_stream.so) tests and C5 timings, then the decoder build-variant A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/stream
mkdir -p $O
step() {  # name, then the command; stops the script on a crash / time limit
  local name=$1; shift
  "$@"; local rc=$?
  echo "[$name] rc=$rc"
  if [ $rc -ge 124 ]; then exit $rc; fi
  return 0
}
step framing timeout -k 10 300 python3 bench.py --only framing > $O/framing.json 2>&1
tail -1 $O/framing.json
# the prefetching one-tile message encode (lib_exp/em_pf.so: -DCPK_EM_PF=1): its tests, then A/B
step em_tests env CPK_LIB=capnp-zig_amd/lib_exp/em_pf.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_configs.py \
  -x -q --timeout 200 --timeout-method thread -k "encode_message" > $O/pytest_em.log 2>&1
tail -3 $O/pytest_em.log
for lib in capnp-zig_amd/lib_exp/em_pf.so capnp-zig_amd/lib/libcapnp_packed.so capnp-zig_amd/lib_exp/em_pf.so; do
  step framing_ab env CPK_LIB=$lib timeout -k 10 300 python3 bench.py --only framing > $O/framing_ab.json 2>&1
  echo "framing lib=$(basename $lib) $(tail -1 $O/framing_ab.json)"
done
# the streaming small-unit encoder (lib_exp/es_stream.so: -DCPK_ES_STREAM=1): encode tests, C5 timings
step es_tests env CPK_LIB=capnp-zig_amd/lib_exp/es_stream.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_small_units.py \
  tests/test_gpu_configs.py tests/test_gpu_stress.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
  -k "encode or c5 or small" > $O/pytest_es.log 2>&1
tail -3 $O/pytest_es.log
for lib in capnp-zig_amd/lib_exp/es_stream.so capnp-zig_amd/lib/libcapnp_packed.so capnp-zig_amd/lib_exp/es_stream.so capnp-zig_amd/lib/libcapnp_packed.so; do
  step c5es env CPK_LIB=$lib timeout -k 10 200 python3 bench.py --only c5 --decoder stream > $O/c5es.json 2>&1
  echo "c5 lib=$(basename $lib) $(tail -1 $O/c5es.json)"
done
step ds_ab bash scripts/dev/ds_ab.sh
