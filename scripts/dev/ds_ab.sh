#!/bin/bash
# Dev-only same-box A/B of decode_stream_kernel build variants (lib_exp/$V.so for V in $VARS,
# all dev builds: the shipped library has no streaming decoder)
# against the shipped library, all with the streaming decoder: decode at p = 0.5 / 0.1 / 0.9.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/ds_ab
mkdir -p $O
for t in ${THRS:-128 26 230}; do
  for r in 1 2; do
    for lib in capnp-zig_amd/lib_exp/dev_decoders.so $(for v in ${VARS:-ds_k32 ds_tst}; do echo capnp-zig_amd/lib_exp/$v.so; done); do
      CPK_LIB=$lib timeout -k 10 120 python3 scripts/microbench.py --reps 9 --zero-thresh $t --only decode --decoder stream > $O/x.json 2>&1
      rc=$?; [ $rc -ge 124 ] && exit $rc
      echo "t=$t lib=$(basename $lib) $(tail -1 $O/x.json)"
    done
  done
done
# the two-pass decoder: index pass with FLAT prefetch loads (lib_exp/ix_flat.so, the previous
# commit) against global asm loads (shipped)
for t in ${THRS:-128 26 230}; do
  for r in 1 2; do
    for lib in capnp-zig_amd/lib/libcapnp_packed.so capnp-zig_amd/lib_exp/ix_flat.so; do
      CPK_LIB=$lib timeout -k 10 120 python3 scripts/microbench.py --reps 9 --zero-thresh $t --only decode,decoded_size --decoder twopass > $O/x.json 2>&1
      rc=$?; [ $rc -ge 124 ] && exit $rc
      echo "twopass t=$t lib=$(basename $lib) $(tail -1 $O/x.json)"
    done
  done
done
