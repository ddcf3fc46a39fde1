#!/bin/bash
# Dev-only: rebuild every lib_exp variant the round-4 A/B scripts use from the current source
# (ix_flat: the index pass with FLAT prefetch loads, from the commit before that change).
# dev_decoders carries the fused and streaming mid-unit decoders (CPK_DEV_DECODERS=1).
set -euo pipefail
cd "$(dirname "$0")/../.."
D="-DCPK_DEV_DECODERS=1"
bash scripts/dev/build_variant.sh dev_decoders "$D"
bash scripts/dev/build_variant.sh ds_k32 "$D -DCPK_DS_K=32"
bash scripts/dev/build_variant.sh ds_tst "$D -DCPK_DS_TSTORE=1"
