#!/bin/bash
# Dev-only: rebuild every lib_exp variant the round-4 A/B scripts use from the current source
# (ix_flat: the index pass with FLAT prefetch loads, from the commit before that change).
set -euo pipefail
cd "$(dirname "$0")/../.."
bash scripts/dev/build_variant.sh ds_k32 "-DCPK_DS_K=32"
bash scripts/dev/build_variant.sh ds_w1 "-DCPK_DS_WAVES=1"
bash scripts/dev/build_variant.sh ds_w2 "-DCPK_DS_WAVES=2"
bash scripts/dev/build_variant.sh ds_tst "-DCPK_DS_TSTORE=1"
