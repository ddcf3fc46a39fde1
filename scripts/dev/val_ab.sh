#!/bin/bash
# DEV (round 6): A/B of VAR=v1,v2,... on the words decoder (dec_ab.py, one process per run)
# usage: bash scripts/dev/val_ab.sh VAR "0 1 2" [reps]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
VAR=$1; VALS=$2; REPS=${3:-2}
for r in $(seq 1 $REPS); do
  for v in $VALS; do
    echo "$VAR=$v"
    env $VAR=$v timeout -k 10 120 python3 scripts/dev/dec_ab.py --decoders words --reps 5 2>&1 | tail -1
  done
done
