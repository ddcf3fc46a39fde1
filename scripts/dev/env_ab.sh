#!/bin/bash
# DEV (round 6): A/B of an environment switch on the words decoder (dec_ab.py, one process per run)
# usage: bash scripts/dev/env_ab.sh VAR [reps]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
VAR=$1; REPS=${2:-2}
for r in $(seq 1 $REPS); do
  for v in off on; do
    echo "$VAR=$v"
    if [ $v = on ]; then export $VAR=1; else unset $VAR; fi
    timeout -k 10 120 python3 scripts/dev/dec_ab.py --decoders words --reps 5 2>&1 | tail -1
  done
done
