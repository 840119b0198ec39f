#!/bin/bash
# Duplex workgroup size (ENET_DUPLEX_RPW: 64 vs 256 records per workgroup) for wire frames at C3 and
# C2 shapes and chunk store at C2, interleaved repetitions.  usage (on the box): bash tools/dx_rpw_ab.sh reps
set -uo pipefail
export TMPDIR=/tmp
for rep in $(seq ${1:-2}); do
  for args in "--mode wire --records 1048576 --record-bytes 1500" "--mode wire" "--mode store"; do
    for r in 256 64; do
      ENET_DUPLEX_RPW=$r timeout -k 10 180 python bench.py $args --steps 20 --warmup 3 --no-cpu-baseline --no-power | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('rpw=$r', '$args', d['value'])" || exit 1
    done
  done
done
