#!/bin/bash
# C3 (1 M x 1 500 B AEAD): line staging with (ENET_LINES_LOCKSTEP=1, COOP 6) and without the lockstep
# keystream, interleaved repetitions.  usage (on the box): bash tools/c3_lock_ab.sh reps
set -uo pipefail
export TMPDIR=/tmp
for rep in $(seq ${1:-2}); do
  for v in 0 1; do
    ENET_LINES_LOCKSTEP=$v timeout -k 10 180 python bench.py --records 1048576 --record-bytes 1500 --steps 20 --warmup 3 --no-cpu-baseline --no-power | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('lines_lockstep=$v rep=$rep', d['value'], d['seal_ms'], d['open_ms'])" || exit 1
  done
done
