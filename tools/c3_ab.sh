#!/bin/bash
# C3 (1 M x 1 500 B) AEAD: line staging in 256-thread workgroups (COOP 4, default) vs 512-thread
# lockstep workgroups (COOP 6, ENET_LINES_LOCKSTEP=1), interleaved.  usage: bash tools/c3_ab.sh TAG [reps]
set -euo pipefail
O=gpurun_out/${1:-c3ab}
mkdir -p $O
export TMPDIR=/tmp
for r in $(seq ${2:-2}); do for ll in 0 1; do
  ENET_LINES_LOCKSTEP=$ll timeout -k 10 200 python bench.py --no-cpu-baseline --no-power --records 1048576 --record-bytes 1500 --steps 30 --warmup 5 > $O/l${ll}_$r.json 2>> $O/err.log
  python3 -c "import json;d=json.load(open('$O/l${ll}_$r.json'));print('lines_lockstep $ll rep $r', d['value'], d['seal_ms'], d['open_ms'])"
done; done
