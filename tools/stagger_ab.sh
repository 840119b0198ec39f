#!/bin/bash
# A/B of stream-kernel code variants (ENET_STREAM_VAR) at C2 in the bench's alternation, interleaved
# repetitions on one box.  usage (on the box): bash tools/stagger_ab.sh "0 1 2" reps [aead|xor]
set -uo pipefail
export TMPDIR=/tmp
VS=${1:-0 1 2}; R=${2:-2}; M=${3:-aead}
O=gpurun_out/stagger; mkdir -p $O
for rep in $(seq $R); do
  for v in $VS; do
    ENET_STREAM_VAR=$v timeout -k 10 120 python bench.py --mode $M --steps 200 --warmup 20 --no-cpu-baseline > $O/v${v}_$rep.json 2>$O/v${v}_$rep.err || { echo "var $v failed"; tail -5 $O/v${v}_$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/v${v}_$rep.json'));print('var=$v rep=$rep', d['value'], d.get('seal_ms'), d.get('open_ms'))"
  done
done
