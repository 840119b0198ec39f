#!/bin/bash
# Session-keyed wire frames (C3 shape, 1 M x 1 500 B): per-frame keys vs K session keys with HMAC
# midstates, interleaved.  usage: bash tools/sessions_ab.sh TAG PAIRS
set -euo pipefail
T=${1:-sessions}; N=${2:-3}
O=gpurun_out/$T
mkdir -p $O
: > $O/ab.jsonl
for i in $(seq 1 $N); do
  for k in 0 16384 1; do
    timeout -k 10 200 python bench.py --mode wire --records 1048576 --record-bytes 1500 --steps 50 --warmup 10 \
      --no-cpu-baseline --no-power --sessions $k > $O/one.json 2>> $O/ab.err
    python -c "import json; d=json.load(open('$O/one.json')); d['sessions']=$k; print(json.dumps(d))" >> $O/ab.jsonl
    python -c "import json; d=json.load(open('$O/one.json')); r=d['roofline']; print('sessions $k', d['value'], r['frac'], d.get('seal_ms'), d.get('open_ms'))"
  done
done
