#!/bin/bash
# Streaming kernel (stream.hip) vs the round-1 lockstep staging (ENET_STREAM=0): GPU parity
# suite, then C2 / C4 / xor-pass A/B on the same box.
# usage (on the box, from the repo root): bash tools/stream_ab.sh [tag]
set -euo pipefail
T=${1:-ab}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 120 python bench.py --steps 300 --warmup 30 --no-cpu-baseline > $O/c2_$tag.json 2>/dev/null
  env "$@" timeout -k 10 120 python bench.py --records 32768 --record-bytes 65536 --steps 20 --warmup 5 --no-cpu-baseline > $O/c4_$tag.json 2>/dev/null
  env "$@" timeout -k 10 120 python bench.py --mode xor --steps 300 --warmup 30 --no-cpu-baseline > $O/xor_$tag.json 2>/dev/null
  python3 -c "
import json
for c in ('c2','c4','xor'):
    d=json.load(open('$O/'+c+'_$tag.json')); print('$tag', c, d['value'], d.get('seal_ms'), d.get('open_ms'))"
}
run stream ENET_STREAM=1
run lock ENET_STREAM=0
run stream2 ENET_STREAM=1
