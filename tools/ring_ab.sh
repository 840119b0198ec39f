#!/bin/bash
# C3-class output-ring streaming kernel: focused parity tests, then C3 AEAD with the ring kernel
# against the line-staging records kernel (ENET_STREAM_RING=0), interleaved.
# usage (on the box, from the repo root): bash tools/ring_ab.sh TAG [pairs]
set -euo pipefail
T=${1:-ring}
N=${2:-2}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step pytest
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "uniform_batches or uniform_aad or lying_hints or full_size or out_arena_phase or ring" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
: > $O/c3.jsonl
for i in $(seq 1 $N); do
  for r in 1 0; do
    step "C3 ring=$r"
    ENET_STREAM_RING=$r timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-power --records 1048576 --record-bytes 1500 >> $O/c3.jsonl 2>> $O/c3.err
    tail -1 $O/c3.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('ring', $r, d['value'], d.get('roofline',{}).get('frac'))"
  done
done
step done
