#!/bin/bash
# Session-frame throughput: SessionManager::send / receive as written (per call,
# on every session thread) on the reference library and on the drop-in, and through the shared
# FrameQueue / FrameReceiveQueue (policy device / auto / host), 16 and 256 session threads.
# usage (on the box, from the repo root): bash tools/queue_bench.sh TAG
set -euo pipefail
T=${1:-queue}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_frame_queue.py -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for pol in device auto host; do
  timeout -k 10 300 oracle/_ref/scalar_latency_gpu 50 $pol 16 256 > $O/latency_$pol.jsonl 2> $O/latency_$pol.err
  grep frame $O/latency_$pol.jsonl | sed "s/^/$pol /"
done
timeout -k 10 300 oracle/_ref/scalar_latency_ref 50 x 16 256 > $O/latency_ref.jsonl 2> $O/latency_ref.err
grep frame $O/latency_ref.jsonl | sed "s/^/ref /"
