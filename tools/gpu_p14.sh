#!/bin/bash
# round-4: crypto::batch C3 wire frames from std::vector records: worker threads x chunk size
# usage (on the box): bash tools/gpu_p14.sh TAG
set -o pipefail
T=${1:-p14}
O=gpurun_out/$T
mkdir -p $O
step() { echo "[$(date +%T)] $*"; }
for th in 8 12 15; do
  for ch in 16 32; do
    step "threads $th chunk $ch"
    ENET_HOST_THREADS=$th ENET_HOST_CHUNK_MIB=$ch timeout -k 10 200 tools/batch_bench c3 3 > $O/x.jsonl 2>> $O/bb.err || { echo bb failed; exit 1; }
    grep packed $O/x.jsonl | python -c "import sys, json; d=json.loads(sys.stdin.read()); d['threads']=$th; d['chunk_mib']=$ch; print(json.dumps(d))" | tee -a $O/bb.jsonl
  done
done
ENET_HOST_TRACE=1 timeout -k 10 200 tools/batch_bench c3 1 > $O/x.jsonl 2> $O/trace.err || { echo bb failed; exit 1; }
grep "enet host" $O/trace.err | tail -4
step done
