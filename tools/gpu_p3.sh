#!/bin/bash
# round-4 host pipeline tuning sweep: tools/host_sweep.py (C2 e2e, C5 host per-GPU share) and the
# C++ batch API's packed path with the runtime's per-job time breakdown (ENET_HOST_TRACE=1).
# usage (on the box): bash tools/gpu_p3.sh TAG
set -o pipefail
T=${1:-p3}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step host_sweep
timeout -k 10 500 python -u tools/host_sweep.py all > $O/sweep.jsonl 2> $O/sweep.err; rc=$?; cat $O/sweep.jsonl; tail -3 $O/sweep.err; [ $rc -eq 0 ] || exit $rc
step batch_bench
: > $O/batch.jsonl
for cfg in "3 16" "4 16" "6 16" "4 8" "4 32" "6 8"; do
  set -- $cfg
  ENET_HOST_MODE=split ENET_HOST_THREADS=15 ENET_HOST_SLOTS=$1 ENET_HOST_CHUNK_MIB=$2 ENET_HOST_TRACE=1 timeout -k 10 300 tools/batch_bench all 2 > $O/x.jsonl 2> $O/trace_$1_$2.err || { echo "batch $cfg failed"; tail -3 $O/trace_$1_$2.err; exit 1; }
  grep packed $O/x.jsonl | sed "s/^{/{\"slots\":$1,\"chunk_mib\":$2,/" >> $O/batch.jsonl
done
cat $O/batch.jsonl
step done
