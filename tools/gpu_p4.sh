#!/bin/bash
# round-4: host runtime after the combined gather/scatter pass and ramped chunks -- parity of the
# pipelines / batch API / queues, then C2 e2e + C5 host sweep and the batch API throughput.
set -o pipefail
T=${1:-p4}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step pytest
timeout -k 10 500 python -u -m pytest tests/test_gpu_pipeline.py tests/test_cpp_api.py tests/test_frame_queue.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
step host_sweep
SWEEP_MODES=split,splitk timeout -k 10 500 python -u tools/host_sweep.py all > $O/sweep.jsonl 2> $O/sweep.err; rc=$?; cat $O/sweep.jsonl; tail -3 $O/sweep.err; [ $rc -eq 0 ] || exit $rc
step batch_bench
: > $O/batch.jsonl
for cfg in "3 16 split" "3 32 split" "4 32 split" "3 16 splitk"; do
  set -- $cfg
  ENET_HOST_MODE=$3 ENET_HOST_THREADS=15 ENET_HOST_SLOTS=$1 ENET_HOST_CHUNK_MIB=$2 ENET_HOST_TRACE=1 timeout -k 10 300 tools/batch_bench all 3 > $O/x.jsonl 2> $O/trace_$1_$2_$3.err || { echo "batch $cfg failed"; tail -3 $O/trace_$1_$2_$3.err; exit 1; }
  sed "s/^{/{\"slots\":$1,\"chunk_mib\":$2,\"mode\":\"$3\",/" $O/x.jsonl >> $O/batch.jsonl
done
cat $O/batch.jsonl
step done
