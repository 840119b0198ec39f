#!/bin/bash
# round-4 host-path session: GPU tests of the host-memory runtime, PCIe / zero-copy probe, C++
# batch API throughput, queue throughput.  usage (on the box): bash tools/gpu_p1.sh TAG
set -o pipefail
T=${1:-p1}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step pytest
timeout -k 10 400 python -u -m pytest tests/test_cpp_api.py tests/test_gpu_pipeline.py tests/test_frame_queue.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -15 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
step probe
timeout -k 10 360 tools/host_path_probe 65536 4096 all > $O/probe.jsonl 2> $O/probe.err; rc=$?; cat $O/probe.jsonl; tail -3 $O/probe.err; [ $rc -eq 0 ] || exit $rc
step batch_bench
timeout -k 10 300 tools/batch_bench all 3 > $O/batch.jsonl 2> $O/batch.err; rc=$?; cat $O/batch.jsonl; tail -3 $O/batch.err; [ $rc -eq 0 ] || exit $rc
step queue_bench
: > $O/queue.jsonl
for args in "device sync 16" "device sync 256" "device async 16 256" "auto sync 16" "auto sync 256" "host async 16 256"; do
  timeout -k 10 60 tools/queue_bench $args >> $O/queue.jsonl 2>> $O/queue.err || { echo "queue_bench $args failed"; exit 1; }
done
cat $O/queue.jsonl
step done
