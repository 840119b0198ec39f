#!/bin/bash
# round-4: crypto::batch with merged arena copies and 32 MiB gather chunks; C++ API tests
# usage (on the box): bash tools/gpu_p15.sh TAG
set -o pipefail
T=${1:-p15}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step pytest C++ API + pipeline
timeout -k 10 400 python -u -m pytest tests/test_cpp_api.py tests/test_gpu_pipeline.py tests/test_frame_queue.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  step "batch_bench $i"
  timeout -k 10 300 tools/batch_bench all 3 >> $O/batch_bench.jsonl 2>> $O/batch_bench.err || { echo bb failed; exit 1; }
done
cat $O/batch_bench.jsonl
step done
