#!/bin/bash
# round-4: frame-queue device passes through zero-copy engines (default) vs SDMA modes
# usage (on the box): bash tools/gpu_p20.sh TAG
set -o pipefail
T=${1:-p20}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step pytest queues + C++ API
timeout -k 10 400 python -u -m pytest tests/test_frame_queue.py tests/test_cpp_api.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for qm in 0 1 3; do
  for args in "device sync 16 1 3" "device sync 256 1 3" "device async 16 256 3"; do
    step "mode $qm: $args"
    ENET_QUEUE_HOST_MODE=$qm timeout -k 10 120 tools/queue_bench $args > $O/x.json 2>> $O/qb.err || { echo qb failed; exit 1; }
    python -c "import json; d=json.loads(open('$O/x.json').read().strip().splitlines()[-1]); d['queue_host_mode']=$qm; print(json.dumps(d))" | tee -a $O/qb.jsonl
  done
done
step done
