#!/bin/bash
# round-4: per-record outputs written zero-copy into the pinned small block (no small D2H per
# chunk): pipeline / C++ API tests, host legs, C2 copy trace, batch_bench.
# usage (on the box): bash tools/gpu_p13.sh TAG
set -o pipefail
T=${1:-p13}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step pytest pipeline + C++ API + queues
timeout -k 10 400 python -u -m pytest tests/test_gpu_pipeline.py tests/test_cpp_api.py tests/test_frame_queue.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
step e2e x2 / c5 x2
for i in 1 2; do
timeout -k 10 120 python bench.py --e2e > $O/e2e.json 2>> $O/e2e.err || { echo e2e failed; exit 1; }
cat $O/e2e.json >> $O/e2e.jsonl; python -c "import json; d=json.load(open('$O/e2e.json')); print('e2e', d['value'], d['seal_GiBs'], d['open_GiBs'])"
timeout -k 10 200 python bench.py --c5 --records 65536 > $O/c5.json 2>> $O/c5.err || { echo c5 failed; exit 1; }
cat $O/c5.json >> $O/c5.jsonl; python -c "import json; d=json.load(open('$O/c5.json')); print('c5', d['value'])"
done
step c2 copy trace
ONE=splitk,4,32 timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -o c2 -- python3 tools/host_sweep.py c2one > $O/c2trace.json 2> $O/c2trace.err; rc=$?; cat $O/c2trace.json; [ $rc -eq 0 ] || exit $rc
step batch_bench
timeout -k 10 300 tools/batch_bench all 3 > $O/batch_bench.jsonl 2> $O/batch_bench.err; rc=$?; cat $O/batch_bench.jsonl; [ $rc -eq 0 ] || exit $rc
step done
