#!/bin/bash
# round-4: pipeline tests + host legs with ramp-up only (the new default)
# usage (on the box): bash tools/gpu_p22.sh TAG
set -o pipefail
T=${1:-p22}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step pytest pipeline + C++ API + queues
timeout -k 10 400 python -u -m pytest tests/test_gpu_pipeline.py tests/test_cpp_api.py tests/test_frame_queue.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 120 python bench.py --e2e > $O/e2e.json 2>> $O/err || { echo e2e failed; exit 1; }
  python -c "import json; d=json.load(open('$O/e2e.json')); print('e2e', d['value'])" | tee -a $O/host.txt
  timeout -k 10 200 python bench.py --c5 --records 65536 > $O/c5.json 2>> $O/err || { echo c5 failed; exit 1; }
  python -c "import json; d=json.load(open('$O/c5.json')); print('c5 share', d['value'])" | tee -a $O/host.txt
done
step bench default
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err; rc=$?; [ $rc -eq 0 ] || exit $rc
python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], json.dumps(d['host_resident']))"
step done
