#!/bin/bash
# round-4: host mode chosen by the HIP runtime in use (3 on the system runtime, 4 on another):
# pipeline tests, e2e probe both orders, bench default line, --c5 share.
# usage (on the box): bash tools/gpu_p19.sh TAG
set -o pipefail
T=${1:-p19}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step pytest pipeline + C++ API
timeout -k 10 400 python -u -m pytest tests/test_gpu_pipeline.py tests/test_cpp_api.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for o in torch_first lib_first; do
  timeout -k 10 120 python tools/e2e_probe.py $o > $O/x.json 2>> $O/probe.err || { echo probe failed; exit 1; }
  cat $O/x.json | tee -a $O/probe.jsonl
done
step bench default
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err; rc=$?; [ $rc -eq 0 ] || exit $rc
python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], json.dumps(d['host_resident']))"
step c5 share
timeout -k 10 200 python bench.py --c5 --records 65536 > $O/c5.json 2> $O/c5.err; rc=$?; cat $O/c5.json; [ $rc -eq 0 ] || exit $rc
step done
