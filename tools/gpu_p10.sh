#!/bin/bash
# round-4: host runtime creating only the streams a job needs; the e2e rate under torch's HIP
# runtime (bench.py) vs the library's own (library loaded first), a C2 copy trace, parity.
# usage (on the box): bash tools/gpu_p10.sh TAG
set -o pipefail
T=${1:-p10}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step pytest pipeline + parity subset
timeout -k 10 400 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_parity.py tests/test_cpp_api.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
step e2e probe
for o in torch_first lib_first; do
  timeout -k 10 120 python tools/e2e_probe.py $o >> $O/e2e_probe.jsonl 2>> $O/e2e_probe.err || { echo probe failed; exit 1; }
  tail -1 $O/e2e_probe.jsonl
done
step bench e2e / c5
timeout -k 10 120 python bench.py --e2e > $O/e2e.json 2>> $O/e2e.err || { echo e2e failed; exit 1; }
cat $O/e2e.json
timeout -k 10 200 python bench.py --c5 > $O/c5.json 2>> $O/c5.err || { echo c5 failed; exit 1; }
cat $O/c5.json
step bench default
timeout -k 10 240 python bench.py > $O/bench.json 2> $O/bench.err; rc=$?; cat $O/bench.json; [ $rc -eq 0 ] || exit $rc
step c2 copy trace
ONE=splitk,4,32 timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -o c2 -- python3 tools/host_sweep.py c2one > $O/c2trace.json 2> $O/c2trace.err; rc=$?; cat $O/c2trace.json; [ $rc -eq 0 ] || exit $rc
python tools/copy_trace.py $O/trace/c2 > $O/c2trace_summary.jsonl; cat $O/c2trace_summary.jsonl
step done
