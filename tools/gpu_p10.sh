#!/bin/bash
# round-4: parity after removing the streaming tail kernel; host-resident C2 with the HIP runtime
# of torch vs /opt/rocm (library loaded after / before torch).  usage (on the box): bash tools/gpu_p10.sh TAG
set -o pipefail
T=${1:-p10}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step pytest parity
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_parity.log 2>&1; rc=$?; tail -2 $O/pytest_parity.log; [ $rc -eq 0 ] || exit $rc
step e2e probe
for o in torch_first lib_first torch_first lib_first; do
  timeout -k 10 120 python tools/e2e_probe.py $o >> $O/e2e_probe.jsonl 2>> $O/e2e_probe.err || { echo probe failed; exit 1; }
  tail -1 $O/e2e_probe.jsonl
done
step c2 copy trace
ONE=splitk,4,32 timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -o c2 -- python3 tools/host_sweep.py c2one > $O/c2trace.json 2> $O/c2trace.err; rc=$?; cat $O/c2trace.json; [ $rc -eq 0 ] || exit $rc
python tools/copy_trace.py $O/trace/c2 > $O/c2trace_summary.jsonl; cat $O/c2trace_summary.jsonl
step done
