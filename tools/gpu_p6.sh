#!/bin/bash
# round-4: host runtime with a dedicated kernel stream (SdmaSplitK) -- pipeline parity, C2 / C5
# sweep, C5 timeline.  usage (on the box): bash tools/gpu_p6.sh TAG
set -o pipefail
T=${1:-p6}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step pytest
timeout -k 10 500 python -u -m pytest tests/test_gpu_pipeline.py tests/test_cpp_api.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
step host_sweep
SWEEP_MODES=splitk timeout -k 10 500 python -u tools/host_sweep.py all > $O/sweep.jsonl 2> $O/sweep.err; rc=$?; cat $O/sweep.jsonl; tail -3 $O/sweep.err; [ $rc -eq 0 ] || exit $rc
step c5 trace
ONE=splitk,4,256 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -o c5 -- python3 tools/host_sweep.py c5one > $O/c5one.json 2> $O/trace.err; rc=$?; cat $O/c5one.json
step done
