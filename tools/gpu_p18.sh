#!/bin/bash
# round-4: host mode 4 (SDMA in, kernels write host memory): parity of the pipelines in every
# mode, then splitk vs zcout under both HIP runtimes, C5 share and the batch path.
# usage (on the box): bash tools/gpu_p18.sh TAG
set -o pipefail
T=${1:-p18}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step pytest pipeline
timeout -k 10 400 python -u -m pytest tests/test_gpu_pipeline.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for m in splitk zcout splitk zcout; do
  for o in torch_first lib_first; do
    ENET_HOST_MODE=$m timeout -k 10 120 python tools/e2e_probe.py $o > $O/x.json 2>> $O/probe.err || { echo probe failed; exit 1; }
    python -c "import json; d=json.load(open('$O/x.json')); print(json.dumps({'mode': '$m', 'order': d['order'], 'c2_32_4': d['c2_32_4'], 'c2_0_0': d['c2_0_0']}))" | tee -a $O/probe.jsonl
  done
  ONE=$m,4,128 timeout -k 10 200 python -u tools/host_sweep.py c5one | tee -a $O/c5.jsonl || { echo c5 failed; exit 1; }
done
for m in splitk zcout; do
  step "batch_bench $m"
  ENET_HOST_MODE=$m timeout -k 10 300 tools/batch_bench all 3 > $O/bb_$m.jsonl 2>> $O/bb.err || { echo bb failed; exit 1; }
  grep -v vectors $O/bb_$m.jsonl
done
step done
