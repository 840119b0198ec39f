#!/bin/bash
# round-4: host-resident C2 under torch's HIP runtime with SDMA knobs of its HSA runtime
# usage (on the box): bash tools/gpu_p11.sh TAG
set -o pipefail
T=${1:-p11}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
for env in "X=0" "HSA_ENABLE_SDMA_GANG=0" "HSA_ENABLE_SDMA_GANG=1" "HSA_ENABLE_SDMA_RECOMMENDED_ENG=0" "HSA_ENABLE_SDMA_RECOMMENDED_ENG=1"; do
  for o in torch_first lib_first; do
    step "$env $o"
    env $env timeout -k 10 120 python tools/e2e_probe.py $o > $O/x.json 2>> $O/probe.err || { echo probe failed; exit 1; }
    python -c "import json; d=json.load(open('$O/x.json')); d['env']='$env'; print(json.dumps({k: d[k] for k in ('env', 'order', 'c2_32_4', 'c2_0_0')}))" | tee -a $O/probe.jsonl
  done
done
step done
