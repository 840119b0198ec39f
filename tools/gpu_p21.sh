#!/bin/bash
# round-4: host pipeline chunk ramps (ENET_HOST_RAMP 3 = up+down, 1 = up only, 2 = down only,
# 0 = none) x C2 chunk 32 / 48 MiB, interleaved on one box
# usage (on the box): bash tools/gpu_p21.sh TAG
set -o pipefail
T=${1:-p21}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do
  for r in 3 1 2 0; do
    for ch in 32 48; do
      ENET_HOST_RAMP=$r ONE=splitk,4,$ch timeout -k 10 120 python -u tools/host_sweep.py c2one > $O/x.json 2>> $O/err || { echo failed; exit 1; }
      python -c "import json; d=json.load(open('$O/x.json')); d['ramp']=$r; print(json.dumps(d))" | tee -a $O/ramp.jsonl
    done
  done
done
