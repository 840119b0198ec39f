#!/bin/bash
# round-4: C5 share with ramp-up (default) vs no ramp, interleaved
set -o pipefail
T=${1:-p24}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2 3; do
  for r in 1 0; do
    ENET_HOST_RAMP=$r ONE=splitk,4,128 timeout -k 10 150 python -u tools/host_sweep.py c5one > $O/x.json 2>> $O/err || { echo failed; exit 1; }
    python -c "import json; d=json.load(open('$O/x.json')); d['ramp']=$r; print(json.dumps(d))" | tee -a $O/ramp.jsonl
  done
done
