#!/bin/bash
# round-4: C5 share with / without a tail ramp for hash-chain-bound jobs (ENET_HOST_RAMP 1 vs 5),
# 4 x 128 MiB and 4 x 256 MiB, interleaved
set -o pipefail
T=${1:-p23}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2 3; do
  for r in 1 5; do
    for ch in 128 256; do
      ENET_HOST_RAMP=$r ONE=splitk,4,$ch timeout -k 10 150 python -u tools/host_sweep.py c5one > $O/x.json 2>> $O/err || { echo failed; exit 1; }
      python -c "import json; d=json.load(open('$O/x.json')); d['ramp']=$r; print(json.dumps(d))" | tee -a $O/ramp.jsonl
    done
  done
done
