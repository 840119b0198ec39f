#!/bin/bash
# Interleaved A/B of the default bench line between the in-tree library and a previous build
# (ephemeralnet_amd/libenet_crypto_prev.so, ENET_LIB_PATH).  usage: bash tools/ab_lib.sh TAG PAIRS [bench args]
set -euo pipefail
T=${1:-ab}; N=${2:-3}; shift 2 || true
O=gpurun_out/$T
mkdir -p $O
: > $O/ab.jsonl
for i in $(seq 1 $N); do
  for v in prev new; do
    if [ $v = prev ]; then export ENET_LIB_PATH=$PWD/ephemeralnet_amd/libenet_crypto_prev.so; else unset ENET_LIB_PATH; fi
    timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-power "$@" > $O/one.json 2>> $O/ab.err
    python -c "import json,sys; d=json.load(open('$O/one.json')); d['lib']='$v'; print(json.dumps(d))" >> $O/ab.jsonl
    python -c "import json; d=json.load(open('$O/one.json')); print('$v', d['value'], d['roofline']['frac'])"
  done
done
