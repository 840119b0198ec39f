#!/bin/bash
# Streaming kernel code variants (ENET_STREAM_VAR) x probes (ENET_STREAM_DBG) at C2.
# usage (on the box): bash tools/stream_var.sh tag "vars" "dbgs"
set -euo pipefail
T=${1:-var}; VS=${2:-0 1 2 3}; DS=${3:-0 257}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
for v in $VS; do export ENET_STREAM_VAR=$v
  for d in $DS; do
    for m in aead xor; do
      ENET_STREAM_VAR=$v ENET_STREAM_DBG=$d timeout -k 10 120 python tools/stream_probe.py --mode $m $ALT > $O/v${v}_d${d}_$m.json
      echo "var $v dbg $d $m $(cat $O/v${v}_d${d}_$m.json)"
    done
  done
done
