#!/bin/bash
# Timing probes of the streaming kernel (ENET_STREAM_DBG, wrong output by design): seal and
# xor kernel time at C2 with parts of the work switched off.
# usage: python ephemeralnet_amd/build.py --tools (here), then on the box:
#   bash tools/stream_probe.sh [tag] [dbg values...]
set -euo pipefail
T=${1:-probe}; shift || true
DS=${@:-0 1 4 16 256 257}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
# the probes exist only in the tools build of the library (build.py --tools)
export ENET_LIB_PATH=$PWD/ephemeralnet_amd/libenet_crypto_tools.so
for d in $DS; do
  for m in aead xor; do
    ENET_STREAM_DBG=$d timeout -k 10 120 python tools/stream_probe.py --mode $m > $O/d${d}_$m.json
    echo "dbg $d $m $(cat $O/d${d}_$m.json)"
  done
done
