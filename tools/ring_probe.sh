#!/bin/bash
# Seal kernel time at C3 (1 M x 1 500 B) of the output-ring streaming kernel under the tools
# build's probes (ENET_STREAM_DBG: 64 no unit stores, 128 no input loads, 2 no keystream, 16 no
# ring writes, 8 no ragged end; ENET_STREAM_VAR: 1 non-temporal unit stores, 2 input through the
# memory waves' VGPRs instead of LDS DMAs), beside the line-staging records kernel
# (ENET_STREAM_RING=0).  usage: bash tools/ring_probe.sh TAG "VARS" "DBGS"
set -euo pipefail
T=${1:-ring_probe}
VARS=${2:-"0 1 2 3"}
DBGS=${3:-"0 90"}
O=gpurun_out/$T
mkdir -p $O
: > $O/probe.jsonl
run() { timeout -k 10 120 python tools/stream_probe.py --alt --records 1048576 --record-bytes 1500 --reps 40 >> $O/probe.jsonl; tail -1 $O/probe.jsonl; }
echo "records kernel"; ENET_STREAM_RING=0 run
export ENET_LIB_PATH=$PWD/ephemeralnet_amd/libenet_crypto_tools.so ENET_STREAM_RING=1
for v in $VARS; do for d in $DBGS; do echo "var $v dbg $d"; ENET_STREAM_VAR=$v ENET_STREAM_DBG=$d run; done; done
