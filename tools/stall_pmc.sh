#!/bin/bash
# Stall counters of the streaming kernel: full, no stores, compute only (tools/pmc.py --passes stall).
set -euo pipefail
T=${1:-stall}; V=${2:-6}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
for d in 0 64 257; do
  ENET_STREAM_VAR=$V ENET_STREAM_DBG=$d timeout -k 10 300 python tools/pmc.py --passes stall --out $O/p_d$d --summary $O/stall_d$d.json -- python3 tools/stream_probe.py --mode aead --reps 20 > $O/log_d$d.txt 2>&1
  echo "dbg $d done"
done
