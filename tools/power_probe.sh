#!/bin/bash
# Board power and clocks while the C2 seal kernel runs back to back (tools/stream_probe.py with many
# reps) under ENET_STREAM_DBG: 0 full, 1 memory waves idle (no HBM), 2 no keystream (memory only).
# usage (on the box): bash tools/power_probe.sh "0 1 2"
set -uo pipefail
export TMPDIR=/tmp
DS=${1:-0 1 2}
O=gpurun_out/power; mkdir -p $O
(rocm-smi --showpower --showclocks --showtemp 2>&1 || true) > $O/idle.txt
for d in $DS; do
  ENET_STREAM_DBG=$d timeout -k 10 120 python tools/stream_probe.py --mode aead --reps 150000 --alt > $O/d$d.json &
  pid=$!
  sleep 5
  for k in 1 2 3 4 5 6; do (rocm-smi --showpower --showclocks 2>&1 || true) >> $O/d$d.smi; sleep 1; done
  wait $pid || exit 1
  echo "dbg $d $(cat $O/d$d.json)"
  grep -iE "power|sclk|mclk|fclk" $O/d$d.smi | sort | uniq -c | head -20
done
