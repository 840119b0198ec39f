#!/bin/bash
# Power / sclk of a linear device copy (tools/copy_power.py) and of the ChaCha20-only C2 pass
# (ENET_STREAM_DBG 0 / 1, --mode xor), sampled by rocm-smi while they run.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/power2; mkdir -p $O
smi() { for k in 1 2 3 4 5 6; do (rocm-smi --showpower --showclocks 2>&1 || true) | grep -E "Power \(W\)|sclk" >> $1; sleep 1; done; }
timeout -k 10 60 python tools/copy_power.py 14 > $O/copy.json & pid=$!; sleep 5; smi $O/copy.smi; wait $pid || exit 1
echo "copy $(cat $O/copy.json)"; sort $O/copy.smi | uniq -c
for d in 0 1; do
  ENET_STREAM_DBG=$d timeout -k 10 120 python tools/stream_probe.py --mode xor --reps 150000 --alt > $O/x$d.json & pid=$!
  sleep 5; smi $O/x$d.smi; wait $pid || exit 1
  echo "xor dbg $d $(cat $O/x$d.json)"; sort $O/x$d.smi | uniq -c
done
