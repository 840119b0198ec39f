#!/bin/bash
# Energy per byte of the streaming kernel's memory path vs a linear copy: power / sclk under
# ChaCha20-only ENET_STREAM_DBG 2 (memory waves only: DMA + LDS + stores) and 3 (barriers only),
# and tools/copy_power.py, sampled by rocm-smi while each runs.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/power3; mkdir -p $O
smi() { for k in 1 2 3 4 5 6; do (rocm-smi --showpower --showclocks 2>&1 || true) | grep -E "Power \(W\)|sclk" >> $1; sleep 1; done; }
for d in 2 3; do
  ENET_STREAM_DBG=$d timeout -k 10 120 python tools/stream_probe.py --mode xor --reps 200000 --alt > $O/x$d.json & pid=$!
  sleep 5; smi $O/x$d.smi; wait $pid || exit 1
  echo "xor dbg $d $(cat $O/x$d.json)"; sort $O/x$d.smi | uniq -c | sort -rn | head -4
done
timeout -k 10 60 python tools/copy_power.py 14 > $O/copy.json & pid=$!; sleep 5; smi $O/copy.smi; wait $pid || exit 1
echo "copy $(cat $O/copy.json)"; sort $O/copy.smi | uniq -c | sort -rn | head -4
