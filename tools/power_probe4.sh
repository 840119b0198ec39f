#!/bin/bash
# Package power / sclk while the C3 (1 M x 1 500 B) and C4-share (32 768 x 64 KiB) AEAD seal kernels
# loop (tools/stream_probe.py), sampled by rocm-smi.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/power4; mkdir -p $O
smi() { for k in 1 2 3 4 5 6; do (rocm-smi --showpower --showclocks 2>&1 || true) | grep -E "Power \(W\)|sclk" >> $1; sleep 1; done; }
for sh in "1048576 1500 30000" "32768 65536 30000"; do
  set -- $sh
  timeout -k 10 120 python tools/stream_probe.py --records $1 --record-bytes $2 --mode aead --reps $3 --alt > $O/r$2.json & pid=$!
  sleep 6; smi $O/r$2.smi; wait $pid || exit 1
  echo "L=$2 $(cat $O/r$2.json)"; sort $O/r$2.smi | uniq -c | sort -rn | head -4
done
