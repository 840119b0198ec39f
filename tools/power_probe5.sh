#!/bin/bash
# Package power / sclk while the duplex kernels (cipher + hash lanes) loop: wire frames and chunk
# store+fetch at the C2 shape (bench.py --mode wire / store with many steps), sampled by rocm-smi.
set -uo pipefail
export TMPDIR=/tmp
O=gpurun_out/power5; mkdir -p $O
smi() { for k in 1 2 3 4 5; do (rocm-smi --showpower --showclocks 2>&1 || true) | grep -E "Power \(W\)|sclk" >> $1; sleep 1; done; }
for m in wire store; do
  timeout -k 10 180 python bench.py --mode $m --steps 6000 --warmup 20 --no-cpu-baseline --no-power > $O/$m.json 2>/dev/null & pid=$!
  sleep 8; smi $O/$m.smi; wait $pid || exit 1
  python3 -c "import json; d=json.load(open('$O/$m.json')); print('$m', d['value'], d['seal_ms'], d['open_ms'])"
  sort $O/$m.smi | uniq -c | sort -rn | head -4
done
