#!/bin/bash
# C5 experiments: device-resident with and without step overlap and the duplex kernel's
# length-graded priority (ENET_DUPLEX_PRIO=-1: off); host-resident pipeline chunk sizes with
# more hardware queues (GPU_MAX_HW_QUEUES, HIP's default 4).  usage: bash tools/c5_probe.sh TAG
set -euo pipefail
O=gpurun_out/${1:-c5}
mkdir -p $O
export TMPDIR=/tmp
: > $O/c5.jsonl
for pr in 0 -1; do
for a in "--c5-device --records 65536" "--c5-device --records 65536 --c5-overlap"; do
  echo "prio $pr $a"; ENET_DUPLEX_PRIO=$pr timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --warmup 3 $a >> $O/c5.jsonl 2>> $O/c5.err
  tail -1 $O/c5.jsonl | cut -c1-120
done; done
for q in 4 16; do for ch in 32 64 128; do
  echo "hwq $q chunk $ch"
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --no-cpu-baseline --c5 --steps 2 --warmup 1 --c5-streams 12 --c5-chunk-mib $ch > $O/c5_q${q}_c${ch}.json 2>> $O/c5.err
  cut -c1-160 $O/c5_q${q}_c${ch}.json
done; done
