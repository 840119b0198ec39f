#!/bin/bash
# wire frames / chunk store at the C3 shape (1 M records, 1 500-byte messages: two-pass path) and
# at 1 536 bytes (a 128-byte multiple: fused path)
set -e
mkdir -p gpurun_out
: > gpurun_out/c3_side.jsonl
for L in 1500 1536; do for m in wire store; do
  timeout -k 10 200 python bench.py --mode $m --records 1048576 --record-bytes $L --steps 50 --warmup 5 --no-cpu-baseline >> gpurun_out/c3_side.jsonl
done; done
python -c "import json; [print(d['metric'][:36], d['config']['record_bytes'], d['value'], d['seal_ms'], d['open_ms']) for d in map(json.loads, open('gpurun_out/c3_side.jsonl'))]"
