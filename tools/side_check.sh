#!/bin/bash
# GPU parity suite, then the SHA-bound side modes (wire frames, chunk store/fetch both id modes)
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
: > gpurun_out/side.jsonl
for a in "--mode wire" "--mode store --store-ids given" "--mode store --store-ids content" "--mode xor"; do
  timeout -k 10 200 python bench.py $a --steps 100 --warmup 20 --no-cpu-baseline >> gpurun_out/side.jsonl
done
python -c "import sys,json; [print(d['metric'][:40], d['config'].get('chunk_ids',''), d['value'], d['seal_ms'], d['open_ms']) for d in map(json.loads, open('gpurun_out/side.jsonl'))]"
