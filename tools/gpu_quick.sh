#!/bin/bash
# A short GPU session: parity suite, the default bench line, C3 (AEAD and wire frames), and
# optionally the PMC passes of C2 and C3 (tools/pmc.py; separate --pmc runs, no tracing).
# usage (on the box, from the repo root): bash tools/gpu_quick.sh TAG [pmc]
set -euo pipefail
T=${1:-quick}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step pytest
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
step bench default
timeout -k 10 240 python bench.py > $O/bench.json 2> $O/bench.err
cat $O/bench.json
step side
: > $O/side.jsonl
for args in "--records 1048576 --record-bytes 1500" "--mode wire --records 1048576 --record-bytes 1500"; do
  step "  $args"
  timeout -k 10 240 python bench.py --steps 10 --warmup 3 --no-cpu-baseline $args >> $O/side.jsonl 2>> $O/side.err
done
step scalar latency
for pol in auto device; do
  timeout -k 10 180 oracle/_ref/scalar_latency_gpu 200 $pol 16 > $O/latency_$pol.jsonl 2> $O/latency_$pol.err
done
timeout -k 10 180 oracle/_ref/scalar_latency_ref 200 x 16 > $O/latency_ref.jsonl 2> $O/latency_ref.err
if [ "${2:-}" = pmc ]; then
step pmc
timeout -k 10 600 python tools/pmc.py --out $O/pmc --summary $O/pmc_summary.json --config "{\"records\": 65536, \"record_bytes\": 4096}" -- python3 bench.py --no-cpu-baseline --no-power --steps 3 --warmup 1 > $O/pmc.log 2>&1
timeout -k 10 600 python tools/pmc.py --out $O/pmc_c3 --summary $O/pmc_c3_summary.json --config "{\"records\": 1048576, \"record_bytes\": 1500}" -- python3 bench.py --no-cpu-baseline --no-power --records 1048576 --record-bytes 1500 --steps 2 --warmup 1 > $O/pmc_c3.log 2>&1
fi
step done
