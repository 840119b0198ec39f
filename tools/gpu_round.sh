#!/bin/bash
# One GPU session producing the round's evidence under gpurun_out/r$R/: GPU parity suite, the
# default bench line, side configs/modes, rocprofv3 kernel stats, and PMC passes.
# usage (on the box, from the repo root): bash tools/gpu_round.sh 01
set -euo pipefail
R=${1:-01}
O=gpurun_out/r$R
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step pytest
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -2 $O/pytest_gpu.log
step bench default
timeout -k 10 240 python bench.py > $O/bench.json 2> $O/bench.err
cat $O/bench.json
step side configs
: > $O/side.jsonl
for args in "--records 1048576 --record-bytes 1500" "--records 32768 --record-bytes 65536" \
            "--mode xor" "--mode wire" "--mode store" "--e2e" "--c5"; do
  step "  $args"
  timeout -k 10 240 python bench.py --no-cpu-baseline --steps 100 --warmup 20 $args >> $O/side.jsonl 2>> $O/side.err
done
step rocprof stats
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --no-cpu-baseline --steps 50 --warmup 10 > $O/prof_bench.json 2> $O/prof.err
find $O/prof -name "*stats*" | head
step pmc
timeout -k 10 600 python tools/pmc.py --out $O/pmc --summary $O/pmc_summary.json --config "{\"records\": 65536, \"record_bytes\": 4096}" -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > $O/pmc.log 2>&1
step done
