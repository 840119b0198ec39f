#!/bin/bash
# One GPU session: parity suite, default bench, rocprof kernel stats of the bench.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 200 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
cat gpurun_out/bench.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --no-cpu-baseline --steps 50 --warmup 5 > gpurun_out/bench_prof.json 2> gpurun_out/prof.err
find gpurun_out/prof -name "*kernel_stats.csv" | head -3
