#!/bin/bash
# round-4: full parity (C3 line-staging change), C3 AEAD bench + PMC, host sweep with two kernel
# streams.  usage (on the box): bash tools/gpu_p7.sh TAG
set -o pipefail
T=${1:-p7}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step pytest
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
step c3 bench
: > $O/c3.jsonl
for i in 1 2; do
timeout -k 10 200 python bench.py --records 1048576 --record-bytes 1500 --steps 20 --warmup 5 --no-cpu-baseline --no-power --no-host > $O/x.json 2>> $O/c3.err || { echo c3 failed; exit 1; }
cat $O/x.json >> $O/c3.jsonl
python -c "import json; d=json.load(open('$O/x.json')); print('C3', d['value'], d['seal_ms'], d['open_ms'])"
done
step c3 pmc
timeout -k 10 600 python tools/pmc.py --out $O/pmc_c3 --summary $O/pmc_c3_summary.json --config "{\"records\": 1048576, \"record_bytes\": 1500}" -- python3 bench.py --no-cpu-baseline --no-power --no-host --records 1048576 --record-bytes 1500 --steps 2 --warmup 1 > $O/pmc_c3.log 2>&1; rc=$?; tail -3 $O/pmc_c3.log; [ $rc -eq 0 ] || exit $rc
step host_sweep
SWEEP_MODES=splitk timeout -k 10 500 python -u tools/host_sweep.py all > $O/sweep.jsonl 2> $O/sweep.err; rc=$?; cat $O/sweep.jsonl; tail -3 $O/sweep.err; [ $rc -eq 0 ] || exit $rc
step done
