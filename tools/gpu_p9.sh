#!/bin/bash
# round-4: the stream kernel's stream tail kernel for C3 (parity first), C3 A/B against line staging,
# C3 PMC, and the default bench line beside one-shot host pipeline runs on the same box.
# usage (on the box): bash tools/gpu_p9.sh TAG
set -o pipefail
T=${1:-p9}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step pytest tail shapes
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "one_lane_shapes or uniform_batches or lying or uniform_aad or full_size" > $O/pytest_tail.log 2>&1; rc=$?; tail -3 $O/pytest_tail.log; [ $rc -eq 0 ] || exit $rc
step pytest all
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
step c3 A/B
: > $O/c3.jsonl
for v in 3 1 3 1; do
ENET_STREAM=$v timeout -k 10 200 python bench.py --records 1048576 --record-bytes 1500 --steps 50 --warmup 10 --no-cpu-baseline --no-power --no-host > $O/x.json 2>> $O/c3.err || { echo c3 failed; exit 1; }
python -c "import json; d=json.load(open('$O/x.json')); d['ENET_STREAM']=$v; print(json.dumps(d))" >> $O/c3.jsonl
python -c "import json; d=json.load(open('$O/x.json')); print('C3 ENET_STREAM=$v', d['value'], d['seal_ms'], d['open_ms'])"
done
step c3 rocprof
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o c3 -- python3 bench.py --no-cpu-baseline --no-power --no-host --records 1048576 --record-bytes 1500 --steps 10 --warmup 3 > $O/prof_c3.json 2> $O/prof_c3.err; rc=$?; [ $rc -eq 0 ] || exit $rc
step c3 pmc
timeout -k 10 600 python tools/pmc.py --out $O/pmc_c3 --summary $O/pmc_c3_summary.json --config "{\"records\": 1048576, \"record_bytes\": 1500}" -- python3 bench.py --no-cpu-baseline --no-power --no-host --records 1048576 --record-bytes 1500 --steps 2 --warmup 1 > $O/pmc_c3.log 2>&1; rc=$?; tail -3 $O/pmc_c3.log; [ $rc -eq 0 ] || exit $rc
step bench default
timeout -k 10 240 python bench.py > $O/bench.json 2> $O/bench.err; rc=$?; cat $O/bench.json; [ $rc -eq 0 ] || exit $rc
step host one-shots
for one in c2one:splitk,4,32 c5one:splitk,4,128 c2one:splitk,3,32; do
  ONE=${one#*:} timeout -k 10 200 python -u tools/host_sweep.py ${one%%:*} >> $O/sweep.jsonl 2>> $O/sweep.err || { echo sweep failed; exit 1; }
done
cat $O/sweep.jsonl
step e2e variants
for a in "" "--chunk-mib 32 --streams 4" "--chunk-mib 32" "--streams 4"; do
  timeout -k 10 120 python bench.py --e2e $a > $O/x.json 2>> $O/e2e.err || { echo e2e failed; exit 1; }
  python -c "import json; d=json.load(open('$O/x.json')); print('e2e [$a]', d['value'], d['seal_GiBs'], d['open_GiBs'])" | tee -a $O/e2e.txt
done
ENET_HOST_TRACE=1 timeout -k 10 120 python bench.py --e2e > $O/x.json 2> $O/e2e_trace.err || { echo e2e failed; exit 1; }
tail -5 $O/e2e_trace.err
step done
