#!/bin/bash
# round-4: full GPU suite, smoke, the default bench line (now with host-resident keys), and a
# kernel + memory-copy timeline of the C5 host pipeline.  usage (on the box): bash tools/gpu_p5.sh TAG
set -o pipefail
T=${1:-p5}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step pytest
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; tail -2 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
step bench
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err; rc=$?; cat $O/bench.json; tail -3 $O/bench.err; [ $rc -eq 0 ] || exit $rc
step c5 trace
ONE=splitk,3,256 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -o c5 -- python3 tools/host_sweep.py c5one > $O/c5one.json 2> $O/trace.err; rc=$?; cat $O/c5one.json; tail -3 $O/trace.err
find $O/trace -name "*.csv" | head
step rehearsal N=2 gloo on one card
ENET_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --steps 50 --warmup 10 --no-cpu-baseline > $O/rehearsal_n2.json 2> $O/rehearsal_n2.err; rc=$?; cat $O/rehearsal_n2.json; tail -3 $O/rehearsal_n2.err
step done
