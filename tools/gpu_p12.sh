#!/bin/bash
# round-4: bench host legs in child processes (system HIP runtime): default line, --e2e, --c5
# share, and the N = 2 gloo rehearsal on one card (two children in lockstep).
# usage (on the box): bash tools/gpu_p12.sh TAG
set -o pipefail
T=${1:-p12}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step bench default
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err; rc=$?; cat $O/bench.json; [ $rc -eq 0 ] || exit $rc
step e2e
timeout -k 10 120 python bench.py --e2e > $O/e2e.json 2> $O/e2e.err; rc=$?; cat $O/e2e.json; [ $rc -eq 0 ] || exit $rc
step c5 share
timeout -k 10 200 python bench.py --c5 --records 65536 > $O/c5.json 2> $O/c5.err; rc=$?; cat $O/c5.json; [ $rc -eq 0 ] || exit $rc
step rehearsal N=2 gloo on one card
ENET_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29551 bench.py --gpus 2 --steps 50 --warmup 10 --no-cpu-baseline > $O/rehearsal_n2.json 2> $O/rehearsal_n2.err; rc=$?; cat $O/rehearsal_n2.json; [ $rc -eq 0 ] || exit $rc
step done
