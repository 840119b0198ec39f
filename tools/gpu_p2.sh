#!/bin/bash
# round-4 host-mode sweep: pipeline parity in every mode, C2 e2e and C5 host (per-GPU share) per
# mode and chunk size, the C++ batch API per mode and worker count.
# usage (on the box): bash tools/gpu_p2.sh TAG
set -o pipefail
T=${1:-p2}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step pytest
timeout -k 10 400 python -u -m pytest tests/test_gpu_pipeline.py tests/test_cpp_api.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
step e2e / c5 sweep
: > $O/host.jsonl
for m in zc sdma split splitk; do
  for c in 0 16 64; do
    ENET_HOST_MODE=$m timeout -k 10 120 python bench.py --e2e --chunk-mib $c > $O/x.json 2>> $O/host.err || { echo "e2e $m $c failed"; exit 1; }
    python -c "import json,sys; d=json.load(open('$O/x.json')); d['mode']='$m'; print(json.dumps(d))" >> $O/host.jsonl
  done
  for c in 0 64 256; do
    ENET_HOST_MODE=$m timeout -k 10 180 python bench.py --c5 --records 65536 --c5-chunk-mib $c > $O/x.json 2>> $O/host.err || { echo "c5 $m $c failed"; exit 1; }
    python -c "import json,sys; d=json.load(open('$O/x.json')); d['mode']='$m'; print(json.dumps(d))" >> $O/host.jsonl
  done
done
python -c "
import json
for l in open('$O/host.jsonl'):
    d=json.loads(l); c=d['config']; print(d['mode'], c.get('workload','C2'), c.get('chunk_mib', c.get('c5_chunk_mib')), d['value'])"
step batch_bench
: > $O/batch.jsonl
for cfg in "split 8 1" "split 15 1" "split 15 0" "zc 15 1"; do
  set -- $cfg
  ENET_HOST_MODE=$1 ENET_HOST_THREADS=$2 ENET_HOST_NT=$3 timeout -k 10 300 tools/batch_bench all 3 > $O/x.jsonl 2>> $O/batch.err || { echo "batch $cfg failed"; exit 1; }
  sed "s/^{/{\"mode\":\"$1\",\"threads\":$2,\"nt\":$3,/" $O/x.jsonl >> $O/batch.jsonl
done
cat $O/batch.jsonl
step done
