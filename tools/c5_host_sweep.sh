#!/bin/bash
# C5 host-resident (H2D + kernels + D2H) pipeline: chunk size x streams, and the BASELINE C5 size
# (524 288 records) beside the 65 536-record default.  usage: bash tools/c5_host_sweep.sh TAG
set -euo pipefail
O=gpurun_out/${1:-c5host}
mkdir -p $O
export TMPDIR=/tmp
: > $O/c5host.jsonl
for rc in "65536 64 8" "65536 128 8" "65536 256 6" "65536 128 4" "524288 256 6" "524288 128 8"; do
  set -- $rc
  echo "records $1 chunk $2 streams $3"
  timeout -k 10 400 python bench.py --no-cpu-baseline --c5 --steps 2 --warmup 1 --records $1 --c5-chunk-mib $2 --c5-streams $3 >> $O/c5host.jsonl 2>> $O/c5host.err
  tail -1 $O/c5host.jsonl | cut -c1-200
done
