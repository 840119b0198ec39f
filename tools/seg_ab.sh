#!/bin/bash
# A/B of hand-built seg probe libraries on tools/seg_bench.py (1 x 32 MiB, seal+open and XOR pairs):
#   bash tools/seg_ab.sh OUT ship VARIANT...   (VARIANT = a libenet_probe_<VARIANT>.so)
set -o pipefail
O=gpurun_out/$1; shift
mkdir -p $O
export PYTHONPATH=$PWD
for v in "$@"; do
  lib=""; [ $v != ship ] && lib=$PWD/ephemeralnet_amd/libenet_probe_$v.so
  ENET_LIB_PATH=$lib timeout -k 10 120 python3 tools/seg_bench.py 40 > $O/$v.json 2> $O/$v.err || exit 1
  echo "$v $(cat $O/$v.json)"
  if [[ $v == *TRACE* ]]; then
    ENET_LIB_PATH=$lib timeout -k 10 120 python3 tools/seg_trace.py > $O/$v.trace.json 2>> $O/$v.err || exit 1
  fi
done
