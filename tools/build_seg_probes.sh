#!/bin/bash
# Hand-built timing-probe libraries (wrong tags by design): segments.hip recompiled with one
# or more ENET_SEG_PROBE_* switches (A+B), linked with the product's other objects into
# ephemeralnet_amd/libenet_probe_<SWITCH>.so; tools/seg_probe.sh times them beside the shipping
# library.  Run after `python -m ephemeralnet_amd.build`.
set -euo pipefail
cd "$(dirname "$0")/.."
B=ephemeralnet_amd/build
for v in "$@"; do
  o=/tmp/seg_probe_$v.o
  defs=""; for d in ${v//+/ }; do defs="$defs -DENET_SEG_PROBE_$d"; done
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++20 -fPIC -fvisibility=hidden -Wall -Wno-unused-function \
    -Iinclude $defs -c ephemeralnet_amd/csrc/segments.hip -o $o
  objs=$(ls $B/*.o | grep -v '/segments.o$')
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -fPIC -shared $objs $o -o ephemeralnet_amd/libenet_probe_$v.so
  echo built ephemeralnet_amd/libenet_probe_$v.so
done
