#!/bin/bash
# round-4: what torch's bundled HIP runtime does with the host pipeline's copies (trace)
# usage (on the box): bash tools/gpu_p17.sh TAG
set -o pipefail
T=${1:-p17}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
step trace torch_first
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/tt -o tt -- python3 tools/e2e_probe.py torch_first > $O/tt.json 2> $O/tt.err; rc=$?; cat $O/tt.json; [ $rc -eq 0 ] || exit $rc
step trace lib_first
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/lf -o lf -- python3 tools/e2e_probe.py lib_first > $O/lf.json 2> $O/lf.err; rc=$?; cat $O/lf.json; [ $rc -eq 0 ] || exit $rc
for x in tt lf; do echo "== $x kernels"; cut -d, -f1-4 $O/$x/${x}_kernel_stats.csv | head -8; echo "== $x copies"; cat $O/$x/${x}_memory_copy_stats.csv 2>/dev/null | head -5; done
step done
