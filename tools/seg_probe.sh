#!/bin/bash
# seg_kernel timing probes: the shipping library vs hand-built libraries without the last-arriver
# combine (NO_TAIL) or the per-lane scaling (NO_SCALE); wrong tags by design, timing only.
set -o pipefail
O=gpurun_out/${1:-r06i_probe}
mkdir -p $O
export TMPDIR=/tmp
for v in ${VARIANTS:-ship NO_TAIL NO_SCALE}; do
  lib=""; [ $v != ship ] && lib=ephemeralnet_amd/libenet_probe_$v.so
  ENET_LIB_PATH=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o p -- python3 bench.py --long-only > $O/$v.json 2> $O/$v.err || exit 1
  python3 - $O/$v <<'PY'
import csv, glob, sys, statistics as S
rows = list(csv.DictReader(open(glob.glob(sys.argv[1] + '/*kernel_trace.csv')[0])))
g = {}
for r in rows:
    n = r['Kernel_Name']
    if 'seg_kernel' in n or 'seg_plan' in n or 'seg_uniform' in n:
        mode = 'seal' if '<1>' in n else 'open' if '<2>' in n else ''
        g.setdefault((n[:32], mode, r['Grid_Size_X']), []).append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1000)
for k, v in sorted(g.items()):
    print(sys.argv[1].split('/')[-1], k, len(v), round(S.median(v), 2))
PY
done
