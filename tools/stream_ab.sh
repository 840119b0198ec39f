#!/bin/bash
# A/B of stream-kernel variants (tools build, ENET_STREAM_VAR) at C2, interleaved, bench line values.
# usage (after python ephemeralnet_amd/build.py --tools): bash tools/stream_ab.sh TAG "VARS" [reps]
set -euo pipefail
O=gpurun_out/${1:-sab}
VARS=${2:-"0 20"}
REPS=${3:-2}
mkdir -p $O
export TMPDIR=/tmp
export ENET_LIB_PATH=$PWD/ephemeralnet_amd/libenet_crypto_tools.so
for r in $(seq $REPS); do for v in $VARS; do
  ENET_STREAM_VAR=$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-power --steps 200 --warmup 30 > $O/v${v}_$r.json 2>> $O/err.log
  python3 -c "import json;d=json.load(open('$O/v${v}_$r.json'));print('var $v rep $r', d['value'], d['seal_ms'], d['open_ms'], d['power'] if 'power' in d else '')"
done; done
