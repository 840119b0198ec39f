#!/bin/bash
# round-4: crypto::batch gather chunk 16 vs 32 MiB, interleaved on one box
# usage (on the box): bash tools/gpu_p16.sh TAG
set -o pipefail
T=${1:-p16}
O=gpurun_out/$T
mkdir -p $O
step() { echo "[$(date +%T)] $*"; }
for i in 1 2 3; do
  for ch in 16 32; do
    step "chunk $ch ($i)"
    ENET_HOST_CHUNK_MIB=$ch timeout -k 10 200 tools/batch_bench all 3 > $O/x.jsonl 2>> $O/bb.err || { echo bb failed; exit 1; }
    python - "$ch" "$O/x.jsonl" <<'PY' | tee -a $O/ab.jsonl
import json, sys
ch, path = sys.argv[1], sys.argv[2]
rows = [json.loads(l) for l in open(path)]
get = lambda shape, key: next(r["seal_open_GiBs"] for r in rows if r["shape"] == shape and key in r["path"])
print(json.dumps({"chunk_mib": int(ch), "c2_packed": get("C2", "packed"), "c2_pinned": get("C2", "pinned"),
                  "c3_packed": get("C3 wire", "packed"), "c3_pinned": get("C3 wire", "pinned")}))
PY
  done
done
step done
