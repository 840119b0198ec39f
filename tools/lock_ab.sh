# A/B of the staging variants (same box): ENET_COOP=1 (default: lockstep + line staging),
# 4 (plain run staging), ENET_LOCKSTEP=0 (default without lockstep) on C2, C4 and C3.
set -e
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 120 python bench.py --steps 300 --warmup 30 --no-cpu-baseline > gpurun_out/lk_c2_$tag.json 2>/dev/null
  env "$@" timeout -k 10 120 python bench.py --records 32768 --record-bytes 65536 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/lk_c4_$tag.json 2>/dev/null
  env "$@" timeout -k 10 120 python bench.py --records 1048576 --record-bytes 1500 --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/lk_c3_$tag.json 2>/dev/null
  python3 -c "
import json
for c in ('c2','c4','c3'):
    d=json.load(open('gpurun_out/lk_'+c+'_$tag.json')); print('$tag', c, d['value'], d['seal_ms'], d['open_ms'])"
}
run default ENET_COOP=1
run nolock ENET_LOCKSTEP=0
run lineslock ENET_LINES_LOCKSTEP=1
run plain ENET_COOP=4
run default2 ENET_COOP=1
