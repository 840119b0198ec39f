# Same-box A/B of non-temporal whole-line output stores (ENET_NT_STORES=0/1): C2 and 1472-byte
# records (half-line-aligned runs).
set -e
for nt in 0 1; do
  ENET_NT_STORES=$nt timeout -k 10 120 python bench.py --steps 300 --warmup 30 --no-cpu-baseline > gpurun_out/nt_c2_$nt.json 2>/dev/null
  ENET_NT_STORES=$nt timeout -k 10 120 python bench.py --records 1048576 --record-bytes 1472 --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/nt_1472_$nt.json 2>/dev/null
  python3 -c "
import json
for c in ('c2','1472'):
    d=json.load(open('gpurun_out/nt_'+c+'_$nt.json')); print('nt $nt', c, d['value'], d['seal_ms'], d['open_ms'], d['ms_per_step'])"
done
