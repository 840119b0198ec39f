# A/B of the lockstep barrier spacing (one barrier per 1, 2 or 4 step groups of 24 instructions)
set -e
cp ephemeralnet_amd/libenet_crypto.so /tmp/libenet_le1.so
for e in 1 2 4 1; do
  cp /tmp/libenet_le$e.so ephemeralnet_amd/libenet_crypto.so 2>/dev/null || cp tools/libenet_le$e.so ephemeralnet_amd/libenet_crypto.so
  timeout -k 10 120 python bench.py --steps 300 --warmup 30 --no-cpu-baseline > gpurun_out/le_c2_$e.json 2>/dev/null
  timeout -k 10 120 python bench.py --records 32768 --record-bytes 65536 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/le_c4_$e.json 2>/dev/null
  python3 -c "
import json
for c in ('c2','c4'):
    d=json.load(open('gpurun_out/le_'+c+'_$e.json')); print('every $e', c, d['value'], d['seal_ms'], d['open_ms'])"
done
