# Wire frames (C2 shape): fused HMAC + ChaCha20 kernel vs the two-pass path (ENET_FUSED_FRAMES=0)
set -e
for t in fused twopass fused2; do
  e=1; [ $t = twopass ] && e=0
  ENET_FUSED_FRAMES=$e timeout -k 10 120 python bench.py --mode wire --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/fab_$t.json 2>/dev/null
  python3 -c "
import json; d=json.load(open('gpurun_out/fab_$t.json')); print('$t', d['value'], d['seal_ms'], d['open_ms'])"
done
