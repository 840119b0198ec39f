set -e
for coop in 1 2; do
  for cfg in "65536 4096 2" "65536 4096 4" "1048576 1500 1" "32768 65536 4" "32768 65536 8" "32768 65536 16"; do
    set -- $cfg
    ENET_COOP=$coop timeout -k 10 100 python bench.py --no-cpu-baseline --records $1 --record-bytes $2 --lanes $3 --steps 200 --warmup 30 > gpurun_out/sw_${coop}_$1_$3.json
    python -c "import json; d=json.load(open('gpurun_out/sw_${coop}_$1_$3.json')); print('coop', $coop, 'n', $1, 'L', $2, 'P', $3, d['value'], d['seal_ms'], d['open_ms'])"
  done
done
