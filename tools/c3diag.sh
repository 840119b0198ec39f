set -e
for cfg in "1500 0" "1500 2" "1504 0" "1536 0" "1472 0" "1536 2"; do
  set -- $cfg
  timeout -k 10 120 python bench.py --records 1048576 --record-bytes $1 --lanes $2 --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/c3_$1_$2.json 2>/dev/null
  python3 -c "import json; d=json.load(open('gpurun_out/c3_$1_$2.json')); print('$1', '$2', d['value'], d['seal_ms'], d['open_ms'], d['config']['lanes_per_record'])"
done
