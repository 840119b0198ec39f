export TMPDIR=/tmp
O=gpurun_out/prio; mkdir -p $O
for rep in 1 2 3; do
  for D in 0 4096; do
    ENET_STREAM_DBG=$D timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/b.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('$O/b.json'));print('dbg=$D', d['value'], d['seal_ms'], d['open_ms'])"
  done
done
