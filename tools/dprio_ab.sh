export TMPDIR=/tmp
O=gpurun_out/dprio; mkdir -p $O
for P in 0 1 2; do
  for cfg in "--mode wire --records 1048576 --record-bytes 1500" "--mode store --records 32768 --record-bytes 65536" "--mode wire --records 65536 --record-bytes 4096"; do
    ENET_DUPLEX_PRIO=$P timeout -k 10 120 python bench.py $cfg --steps 10 --warmup 3 --no-cpu-baseline > $O/w.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('$O/w.json'));print('prio=$P $cfg', d['value'])"
  done
  ENET_DUPLEX_PRIO=$P timeout -k 10 120 python bench.py --c5-device --records 65536 --steps 5 --warmup 2 > $O/c5.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('$O/c5.json'));print('prio=$P c5dev', d['value'])"
done
