export TMPDIR=/tmp
O=gpurun_out/dx3; mkdir -p $O
for D in 1 0; do
  for ord in sorted none; do
    ENET_DUPLEX=$D timeout -k 10 120 python bench.py --c5-device --c5-order $ord --records 65536 --steps 5 --warmup 2 > $O/c5.json 2>$O/c5.err || { tail $O/c5.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/c5.json'));print('duplex=$D c5dev $ord', d['value'], d['ms_per_step'])"
  done
done
timeout -k 10 200 python bench.py --c5 --records 65536 > $O/c5h.json 2>$O/c5h.err || { tail $O/c5h.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/c5h.json'));print('c5 host', d['value'])"
for cfg in "--records 65536 --record-bytes 4160" "--records 65536 --record-bytes 4096" "--records 262144 --record-bytes 4096"; do
  timeout -k 10 120 python bench.py --mode wire $cfg --steps 20 --warmup 5 --no-cpu-baseline > $O/w.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('$O/w.json'));print('wire $cfg', d['value'], d.get('seal_ms'), d.get('open_ms'))"
done
