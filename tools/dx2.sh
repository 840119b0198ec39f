export TMPDIR=/tmp
O=gpurun_out/dx2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_duplex.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for cfg in "--records 1048576 --record-bytes 1500" "--records 65536 --record-bytes 1536" "--records 65536 --record-bytes 4096"; do
  timeout -k 10 120 python bench.py --mode wire $cfg --steps 20 --warmup 5 --no-cpu-baseline > $O/w.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('$O/w.json'));print('wire $cfg', d['value'], d.get('seal_ms'), d.get('open_ms'))"
done
timeout -k 10 120 python bench.py --mode store --records 65536 --record-bytes 4096 --steps 20 --warmup 5 --no-cpu-baseline > $O/s.json 2>/dev/null || exit 1
python3 -c "import json;d=json.load(open('$O/s.json'));print('store 4096', d['value'], d.get('seal_ms'), d.get('open_ms'))"
