export TMPDIR=/tmp
O=gpurun_out/dx4; mkdir -p $O
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 120 python bench.py --c5-device --c5-order sorted --records 65536 --steps 5 --warmup 2 > $O/c5.json 2>$O/c5.err || { tail $O/c5.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/c5.json'));print('c5dev sorted', d['value'], d['ms_per_step'])"
for sc in "3 64" "8 64" "8 128" "6 256"; do
  set -- $sc
  timeout -k 10 200 python bench.py --c5 --records 65536 --streams $1 --c5-chunk-mib $2 > $O/c5h.json 2>$O/c5h.err || { tail $O/c5h.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/c5h.json'));print('c5 host streams=$1 chunk=$2', d['value'])"
done
