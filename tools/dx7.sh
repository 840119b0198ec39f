export TMPDIR=/tmp
O=gpurun_out/dx7; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_duplex.py tests/test_gpu_frames_fused.py tests/test_gpu_chunks_fused.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "duplex or fused or frames or chunk or hmac or ragged or mixed" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for cfg in "--mode wire --records 1048576 --record-bytes 1500" "--mode store --records 65536 --record-bytes 4096" "--mode wire --records 65536 --record-bytes 4096"; do
  timeout -k 10 120 python bench.py $cfg --steps 10 --warmup 3 --no-cpu-baseline > $O/w.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('$O/w.json'));print('$cfg', d['value'], d.get('seal_ms'), d.get('open_ms'))"
done
timeout -k 10 120 python bench.py --c5-device --records 65536 --steps 5 --warmup 2 > $O/c5.json 2>/dev/null || exit 1
python3 -c "import json;d=json.load(open('$O/c5.json'));print('c5dev', d['value'], d['ms_per_step'])"
timeout -k 10 100 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d $O/pmc -o lds -- python3 bench.py --mode wire --records 1048576 --record-bytes 1500 --steps 1 --warmup 1 --no-cpu-baseline --prewarm-s 0 > /dev/null 2>&1 || exit 1
python3 - <<'PY'
import csv,glob,collections
d=collections.defaultdict(list)
for f in glob.glob('gpurun_out/dx7/pmc/**/lds_counter_collection.csv',recursive=True):
    for r in csv.DictReader(open(f)):
        if 'duplex' in r['Kernel_Name']: d[(r['Kernel_Name'][:40],r['Counter_Name'])].append(float(r['Counter_Value']))
for k,v in sorted(d.items()): print(k, sum(v)/len(v))
PY
