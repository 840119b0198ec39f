export TMPDIR=/tmp
O=gpurun_out/dx5; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_duplex.py tests/test_gpu_frames_fused.py tests/test_gpu_chunks_fused.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for R in 64 256; do
  for cfg in "--mode wire --records 65536 --record-bytes 4096" "--mode wire --records 1048576 --record-bytes 1500" "--mode store --records 32768 --record-bytes 65536" "--mode store --records 65536 --record-bytes 4096"; do
    ENET_DUPLEX_RPW=$R timeout -k 10 120 python bench.py $cfg --steps 10 --warmup 3 --no-cpu-baseline > $O/w.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('$O/w.json'));print('rpw=$R $cfg', d['value'], d.get('seal_ms'), d.get('open_ms'))"
  done
  ENET_DUPLEX_RPW=$R timeout -k 10 120 python bench.py --c5-device --records 65536 --steps 5 --warmup 2 > $O/c5.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('$O/c5.json'));print('rpw=$R c5dev', d['value'], d['ms_per_step'])"
done
