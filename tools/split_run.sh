# Split-duplex check on the box: its parity tests, the chain probe, C5 / 64 KiB store bench lines,
# and the duplex compute-only model (tools/ubench_duplex.hip, built into oracle/_ref).
# usage: bash tools/split_run.sh TAG
set -euo pipefail
O=gpurun_out/${1:-split}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_duplex.py -x -q --timeout 120 --timeout-method thread -k "split or chunks or c5" > $O/pytest.log 2>&1 || { tail -50 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python tools/c5_overlap_probe.py > $O/probe.json 2> $O/probe.err && cat $O/probe.json
for a in "--c5-device --records 65536" "--c5-device --records 65536 --c5-overlap" "--mode store --records 32768 --record-bytes 65536" "--mode store"; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --warmup 3 $a > $O/b.json 2>> $O/b.err && python3 -c "import json;d=json.load(open('$O/b.json'));print('$a', d['value'], d.get('ms_per_step'))"
done
if [ -x oracle/_ref/ubench_duplex ]; then
  timeout -k 10 120 oracle/_ref/ubench_duplex > $O/ubench_duplex.jsonl 2>&1 && cat $O/ubench_duplex.jsonl
fi
