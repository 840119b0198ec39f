set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_chunks_fused.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_chunks.log 2>&1 || { tail -40 gpurun_out/pytest_chunks.log; exit 1; }
tail -3 gpurun_out/pytest_chunks.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for ids in given content; do timeout -k 10 200 python bench.py --mode store --store-ids $ids --steps 100 --warmup 20 --no-cpu-baseline; done > gpurun_out/store.jsonl
cat gpurun_out/store.jsonl | python -c "import sys,json; [print(d['config']['chunk_ids'], d['value'], d['seal_ms'], d['open_ms']) for d in map(json.loads, sys.stdin)]"
