set -e
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_pipe.log 2>&1 || { tail -30 gpurun_out/pytest_pipe.log; exit 1; }
tail -2 gpurun_out/pytest_pipe.log
for sc in "4 16" "3 16" "4 24"; do
  set -- $sc
  timeout -k 10 120 python bench.py --e2e --streams $1 --chunk-mib $2 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('e2e streams',$1,'chunk',$2,d['value'],d['seal_GiBs'],d['open_GiBs'])"
done
for sc in "4 64" "4 128" "3 256" "2 128"; do
  set -- $sc
  timeout -k 10 120 python bench.py --c5 --streams $1 --c5-chunk-mib $2 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5 streams',$1,'chunk',$2,d['value'])"
done
