set -o pipefail
mkdir -p gpurun_out/p1
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_cpp_api.py tests/test_gpu_pipeline.py tests/test_frame_queue.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/p1/pytest.log 2>&1; rc=$?; tail -15 gpurun_out/p1/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 360 tools/host_path_probe 65536 4096 all > gpurun_out/p1/probe.jsonl 2> gpurun_out/p1/probe.err; rc=$?; cat gpurun_out/p1/probe.jsonl; tail -3 gpurun_out/p1/probe.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 tools/batch_bench all 3 > gpurun_out/p1/batch.jsonl 2> gpurun_out/p1/batch.err; rc=$?; cat gpurun_out/p1/batch.jsonl; tail -3 gpurun_out/p1/batch.err; exit $rc
