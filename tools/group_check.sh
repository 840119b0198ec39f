#!/bin/bash
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -x -v --timeout 120 --timeout-method thread > gpurun_out/group.log 2>&1 || { tail -40 gpurun_out/group.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/group.log | tail -12
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
