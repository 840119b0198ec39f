#!/bin/bash
# duplex / chunk parity subset, then the C3 wire and C2 store kernels under a kernel trace
set -o pipefail
O=gpurun_out/${1:-r06g}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_chunks_fused.py tests/test_gpu_duplex.py tests/test_gpu_frames_fused.py tests/test_gpu_chunks_long.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3w -o c3w -- python3 bench.py --no-cpu-baseline --no-power --mode wire --records 1048576 --record-bytes 1500 --steps 10 --warmup 3 > $O/c3w.json 2> $O/c3w.err
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_st -o st -- python3 bench.py --no-cpu-baseline --no-power --mode store --steps 20 --warmup 5 > $O/st.json 2> $O/st.err
grep duplex $O/prof_c3w/*kernel_stats.csv $O/prof_st/*kernel_stats.csv | cut -d, -f1-4
