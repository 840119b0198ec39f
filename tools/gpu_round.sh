#!/bin/bash
# One GPU session producing the round's evidence under gpurun_out/r$R/: GPU parity suite, the
# default bench line, side configs/modes, the torchrun launch path, rocprofv3 kernel stats, and
# PMC passes (C2 and C3).
# usage (on the box, from the repo root): bash tools/gpu_round.sh 01 [a|b|all]
# (a = parity suite, bench lines and side configs; b = rocprof stats and PMC: two gpurun calls)
set -euo pipefail
R=${1:-01}
PART=${2:-all}
O=gpurun_out/r$R
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
if [ "$PART" != b ]; then
step pytest
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -2 $O/pytest_gpu.log
step smoke
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
step bench default
timeout -k 10 240 python bench.py > $O/bench.json 2> $O/bench.err
cat $O/bench.json
step torchrun path
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 50 --warmup 10 --no-cpu-baseline > $O/bench_torchrun.json 2> $O/bench_torchrun.err
cat $O/bench_torchrun.json
step side configs
: > $O/side.jsonl
for args in "--records 1048576 --record-bytes 1500" "--records 32768 --record-bytes 65536" \
            "--mode xor" "--mode wire --cpu-seconds 5" "--mode store --store-ids given" "--mode store --store-ids content" "--mode pow --cpu-seconds 5" \
            "--mode pow --pow-schedule 0 --no-cpu-baseline" "--e2e" "--c5" \
            "--mode wire --records 1048576 --record-bytes 1500" "--mode store --records 32768 --record-bytes 65536" \
            "--c5-device --records 65536" "--c5-device --records 65536 --c5-overlap" \
            "--c5-device --records 65536 --c5-order none"; do
  step "  $args"
  timeout -k 10 400 python bench.py --steps 100 --warmup 20 $(case "$args" in *pow*|*1048576*|*c5*|*32768*) echo "--steps 10 --warmup 3";; esac) $(case "$args" in *pow*|*wire*) ;; *) echo --no-cpu-baseline;; esac) $args >> $O/side.jsonl 2>> $O/side.err
done
step scalar latency
for pol in auto device; do
  timeout -k 10 240 oracle/_ref/scalar_latency_gpu 200 $pol 16 > $O/latency_$pol.jsonl 2> $O/latency_$pol.err
done
timeout -k 10 240 oracle/_ref/scalar_latency_ref 200 x 16 > $O/latency_ref.jsonl 2> $O/latency_ref.err
step c5 chain probe
timeout -k 10 300 python tools/c5_overlap_probe.py > $O/c5_probe.json 2> $O/c5_probe.err
fi
if [ "$PART" != a ]; then
step rocprof stats
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --no-cpu-baseline --no-power --steps 50 --warmup 10 > $O/prof_bench.json 2> $O/prof.err
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o c3 -- python3 bench.py --no-cpu-baseline --no-power --records 1048576 --record-bytes 1500 --steps 10 --warmup 3 > $O/prof_c3.json 2>> $O/prof.err
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_fused -o fused -- python3 bench.py --no-cpu-baseline --no-power --mode store --steps 20 --warmup 5 > $O/prof_fused.json 2>> $O/prof.err
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3w -o c3w -- python3 bench.py --no-cpu-baseline --no-power --mode wire --records 1048576 --record-bytes 1500 --steps 10 --warmup 3 > $O/prof_c3w.json 2>> $O/prof.err
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o c5 -- python3 bench.py --no-power --c5-device --records 65536 --steps 5 --warmup 2 > $O/prof_c5.json 2>> $O/prof.err
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_st64 -o st64 -- python3 bench.py --no-cpu-baseline --no-power --mode store --records 32768 --record-bytes 65536 --steps 5 --warmup 2 > $O/prof_st64.json 2>> $O/prof.err
find $O/prof $O/prof_c3 $O/prof_fused $O/prof_c3w $O/prof_c5 $O/prof_st64 -name "*stats*"
step pmc
timeout -k 10 600 python tools/pmc.py --out $O/pmc --summary $O/pmc_summary.json --config "{\"records\": 65536, \"record_bytes\": 4096}" -- python3 bench.py --no-cpu-baseline --no-power --steps 3 --warmup 1 > $O/pmc.log 2>&1
timeout -k 10 600 python tools/pmc.py --out $O/pmc_c3 --summary $O/pmc_c3_summary.json --config "{\"records\": 1048576, \"record_bytes\": 1500}" -- python3 bench.py --no-cpu-baseline --no-power --records 1048576 --record-bytes 1500 --steps 2 --warmup 1 > $O/pmc_c3.log 2>&1
timeout -k 10 600 python tools/pmc.py --out $O/pmc_c3w --summary $O/pmc_c3w_summary.json --config "{\"mode\": \"wire\", \"records\": 1048576, \"record_bytes\": 1500}" -- python3 bench.py --no-cpu-baseline --no-power --mode wire --records 1048576 --record-bytes 1500 --steps 2 --warmup 1 > $O/pmc_c3w.log 2>&1
# calibration of FETCH_SIZE for the duplex kernel's per-lane 16-byte access pattern: chunks of
# 4096 B at 128-byte-aligned starts read and write exactly 2 x 256 MiB + ids/keys per launch
timeout -k 10 600 python tools/pmc.py --out $O/pmc_st --summary $O/pmc_st_summary.json --config "{\"mode\": \"store\", \"records\": 65536, \"record_bytes\": 4096}" -- python3 bench.py --no-cpu-baseline --no-power --mode store --steps 2 --warmup 1 > $O/pmc_st.log 2>&1
timeout -k 10 600 python tools/pmc.py --out $O/pmc_c5 --summary $O/pmc_c5_summary.json --config "{\"workload\": \"C5 device\", \"records\": 65536}" -- python3 bench.py --no-power --c5-device --records 65536 --steps 2 --warmup 1 > $O/pmc_c5.log 2>&1
fi
step done
