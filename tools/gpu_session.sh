#!/bin/bash
# The round-5 measurement recipes behind profiles/r05*_ (one gpurun call each), run on the box from
# the repo root:  bash tools/gpu_session.sh <recipe> [tag]
#   verify     GPU suite, smoke, N = 2 torchrun rehearsal, default bench line
#   queue      frame queue: device (view / reuse / ticket / async) vs host engine, 16 threads x
#              256 / 1 024 in flight, two rounds, on the GPU's node
#   queue-prof the same under the tools build's per-phase TSC profile (ENET_QUEUE_PROF=1), plus
#              a rocprofv3 kernel trace of the queue bench
#   crossover  device vs host by threads (1 / 4 / 16) x frames in flight (4 .. 256)
#   auto       AUTO routing by backlog vs device vs host, 16 threads x 16 .. 1 024 in flight
#              (WARMUP=<s>: an untimed leg each way first)
#   mode-diag  host mode 3 vs 4 by host-buffer variant (tools/mode_diag.py) + traced C2 per mode
#   c5-full    C5 host-resident at its full BASELINE size, twice
#   variance   the default bench line five times on one box
#   inflight   device queue by device passes in flight (workers) x frames in flight per thread
#   latency    the reference's scalar signatures through this library, policy auto
#              (oracle/_ref/scalar_latency_gpu: median of 200 calls, then 16 threads)
#   seal       host engine frame seal: stitched vs two-pass by size (tools/seal_variants,
#              tools/seal_bench), then the blocking host-engine queue rows (1 and 16 threads)
#   sessions   the reference's thread-per-session load (SessionManager.cpp:331-332, 337-388, 822):
#              T session threads, each with ONE blocking frame in flight (queue_bench sync), device
#              queue vs host engine vs auto, T = ${THREADS:-64 256 768}, two rounds
#   chunks     long-chunk GPU tests (host-hash route, tiles) and the long-record side leg
#   long-prof  the long-record side leg (1 x 32 MiB, 8 x 1 MiB; bench.py --long-only) plain and
#              under a rocprofv3 kernel trace (per-kernel durations, launch gaps)
# Round-wide evidence (kernel stats, PMC, side configs): tools/gpu_round.sh.
set -euo pipefail
R=${1:?recipe}
T=${2:-r05_$R}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
node_cpus() {
  local node
  node=$(python -c "from ephemeralnet_amd import topo; print(topo.gpu_numa_node(0))")
  cat /sys/devices/system/node/node$node/cpulist
}
qsummary() {
  python - "$1" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print(d["policy"], d["mode"], d["threads"], d["window"],
          "seal %.2fM open %.2fM" % (d["seal_frames_per_s"] / 1e6, d["open_frames_per_s"] / 1e6),
          "cpu %.2f %.2f" % (d["seal_cpu_us_per_frame"], d["open_cpu_us_per_frame"]),
          "pass", d["tx_frames_per_pass"], "evict", d["tx_evicted"], d["rx_evicted"], "ok", d["ok"])
PY
}
case "$R" in
verify)
  step pytest
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
  tail -2 $O/pytest_gpu.log
  step smoke
  timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
  tail -1 $O/smoke.log
  step rehearse n2
  timeout -k 10 500 bash tools/gpu_rehearse_n2.sh $T/n2 > $O/n2.log 2>&1 || { tail -20 $O/n2.log; exit 1; }
  step bench
  timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
  cut -c1-400 $O/bench.json ;;
queue)
  CPUS=$(node_cpus); : > $O/queue_bench.jsonl
  for r in 1 2; do
    for a in "device view 16 256" "device reuse 16 256" "device ticket 16 256" "device async 16 256" \
             "device view 16 1024" "host view 16 256" "host sync 16"; do
      timeout -k 10 60 taskset -c $CPUS tools/queue_bench $a >> $O/queue_bench.jsonl 2>> $O/queue_bench.err
    done
  done
  qsummary $O/queue_bench.jsonl ;;
queue-prof)
  CPUS=$(node_cpus); : > $O/prof.txt
  for w in 256 1024; do
    echo "== window $w" >> $O/prof.txt
    ENET_QUEUE_PROF=1 timeout -k 10 60 taskset -c $CPUS tools/queue_bench_tools device view 16 $w 1.5 > $O/one.json 2> $O/one.err
    grep -v amdgpu.ids $O/one.err >> $O/prof.txt || true
  done
  cat $O/prof.txt
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_queue -o queue -- tools/queue_bench device view 16 256 1.0 > $O/prof_queue.json 2> $O/prof_queue.err
  find $O/prof_queue -name "*kernel_stats.csv" -exec head -5 {} \; ;;
crossover)
  CPUS=$(node_cpus); : > $O/crossover.jsonl
  for t in 1 4 16; do for w in 4 16 32 64 128 256; do for pol in device host; do
    timeout -k 10 60 taskset -c $CPUS tools/queue_bench $pol view $t $w 0.6 >> $O/crossover.jsonl 2>> $O/crossover.err
  done; done; done
  qsummary $O/crossover.jsonl ;;
auto)
  CPUS=$(node_cpus); : > $O/auto.jsonl
  for w in 16 64 128 256 512 1024; do for pol in auto host device; do
    QUEUE_BENCH_WARMUP=${WARMUP:-0} timeout -k 10 60 taskset -c $CPUS tools/queue_bench $pol view 16 $w 0.8 >> $O/auto.jsonl 2>> $O/auto.err
  done; done
  qsummary $O/auto.jsonl ;;
mode-diag)
  : > $O/mode_diag.jsonl
  timeout -k 10 300 python tools/mode_diag.py torch >> $O/mode_diag.jsonl 2> $O/mode_diag.err
  cat $O/mode_diag.jsonl
  for m in splitk zcout; do
    ENET_HOST_TRACE=1 ENET_HOST_MODE=$m timeout -k 10 120 python -c "
import torch, sys
torch.zeros(1, device='cuda')
sys.path.insert(0, '.')
import bench, ephemeralnet_amd as E
E.lib()
print(bench.host_c2(0, 65536, 4096, 2)['gibs'])" > $O/trace_torch_$m.txt 2>&1
  done
  tail -n 3 $O/trace_torch_*.txt ;;
c5-full)
  : > $O/c5.jsonl
  for r in 1 2; do
    timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --c5 >> $O/c5.jsonl 2>> $O/c5.err
  done
  cut -c1-300 $O/c5.jsonl ;;
variance)
  : > $O/bench_repeat.jsonl
  for r in 1 2 3 4 5; do
    timeout -k 10 300 python bench.py --no-cpu-baseline $( [ $r -gt 1 ] && echo --no-host ) >> $O/bench_repeat.jsonl 2>> $O/bench_repeat.err
  done
  python -c "
import json
for l in open('$O/bench_repeat.jsonl'):
    d = json.loads(l); print(d['value'], d['seal_ms'], d['open_ms'], d['roofline']['frac'], (d.get('power') or {}).get('package_w'))" ;;
inflight)
  CPUS=$(node_cpus); : > $O/inflight.jsonl
  for r in 1 2; do for w in ${WINDOWS:-128 256 1024}; do for inf in ${INFLIGHT:-4 8 16}; do
    timeout -k 10 60 taskset -c $CPUS tools/queue_bench device view 16 $w 1.5 1500 $inf >> $O/inflight.jsonl 2>> $O/inflight.err
  done; done; done
  python - $O/inflight.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print(d["window"], d["inflight"], "seal %.2fM open %.2fM" % (d["seal_frames_per_s"] / 1e6, d["open_frames_per_s"] / 1e6),
          "cpu %.2f %.2f" % (d["seal_cpu_us_per_frame"], d["open_cpu_us_per_frame"]),
          "pass", d["tx_frames_per_pass"], "pass_us", d["tx_pass_us"], "kernel_us", d["tx_kernel_us"], "evict", d["tx_evicted"])
PY
  ;;
latency)
  timeout -k 10 240 oracle/_ref/scalar_latency_gpu 200 auto 16 > $O/latency_auto.jsonl 2> $O/latency_auto.err
  cut -c1-200 $O/latency_auto.jsonl ;;
seal)
  CPUS=$(node_cpus); : > $O/host_queue.jsonl
  lscpu | grep -i "model name" > $O/cpu.txt
  timeout -k 10 120 taskset -c $CPUS tools/seal_variants 0 32 64 98 128 200 300 400 480 600 1000 1500 2100 4096 16384 65536 > $O/seal_variants.jsonl
  timeout -k 10 60 taskset -c $CPUS tools/seal_bench 98 600 1500 4096 65536 > $O/seal_bench.jsonl
  for r in 1 2; do for a in "host sync 1" "host sync 16" "host view 16 256"; do
    timeout -k 10 60 taskset -c $CPUS tools/queue_bench $a >> $O/host_queue.jsonl 2>> $O/host_queue.err
  done; done
  cat $O/cpu.txt $O/seal_variants.jsonl $O/seal_bench.jsonl
  qsummary $O/host_queue.jsonl ;;
sessions)
  CPUS=$(node_cpus); : > $O/sessions.jsonl
  for r in 1 2; do for t in ${THREADS:-64 256 768}; do for pol in ${POLICIES:-device host auto}; do
    QUEUE_BENCH_WARMUP=${WARMUP:-0.3} timeout -k 10 90 taskset -c $CPUS tools/queue_bench $pol sync $t 1 1.0 >> $O/sessions.jsonl 2>> $O/sessions.err
  done; done; done
  qsummary $O/sessions.jsonl ;;
long-prof)
  timeout -k 10 180 python bench.py --long-only > $O/long.json 2> $O/long.err
  cut -c1-600 $O/long.json
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_long -o long -- python bench.py --long-only > $O/long_prof.json 2> $O/long_prof.err
  find $O/prof_long -name "*kernel_stats.csv" -exec cat {} \; ;;
chunks)
  step pytest
  timeout -k 10 400 python -u -m pytest tests/test_gpu_chunks_long.py tests/test_gpu_segments.py -x -v --timeout 200 --timeout-method thread > $O/pytest_chunks.log 2>&1 || { tail -60 $O/pytest_chunks.log; exit 1; }
  tail -3 $O/pytest_chunks.log
  step long leg
  timeout -k 10 240 python bench.py --long-only > $O/long.json 2> $O/long.err
  cut -c1-1500 $O/long.json ;;
*)
  echo "unknown recipe $R" >&2; exit 2 ;;
esac
step done
