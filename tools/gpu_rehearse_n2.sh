#!/bin/bash
# The N > 1 torchrun path of bench.py rehearsed on the box's one GPU (gloo: every rank shares the
# card, the barrier / max-reduce / all_gather run on the host).  Shows every rank's placement
# (NUMA node, CPU set, CPU share), its C5 share's staging node and pinned bytes, the total pinned
# bytes over the ranks and the wall time.
# usage: bash tools/gpu_rehearse_n2.sh [TAG] [NPROC (default 2)]
# N > 2 runs with --no-e2e (each rank's C5 child only): the box allows 16 processes on its one GPU,
# and 8 ranks + 8 C5 children are exactly that (on an 8-GPU node each GPU has 2).
set -o pipefail
T=${1:-r05n2}
N=${2:-2}
mkdir -p gpurun_out/$T
t0=$(date +%s.%N)
ENET_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus $N --steps 50 --warmup 10 --no-cpu-baseline $( [ $N -gt 2 ] && echo --no-e2e ) > gpurun_out/$T/rehearsal.json 2> gpurun_out/$T/rehearsal.err; rc=$?
t1=$(date +%s.%N)
grep '^{"metric"' gpurun_out/$T/rehearsal.json | python -c "
import sys, json
d = json.loads(sys.stdin.read())
pr = d['dist']['per_rank']
tot = sum(((r.get('c5_host') or {}).get('process_pinned_bytes') or 0) for r in pr)
print(json.dumps({'world_size': d['dist']['world_size'], 'value': d['value'], 'wall_s': round($t1 - $t0, 1),
                  'total_process_pinned_bytes': tot, 'c5_host_gibs': d['host_resident'].get('c5_host_gibs'),
                  'per_rank': [{k: r.get(k) for k in ('rank', 'numa_node', 'cpus', 'cpu_budget', 'gibs', 'ok')} |
                               {'pinned_bytes': (r.get('c5_host') or {}).get('process_pinned_bytes'),
                                'staging_node': (r.get('c5_host') or {}).get('staging_node')} for r in pr]}))
" | tee gpurun_out/$T/summary.json
exit $rc
