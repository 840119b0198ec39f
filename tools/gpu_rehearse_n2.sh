set -o pipefail
mkdir -p gpurun_out/r04n2
ENET_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/r04n2/rehearsal.json 2> gpurun_out/r04n2/rehearsal.err; rc=$?
grep '^{"metric"' gpurun_out/r04n2/rehearsal.json | python -c "import sys, json; d=json.loads(sys.stdin.read()); print(d['value'], json.dumps(d['dist']), json.dumps(d['host_resident']))"
exit $rc
