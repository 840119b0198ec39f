set -e
mkdir -p gpurun_out
for a in "--steps 20 --warmup 2" "--steps 50 --warmup 10" "--steps 20 --warmup 2 --prewarm-s 0"; do
  timeout -k 10 200 python bench.py $a --no-cpu-baseline > gpurun_out/pw.json
  python -c "import json; d=json.load(open('gpurun_out/pw.json')); print('$a', d['value'], d['ms_per_step'], d['prewarm_steps'])"
done
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/pw_tr.json 2> gpurun_out/pw_tr.err
python -c "import json; d=json.load(open('gpurun_out/pw_tr.json')); print('torchrun', d['value'], d['ms_per_step'], d['prewarm_steps'])"
