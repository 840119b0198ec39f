# A/B: HIP_FORCE_DEV_KERNARG (kernel arguments in device memory) on the C2 bench.
set -e
for k in 0 1; do
  HIP_FORCE_DEV_KERNARG=$k timeout -k 10 120 python bench.py --steps 300 --warmup 30 --no-cpu-baseline > gpurun_out/ka_$k.json 2>/dev/null
  python3 -c "import json; d=json.load(open('gpurun_out/ka_$k.json')); print('kernarg $k', d['value'], d['seal_ms'], d['open_ms'], d['ms_per_step'])"
done
