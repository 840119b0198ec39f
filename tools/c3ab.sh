# A/B of the uniform-batch staging variants over record lengths (1 M records, one lane each):
# default staging (line staging for lengths that are not 128-byte multiples) vs ENET_COOP=4
# (plain run staging).  usage: bash tools/c3ab.sh
set -e
for L in 1500 1504 1472 1400 1536; do
  for v in default 4; do
    if [ $v = default ]; then unset ENET_COOP; else export ENET_COOP=$v; fi
    timeout -k 10 120 python bench.py --records 1048576 --record-bytes $L --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/ab_${L}_$v.json 2>/dev/null
    python3 -c "import json; d=json.load(open('gpurun_out/ab_${L}_$v.json')); print('$L', '$v', d['value'], d['seal_ms'], d['open_ms'])"
  done
done
