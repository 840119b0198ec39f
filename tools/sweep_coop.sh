set -e
# lanes-per-record x COOP variant sweep over the uniform configs (seal+open GiB/s)
# usage: bash tools/sweep_coop.sh "1 2 3"
for coop in ${1:-1 2 3}; do
  for cfg in ${2:-"65536,4096,2" "65536,4096,4" "65536,4096,8" "1048576,1500,1" "1048576,1500,2" "32768,65536,4" "32768,65536,8" "32768,65536,16"}; do
    IFS=, read n L P <<< "$cfg"
    ENET_COOP=$coop timeout -k 10 100 python bench.py --no-cpu-baseline --records $n --record-bytes $L --lanes $P --steps 100 --warmup 20 > gpurun_out/sw_${coop}_${n}_${P}.json
    python -c "import json; d=json.load(open('gpurun_out/sw_${coop}_${n}_${P}.json')); print('coop', $coop, 'n', $n, 'L', $L, 'P', $P, d['value'], d['seal_ms'], d['open_ms'])"
  done
done
