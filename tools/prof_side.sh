# Kernel stats of the wire and store side modes (which kernel dominates each pipeline)
set -e
O=gpurun_out/side_prof
mkdir -p $O
export TMPDIR=/tmp
for m in wire store; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$m -o $m -- python3 bench.py --mode $m --no-cpu-baseline --steps 30 --warmup 5 > $O/$m.json 2> $O/$m.err
  f=$(find $O/$m -name "*kernel_stats.csv")
  python3 -c "
import csv,sys
for r in list(csv.DictReader(open('$f')))[:6]: print('$m', r['Name'][:70], r['Calls'], r['AverageNs'], r['Percentage'])"
done
