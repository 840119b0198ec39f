# duplex evidence: kernel-trace stats + PMC traffic for C5 device-resident and C3 wire frames
export TMPDIR=/tmp
O=gpurun_out/dxprof; mkdir -p $O
timeout -k 10 300 python tools/pmc.py --out $O/pmc_c5 --summary $O/pmc_c5_r02.json --config '{"workload": "C5 device", "records": 65536}' -- python3 bench.py --c5-device --records 65536 --steps 2 --warmup 1 > /dev/null || exit 1
timeout -k 10 300 python tools/pmc.py --out $O/pmc_c3w --summary $O/pmc_c3wire_r02.json --config '{"workload": "C3 wire frames", "records": 1048576, "record_bytes": 1500}' -- python3 bench.py --mode wire --records 1048576 --record-bytes 1500 --steps 2 --warmup 1 --no-cpu-baseline --prewarm-s 0 > /dev/null || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ks_c5 -o c5 -- python3 bench.py --c5-device --records 65536 --steps 5 --warmup 2 > $O/c5.json || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ks_c3w -o c3w -- python3 bench.py --mode wire --records 1048576 --record-bytes 1500 --steps 10 --warmup 3 --no-cpu-baseline > $O/c3w.json || exit 1
find $O -name "*kernel_stats.csv" | head
