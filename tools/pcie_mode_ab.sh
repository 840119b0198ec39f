#!/bin/bash
# Host-resident pipelines (C2 --e2e, C5 --c5) with the HIP copy engine choice: SDMA (default) vs
# blit kernels (HSA_ENABLE_SDMA=0), interleaved, plus the raw PCIe probe under both.
set -euo pipefail
O=gpurun_out/${1:-pcie_ab}
mkdir -p $O
: > $O/ab.jsonl
for i in 1 2; do
  for sd in 1 0; do
    for args in "--e2e" "--c5"; do
      HSA_ENABLE_SDMA=$sd timeout -k 10 300 python bench.py --no-cpu-baseline --no-power --steps 3 --warmup 1 $args > $O/one.json 2>> $O/ab.err
      python -c "import json; d=json.load(open('$O/one.json')); d['sdma']=$sd; print(json.dumps(d))" >> $O/ab.jsonl
      python -c "import json; d=json.load(open('$O/one.json')); print('sdma=$sd', '$args', d['value'])"
    done
  done
done
for sd in 1 0; do HSA_ENABLE_SDMA=$sd timeout -k 10 200 python tools/pcie_probe.py > $O/probe_sdma$sd.json 2>> $O/ab.err; echo "probe sdma=$sd"; cat $O/probe_sdma$sd.json | head -c 600; echo; done
