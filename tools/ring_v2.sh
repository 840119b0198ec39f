#!/bin/bash
# parity of the ring kernel's VGPR-load variant (tools build, ENET_STREAM_VAR=2), then the probes
set -uo pipefail
mkdir -p gpurun_out
ENET_LIB_PATH=$PWD/ephemeralnet_amd/libenet_crypto_tools.so ENET_STREAM_RING=1 ENET_STREAM_VAR=2 timeout -k 10 300 \
  python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "ring or uniform_batches" > gpurun_out/ring_v2_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/ring_v2_pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
bash tools/ring_probe.sh ${1:-rp3} "${2:-0 1 2 3}" "${3:-0 90 2}"
