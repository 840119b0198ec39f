#!/bin/bash
# Measurement programs that no test, smoke() or bench.py default line needs (run here, on the CPU,
# before a gpurun call whose recipe uses them; the binaries travel with the tree):
#   tools/seal_bench, tools/seal_variants      host engine frame seal (gpu_session.sh seal)
#   tools/queue_bench_tools, queue_stress_tools the queue programs over the tools build
#                                               (gpu_session.sh queue-prof, tools/stage_ab.sh)
set -euo pipefail
cd "$(dirname "$0")/.."
python -c "from ephemeralnet_amd import build as B; B.build(verbose=False); B.build(verbose=False, tools=True)"
I="-I include"; L="-L ephemeralnet_amd -Wl,-rpath,\$ORIGIN/../ephemeralnet_amd"
g++ -std=c++20 -O2 $I tools/seal_bench.cpp -o tools/seal_bench $L -lenet_crypto
g++ -std=c++20 -O3 $I tools/seal_variants.cpp -o tools/seal_variants
g++ -std=c++20 -O2 -pthread $I tools/queue_bench.cpp -o tools/queue_bench_tools $L -lenet_crypto_tools
g++ -std=c++20 -O2 -pthread $I tests/cpp/queue_stress.cpp -o tools/queue_stress_tools $L -lenet_crypto_tools
echo "tools built"
