"""Host-resident C2 (bench.host_c2) with the library loaded before or after torch: which HIP
runtime (torch's bundled one or /opt/rocm's) the process ends up with, and the e2e rate.
usage (on the box): python tools/e2e_probe.py torch_first|lib_first"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
order = sys.argv[1] if len(sys.argv) > 1 else "torch_first"
if order == "torch_first":
    import torch  # noqa: F401
import ephemeralnet_amd as E  # noqa: E402
E.lib()
import bench  # noqa: E402
import torch  # noqa: E402,F811


def loaded(name):
    with open("/proc/self/maps") as f:
        return sorted({ln.split()[-1] for ln in f if name in ln})


out = {"order": order, "hip": loaded("libamdhip64"), "hsa": loaded("libhsa-runtime64")}
for chunk, slots in ((32, 4), (0, 0)):
    r = bench.host_c2(0, 65536, 4096, 3, chunk, slots)
    out[f"c2_{chunk}_{slots}"] = round(r["gibs"], 2)
print(json.dumps(out), flush=True)
