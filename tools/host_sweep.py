"""Host-resident pipeline sweep (round 4): C2 e2e and the C5 per-GPU share through
enet_pipeline_* for every host mode x slots x chunk size, in one process (bench.py's own
measurement functions).  One JSON line per configuration.
usage (on the box): python tools/host_sweep.py [c2|c5|all]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402
import ephemeralnet_amd as E  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "all"
MODES = {"zc": 0, "sdma": 1, "split": 2, "splitk": 3, "zcout": 4}
if which in ("c2one", "c5one"):  # one configuration from the environment (for a trace)
    m, slots, chunk = os.environ.get("ONE", "splitk,3,256").split(",")
    E.set_host_mode(MODES[m])
    if which == "c2one":
        r = bench.host_c2(0, 65536, 4096, 3, int(chunk), int(slots))
    else:
        r = bench.c5_host_timed(1, 0, 0, None, 65536, int(chunk), int(slots), steps=2)
    print(json.dumps({"case": which, "mode": m, "slots": int(slots), "chunk_mib": int(chunk),
                      "gibs": round(r["gibs"], 2)}), flush=True)
    sys.exit(0)
if which in ("c2", "all"):
    for m in os.environ.get("SWEEP_MODES", "split,splitk,zc").split(","):
        for slots in (3, 4):
            for chunk in (16, 32, 64):
                E.set_host_mode(MODES[m])
                r = bench.host_c2(0, 65536, 4096, 3, chunk, slots)
                print(json.dumps({"case": "C2 e2e", "mode": m, "slots": slots, "chunk_mib": chunk,
                                  "gibs": round(r["gibs"], 2)}), flush=True)
if which in ("c5", "all"):
    for m, slots, chunk in [("splitk", 3, 128), ("splitk", 3, 256), ("splitk", 4, 128), ("splitk", 4, 256),
                            ("splitk", 3, 512), ("splitk", 6, 64), ("splitk", 6, 128)]:
        E.set_host_mode(MODES[m])
        r = bench.c5_host_timed(1, 0, 0, None, 65536, chunk, slots)
        print(json.dumps({"case": "C5 host share", "mode": m, "slots": slots, "chunk_mib": chunk,
                          "gibs": round(r["gibs"], 2)}), flush=True)
