"""Per-stage timeline of the streaming kernel at C2 (stream.hip probe bit 16384): compute wave 0 of
every workgroup stamps the shader clock at its body start, after each stage barrier S0 and after
F1.  Prints the kernel time and, over workgroups, the median cycles of the prologue (start -> S0 of
stage 0), of each stage, and of the last stage (-> F1).  Run with ENET_STREAM_DBG=16384 (full) and
16385 (memory waves idle)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import ephemeralnet_amd as E  # noqa: E402

n, L = 65536, 4096
dev = torch.device("cuda", 0)
pt = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device=dev)
keys = torch.randint(0, 256, (n * 32,), dtype=torch.uint8, device=dev)
nonces = torch.randint(0, 256, (n * 12,), dtype=torch.uint8, device=dev)
offs = torch.arange(0, (n + 1) * L, L, dtype=torch.int64, device=dev)
ct = torch.empty_like(pt)
back = torch.empty_like(pt)
tags = torch.zeros(16 * n, dtype=torch.uint8, device=dev)
tags2 = torch.zeros_like(tags)
b = E.Batch(pt, offs, keys, nonces, total_bytes_hint=n * L, max_len_hint=L)
b2 = E.Batch(ct, offs, keys, nonces, total_bytes_hint=n * L, max_len_hint=L)
st = torch.cuda.current_stream(dev)
for i in range(300):
    E.aead_seal(b if i % 2 == 0 else b2, ct if i % 2 == 0 else back, tags if i % 2 == 0 else tags2, stream=st)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(st)
for i in range(100):
    E.aead_seal(b if i % 2 == 0 else b2, ct if i % 2 == 0 else back, tags if i % 2 == 0 else tags2, stream=st)
e1.record(st)
e1.synchronize()
us = e0.elapsed_time(e1) / 100 * 1e3
S = 16
lanes = E.lanes_per_record(n, n * L, L)
per_wg = 512 // lanes
w = tags2.view(torch.int64).cpu().numpy().reshape(-1)
firsts = np.arange(0, n, per_wg) * 2
st_ = np.stack([w[firsts + k] for k in range(S + 6)], 1).astype(np.int64)
rt0, c0, cb = st_[:, 0], st_[:, 1], st_[:, 2]
cs = st_[:, 3:3 + S + 1]            # S0(0..S-1), F1
ce, rt1 = st_[:, 4 + S], st_[:, 5 + S]
ghz = (ce - c0) / ((rt1 - rt0) * 10.0)
d = np.diff(cs, axis=1)
T0 = rt0.min()
med = lambda x: float(np.median(x))
out = {"dbg": int(os.environ.get("ENET_STREAM_DBG", "0")), "kernel_us": round(us, 2),
       "clock_ghz_median": round(med(ghz), 3),
       "wg_us_median": med((rt1 - rt0) / 100.0),
       "wg_start_us_p50_p99_max": [float(np.percentile((rt0 - T0) / 100.0, q)) for q in (50, 99, 100)],
       "wg_end_us_p1_p50_max": [float(np.percentile((rt1 - T0) / 100.0, q)) for q in (1, 50, 100)],
       "entry_to_body_cyc": med(cb - c0), "body_to_S0_cyc": med(cs[:, 0] - cb),
       "stage_cyc_median": [med(x) for x in d.T],
       "stage_cyc_p90": [float(np.percentile(x, 90)) for x in d.T],
       "F1_to_exit_cyc": med(ce - cs[:, -1])}
print(json.dumps(out))
