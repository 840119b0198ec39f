"""Kernel time of one seal (or xor) launch at C2 under ENET_STREAM_DBG (tools/stream_probe.sh)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import ephemeralnet_amd as E  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--records", type=int, default=65536)
ap.add_argument("--record-bytes", type=int, default=4096)
ap.add_argument("--mode", default="aead")
ap.add_argument("--reps", type=int, default=200)
a = ap.parse_args()
n, L = a.records, a.record_bytes
dev = torch.device("cuda", 0)
pt = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device=dev)
keys = torch.randint(0, 256, (n * 32,), dtype=torch.uint8, device=dev)
nonces = torch.randint(0, 256, (n * 12,), dtype=torch.uint8, device=dev)
offs = torch.arange(0, (n + 1) * L, L, dtype=torch.int64, device=dev)
ct = torch.empty_like(pt)
tags = torch.empty(16 * n, dtype=torch.uint8, device=dev)
b = E.Batch(pt, offs, keys, nonces, total_bytes_hint=n * L, max_len_hint=L)
st = torch.cuda.current_stream(dev)


def f():
    if a.mode == "aead":
        E.aead_seal(b, ct, tags, stream=st)
    else:
        E.chacha20_xor(b, ct, stream=st)


for _ in range(300):
    f()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(st)
for _ in range(a.reps):
    f()
e1.record(st)
e1.synchronize()
us = e0.elapsed_time(e1) / a.reps * 1e3
dbg = int(os.environ.get("ENET_STREAM_DBG", "0"))
out = {"dbg": dbg, "mode": a.mode, "us": round(us, 2), "GBs_alg": round(n * (2 * L + 64) / us / 1e3, 1)}
if dbg & 256 and a.mode == "aead":
    # per-workgroup stamps (stream.hip): in-kernel clock = d(memtime) / d(memrealtime) * 100 MHz
    lanes = E.lanes_per_record(n, n * L, L)
    per_wg = 512 // lanes
    t = tags.view(torch.int64).cpu().view(-1, 2)[::per_wg][:, :].reshape(-1)
    w = tags.view(torch.int64).cpu().view(n, 2)
    firsts = torch.arange(0, n, per_wg)
    d = torch.stack([w[firsts, 0], w[firsts, 1], w[firsts + 1, 0], w[firsts + 1, 1]], 1).double()
    ghz = (d[:, 2] - d[:, 0]) / (d[:, 3] - d[:, 1]) * 0.1
    out["clock_ghz_median"] = round(float(ghz.median()), 3)
    out["clock_ghz_min"] = round(float(ghz.min()), 3)
    out["wg_us_median"] = round(float(((d[:, 3] - d[:, 1]) / 100.0).median()), 2)
print(json.dumps(out))
