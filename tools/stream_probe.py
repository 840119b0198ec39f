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
ap.add_argument("--alt", action="store_true",
                help="alternate seal(pt -> ct) and seal(ct -> back), the bench's memory pattern "
                     "(each kernel reads what the previous one wrote; back-to-back launches of one "
                     "kernel re-read an input the 256 MiB Infinity Cache partly holds)")
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
b2 = E.Batch(ct, offs, keys, nonces, total_bytes_hint=n * L, max_len_hint=L)
back = torch.empty_like(pt)
tags2 = torch.empty_like(tags)
st = torch.cuda.current_stream(dev)
flip = [0]


def f():
    src, dst, tg = (b, ct, tags) if not (a.alt and flip[0]) else (b2, back, tags2)
    flip[0] ^= 1
    if a.mode == "aead":
        E.aead_seal(src, dst, tg, stream=st)
    else:
        E.chacha20_xor(src, dst, stream=st)


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
out = {"alt": a.alt, "dbg": dbg, "mode": a.mode, "us": round(us, 2), "GBs_alg": round(n * (2 * L + 64) / us / 1e3, 1)}
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
if dbg & 8192 and a.mode == "aead":
    # memory-wave trace (stream.hip): per (workgroup, memory wave) 64 barrier-exit stamps and 16
    # store issue times of stage 3
    t = tags.view(torch.int32).cpu().numpy().view("u4")[: 4 * 4 * 128].reshape(16, 128).astype("int64")
    import numpy as np
    ex, ar = t[:, :64], t[:, 64:128]
    own = ar[:, 1:] - ex[:, :-1]   # memory wave: previous barrier exit -> this arrival
    wait = ex[:, 1:] - ar[:, 1:]   # memory wave: arrival -> exit (waiting for the others)
    out["step_cycles_wg0_mw0"] = (ex[0, 1:] - ex[0, :-1]).tolist()
    out["mw_own_cycles_wg0_mw0"] = own[0].tolist()
    out["mw_wait_cycles_wg0_mw0"] = wait[0].tolist()
if dbg & 2048 and a.mode == "aead":
    import numpy as np
    lanes = E.lanes_per_record(n, n * L, L)
    nwg = n * lanes // 512
    w = (tags if not a.alt else tags2).view(torch.int64).cpu().numpy()[: nwg * 4]
    out["stage_end_dma_wait_cycles_per_wave_median"] = float(np.median(w))
    out["stage_end_dma_wait_cycles_per_wave_max"] = float(np.max(w))
print(json.dumps(out))
