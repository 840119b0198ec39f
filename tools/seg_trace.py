#!/usr/bin/env python3
"""Phase timeline of seg_uniform_aead_kernel from a TRACE probe library
(tools/build_seg_probes.sh TRACE; run with ENET_LIB_PATH=ephemeralnet_amd/libenet_probe_TRACE.so).
Stamps (100 MHz wall clock) per workgroup: 0 entry, 1 barrier A passed, 2 data wave 0 at barrier B,
3 power wave at barrier B (table done), 4 barrier B passed, 5 arrival counted, 6 tag (last
arriver).  Prints percentiles relative to the earliest entry, in microseconds."""
import collections
import ctypes
import json
import os

import numpy as np
import torch

import ephemeralnet_amd as E


def main() -> None:
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream(dev)
    L = 32 << 20
    T = (L >> 16 + 1) // 2  # workgroups: two 64 KiB tiles each (segments.hip kUTiles)
    g = torch.Generator(device=dev).manual_seed(5)
    pt = torch.randint(0, 256, (L,), dtype=torch.uint8, device=dev, generator=g)
    keys = torch.randint(0, 256, (32,), dtype=torch.uint8, device=dev, generator=g)
    nonces = torch.randint(0, 256, (12,), dtype=torch.uint8, device=dev, generator=g)
    offs = torch.tensor([0, L], dtype=torch.int64, device=dev)
    ct, back = torch.empty_like(pt), torch.empty_like(pt)
    tags = torch.empty(16, dtype=torch.uint8, device=dev)
    ok = torch.zeros(1, dtype=torch.uint8, device=dev)
    sb = E.Batch(pt, offs, keys, nonces, total_bytes_hint=L, max_len_hint=L)
    ob = E.Batch(ct, offs, keys, nonces, total_bytes_hint=L, max_len_hint=L)
    lib = ctypes.CDLL(os.environ["ENET_LIB_PATH"])
    buf = np.zeros(8192 * 8, dtype=np.uint64)
    out = {}
    for mode in ("seal", "open"):
        for _ in range(5):
            E.aead_seal(sb, ct, tags, stream=stream)
            E.aead_open(ob, back, tags, ok, stream=stream)
        torch.cuda.synchronize(dev)
        if mode == "seal":
            E.aead_seal(sb, ct, tags, stream=stream)
        else:
            E.aead_open(ob, back, tags, ok, stream=stream)
        torch.cuda.synchronize(dev)
        assert lib.enet_probe_trace_read(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(buf.size)) == 0
        st = buf[:8 * T].reshape(T, 8).astype(np.int64)
        t0 = st[:, 0].min()
        rel = (st - t0) / 100.0  # us
        row = {}
        for k, name in enumerate(["entry", "barrierA", "w0_at_B", "pw_at_B", "barrierB", "arrived"]):
            v = rel[:, k]
            row[name] = [round(float(np.percentile(v, q)), 2) for q in (0, 50, 90, 100)]
        last = int(np.argmax(st[:, 6]))
        row["last_arriver"] = {"tile": last, "tag_us": round(float(rel[last, 6]), 2),
                               "arrived_us": round(float(rel[last, 5]), 2)}
        row["durations_p50"] = {
            "entry_to_A": round(float(np.median(rel[:, 1] - rel[:, 0])), 2),
            "A_to_w0B": round(float(np.median(rel[:, 2] - rel[:, 1])), 2),
            "A_to_pwB": round(float(np.median(rel[:, 3] - rel[:, 1])), 2),
            "B_to_arrived": round(float(np.median(rel[:, 5] - rel[:, 4])), 2),
        }
        hw = st[:, 7]
        hwid, xcc = hw & 0xffffffff, hw >> 32
        cu = (xcc & 0xf) * 1000 + ((hwid >> 13) & 0x7) * 100 + ((hwid >> 12) & 1) * 16 + ((hwid >> 8) & 0xf)
        conc, per_cu = [], {}
        for t in range(T):
            per_cu.setdefault(int(cu[t]), []).append((rel[t, 0], rel[t, 5]))
        for iv in per_cu.values():
            ev = sorted([(a, 1) for a, _ in iv] + [(b, -1) for _, b in iv])
            c = m = 0
            for _, d in ev:
                c += d
                m = max(m, c)
            conc.append(m)
        row["cus_used"] = len(per_cu)
        row["wgs_per_cu"] = sorted(collections.Counter(len(v) for v in per_cu.values()).items())
        row["max_concurrent_wgs_per_cu"] = sorted(collections.Counter(conc).items())
        row["entry_hist_us"] = np.histogram(rel[:, 0], bins=11, range=(0, 22))[0].tolist()
        out[mode] = row
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
