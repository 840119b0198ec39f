"""PCIe ceiling on this box: pinned H2D, D2H and both directions at once, for whole 256 MiB
copies and for 16 MiB chunks on several streams (what the host-resident pipeline can reach)."""
import json
import time

import torch

dev = torch.device("cuda", 0)
N = 256 << 20
h_src = torch.empty(N, dtype=torch.uint8).pin_memory()
h_dst = torch.empty(N, dtype=torch.uint8).pin_memory()
d_a = torch.empty(N, dtype=torch.uint8, device=dev)
d_b = torch.empty(N, dtype=torch.uint8, device=dev)
h_src.fill_(3)
d_b.fill_(5)
torch.cuda.synchronize()


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps


s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
out = {}
out["h2d_GBs"] = N / timed(lambda: d_a.copy_(h_src, non_blocking=True)) / 1e9
out["d2h_GBs"] = N / timed(lambda: h_dst.copy_(d_b, non_blocking=True)) / 1e9


def both():
    with torch.cuda.stream(s1):
        d_a.copy_(h_src, non_blocking=True)
    with torch.cuda.stream(s2):
        h_dst.copy_(d_b, non_blocking=True)


out["bidir_total_GBs"] = 2 * N / timed(both) / 1e9
C = 16 << 20
for S in (2, 3, 4, 8):
    ss = [torch.cuda.Stream(dev) for _ in range(S)]

    def chunked():
        for c in range(N // C):
            with torch.cuda.stream(ss[c % S]):
                d_a[c * C:(c + 1) * C].copy_(h_src[c * C:(c + 1) * C], non_blocking=True)
                h_dst[c * C:(c + 1) * C].copy_(d_a[c * C:(c + 1) * C], non_blocking=True)

    out[f"chunk16M_roundtrip_{S}streams_GBs_each_dir"] = N / timed(chunked) / 1e9

# one stream per direction: every H2D chunk back to back on the up stream, the D2H of chunk c on
# the down stream after an event on the up stream (the copy engines never wait on each other's
# queue order), for 16 and 64 MiB chunks; K up / K down streams round-robin for K = 2
for C in (16 << 20, 64 << 20):
    for K in (1, 2):
        ups = [torch.cuda.Stream(dev) for _ in range(K)]
        downs = [torch.cuda.Stream(dev) for _ in range(K)]

        def split():
            for c in range(N // C):
                up, down = ups[c % K], downs[c % K]
                with torch.cuda.stream(up):
                    d_a[c * C:(c + 1) * C].copy_(h_src[c * C:(c + 1) * C], non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(up)
                down.wait_event(ev)
                with torch.cuda.stream(down):
                    h_dst[c * C:(c + 1) * C].copy_(d_a[c * C:(c + 1) * C], non_blocking=True)

        out[f"split_{C >> 20}M_{K}x2streams_GBs_each_dir"] = N / timed(split) / 1e9
print(json.dumps({k: round(v, 1) for k, v in out.items()}))
