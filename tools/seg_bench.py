#!/usr/bin/env python3
"""One 32 MiB record on the sequence-parallel tiles, nothing else: AEAD seal + open and ChaCha20
(XOR) pairs, for counter passes (tools/pmc.py --passes seg) and A/B timing.  Prints one JSON line."""
import json
import sys

import torch

import ephemeralnet_amd as E


def main(reps: int = 20) -> None:
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream(dev)
    L = 32 << 20
    g = torch.Generator(device=dev).manual_seed(77)
    pt = torch.randint(0, 256, (L,), dtype=torch.uint8, device=dev, generator=g)
    keys = torch.randint(0, 256, (32,), dtype=torch.uint8, device=dev, generator=g)
    nonces = torch.randint(0, 256, (12,), dtype=torch.uint8, device=dev, generator=g)
    offs = torch.tensor([0, L], dtype=torch.int64, device=dev)
    ct, back = torch.empty_like(pt), torch.empty_like(pt)
    tags = torch.empty(16, dtype=torch.uint8, device=dev)
    ok = torch.zeros(1, dtype=torch.uint8, device=dev)
    sb = E.Batch(pt, offs, keys, nonces, total_bytes_hint=L, max_len_hint=L)
    ob = E.Batch(ct, offs, keys, nonces, total_bytes_hint=L, max_len_hint=L)
    out = {}
    for mode in ("aead", "xor"):
        def pair():
            if mode == "aead":
                E.aead_seal(sb, ct, tags, stream=stream)
                E.aead_open(ob, back, tags, ok, stream=stream)
            else:
                E.chacha20_xor(sb, ct, stream=stream)
                E.chacha20_xor(ob, back, stream=stream)
        for _ in range(3):
            pair()
        torch.cuda.synchronize(dev)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record(stream)
        for _ in range(reps):
            pair()
        ev[1].record(stream)
        ev[1].synchronize()
        ms = ev[0].elapsed_time(ev[1]) / reps
        good = torch.equal(back, pt) and (mode == "xor" or int(ok.sum()) == 1)
        out[mode] = {"pair_us": round(ms * 1e3, 2), "gibs": round(L / (ms * 1e-3) / 2**30, 1), "ok": bool(good)}
    print(json.dumps(out))


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 20)
