"""Where the C5 device-resident time goes: the serial HMAC chain of the longest records vs the
total work, and whether two duplex kernels on two streams overlap.  Prints one JSON line.

  chain_us[n]   seal of n records of 64 KiB (n = 64: one workgroup, the bare chain)
  seal_us       seal of the C5 batch (65 536 mixed records, length-sorted)
  open_us       open of it
  pair_us       seal of batch B beside open of batch A (two streams), both issued at once
  two_seal_us   two seals of the C5 batch on two streams at once
"""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import ephemeralnet_amd as E  # noqa: E402


def batch(lens, dev, seed):
    offs = torch.from_numpy(np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)).to(dev)
    total = int(lens.sum())
    n = len(lens)
    g = torch.Generator(device=dev).manual_seed(seed)
    pt = torch.randint(0, 256, (total,), dtype=torch.uint8, device=dev, generator=g)
    keys = torch.randint(0, 256, (n * 32,), dtype=torch.uint8, device=dev, generator=g)
    nonces = torch.randint(0, 256, (n * 12,), dtype=torch.uint8, device=dev, generator=g)
    dl = offs[1:] - offs[:-1]
    order = torch.argsort(dl, descending=True).to(torch.int32)
    b = E.Batch(pt, offs, keys, nonces, order=order, total_bytes_hint=total, max_len_hint=int(lens.max()))
    ct = torch.empty_like(pt)
    back = torch.empty_like(pt)
    tags = torch.empty(16 * n, dtype=torch.uint8, device=dev)
    macs = torch.empty(32 * n, dtype=torch.uint8, device=dev)
    ok = torch.empty(n, dtype=torch.uint8, device=dev)
    return dict(b=b, ct=ct, back=back, tags=tags, macs=macs, ok=ok, n=n, offs=offs, keys=keys,
                nonces=nonces, order=order, pt=pt)


def seal(x, s=None):
    E.aead_hmac_seal(x["b"], x["ct"], x["tags"], x["macs"], stream=s)


def opn(x, s=None):
    bo = E.Batch(x["ct"], x["offs"], x["keys"], x["nonces"], order=x["order"],
                 total_bytes_hint=x["b"].total_bytes_hint, max_len_hint=x["b"].max_len_hint)
    E.aead_hmac_open(bo, x["back"], x["tags"], x["macs"], x["ok"], stream=s)


def timed(fn, reps=5):
    torch.cuda.synchronize()
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    dev = torch.device("cuda", 0)
    out = {"chain_us": {}}
    for n in (64, 1024, 8192):
        x = batch(np.full(n, 65536, dtype=np.int64), dev, 3)
        out["chain_us"][n] = round(timed(lambda: seal(x)), 1)
    rng = np.random.default_rng(5)
    lens = np.exp(rng.uniform(np.log(512), np.log(65536), 65536)).astype(np.int64)
    A = batch(lens, dev, 11)
    B = batch(lens, dev, 12)
    seal(A)
    torch.cuda.synchronize()
    out["seal_us"] = round(timed(lambda: seal(B)), 1)
    out["open_us"] = round(timed(lambda: opn(A)), 1)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    main_s = torch.cuda.current_stream(dev)

    def pair():
        s1.wait_stream(main_s)
        s2.wait_stream(main_s)
        seal(B, s1.cuda_stream)
        opn(A, s2.cuda_stream)
        main_s.wait_stream(s1)
        main_s.wait_stream(s2)

    out["pair_us"] = round(timed(pair), 1)

    def two_seal():
        s1.wait_stream(main_s)
        s2.wait_stream(main_s)
        seal(B, s1.cuda_stream)
        seal(A, s2.cuda_stream)
        main_s.wait_stream(s1)
        main_s.wait_stream(s2)

    out["two_seal_us"] = round(timed(two_seal), 1)
    # two one-workgroup chains (64 x 64 KiB each) on two streams: different CUs, no contention
    # -- 2.6 ms if the kernels run concurrently, 5.2 ms if they serialize
    C1 = batch(np.full(64, 65536, dtype=np.int64), dev, 21)
    C2 = batch(np.full(64, 65536, dtype=np.int64), dev, 22)

    def two_chains():
        s1.wait_stream(main_s)
        s2.wait_stream(main_s)
        seal(C1, s1.cuda_stream)
        seal(C2, s2.cuda_stream)
        main_s.wait_stream(s1)
        main_s.wait_stream(s2)

    out["two_chains_us"] = round(timed(two_chains), 1)
    # the same with HIP streams created by hand (non-blocking)
    import ctypes as C
    hip = C.CDLL("libamdhip64.so")
    h1, h2 = C.c_void_p(), C.c_void_p()
    hip.hipStreamCreateWithFlags(C.byref(h1), 1)
    hip.hipStreamCreateWithFlags(C.byref(h2), 1)

    def two_chains_hip():
        torch.cuda.synchronize()
        seal(C1, h1.value)
        seal(C2, h2.value)
        hip.hipStreamSynchronize(h1)
        hip.hipStreamSynchronize(h2)

    import time
    two_chains_hip()
    t0 = time.perf_counter()
    for _ in range(5):
        two_chains_hip()
    out["two_chains_hipstream_us"] = round((time.perf_counter() - t0) / 5 * 1e6, 1)
    seal(A)
    opn(A)
    torch.cuda.synchronize()
    out["ok"] = int(A["ok"].sum()) == A["n"] and bool(torch.equal(A["back"], A["pt"]))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
