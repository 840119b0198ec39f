"""Device-resident timing of one C5-shaped chunk (mixed log-uniform 512 B-64 KiB records):
HMAC-SHA256 kernel alone, AEAD seal alone, both fused, with and without longest-first order."""
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
import ephemeralnet_amd as E

dev = torch.device("cuda", 0)
rng = np.random.default_rng(5)
res = {}
for chunk_mib in (32, 256):
    lens = []
    while sum(lens) < (chunk_mib << 20):
        lens.append(int(np.exp(rng.uniform(np.log(512), np.log(65536)))))
    n = len(lens)
    offs = torch.tensor(np.concatenate([[0], np.cumsum(lens)]), dtype=torch.int64, device=dev)
    total = int(offs[-1])
    pt = torch.randint(0, 256, (total,), dtype=torch.uint8, device=dev)
    keys = torch.randint(0, 256, (32 * n,), dtype=torch.uint8, device=dev)
    nonces = torch.randint(0, 256, (12 * n,), dtype=torch.uint8, device=dev)
    ct = torch.empty_like(pt)
    tags = torch.empty(16 * n, dtype=torch.uint8, device=dev)
    macs = torch.empty(32 * n, dtype=torch.uint8, device=dev)
    order = torch.tensor(np.argsort(-np.array(lens), kind="stable").astype(np.int32), device=dev)
    for name, od in (("unordered", None), ("longest_first", order)):
        b = E.Batch(pt, offs, keys, nonces, order=od, total_bytes_hint=total, max_len_hint=max(lens))

        def t(fn, reps=5):
            fn()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                fn()
            torch.cuda.synchronize()
            return (time.perf_counter() - t0) / reps * 1e3

        res[f"{chunk_mib}MiB_{name}_hmac_ms"] = t(lambda: E.hmac_sha256(keys, pt, offs, macs))
        res[f"{chunk_mib}MiB_{name}_aead_seal_ms"] = t(lambda: E.aead_seal(b, ct, tags))
        res[f"{chunk_mib}MiB_{name}_aead_hmac_seal_ms"] = t(lambda: E.aead_hmac_seal(b, ct, tags, macs))
    res[f"{chunk_mib}MiB_records"] = n
print(json.dumps({k: round(v, 3) if isinstance(v, float) else v for k, v in res.items()}))
