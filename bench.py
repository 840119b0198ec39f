#!/usr/bin/env python3
"""bench.py -- device-resident ChaCha20-Poly1305 seal+open throughput on MI355X.

Workload (BASELINE.json configs[1]): 65 536 records x 4 KiB per GPU, per-record
(key, nonce) as per-peer sessions, synthetic random data resident in HBM before the timed region.
One step = enet_aead_seal_batch over the whole batch followed by enet_aead_open_batch of the
result (every tag verified).  value = sum of plaintext bytes over all ranks * steps / wall time
of the timed region (max over ranks) = sum L / (t_seal + t_open), in GiB/s.

Multi-GPU: records are independent, so each rank seals/opens its own batch with no collective
on the data path (weak scaling; the only collectives are the timing barrier and the max-reduce).

Launch: python bench.py [--gpus N --steps K --warmup W]; for N > 1 under
python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md chip table)
# VALU: gfx950 issues a full-rate wave64 op (v_add/v_xor/v_lshrrev/v_bitop3 ...) every 2 cycles per
# SIMD once two waves share it, half-rate ops (v_alignbit = the ChaCha rotate, v_mad_u64_u32 =
# the Poly1305 limb product, carries) every 4+ (tools/ubench_mix*.hip).  valu_roofline reports the
# ISA bound of the instruction mix (48.3 G blocks/s for seal/open) and, beside it, the measured
# compute-only rate of the kernel itself (memory waves idle), both in VALU_CEILING_FILE.
VALU_ISSUE_PEAK_TOPS = 78.6  # 256 CU x 4 SIMD x 32 lanes x 2.4 GHz, full-rate ops only
WORKLOADS = {(65536, 4096): "C2", (1048576, 1500): "C3", (32768, 65536): "C4 (per-GPU share)"}
METRIC = "GiB/s ChaCha20-Poly1305 seal+open (device-resident) at 1/2/4/8 MI355X"
HOST_MODES = {0: "zero-copy kernels", 3: "SDMA split by direction, kernels on their own streams",
              4: "SDMA in, kernels write host memory"}
MODE_DESC = {"aead": "AEAD seal+open", "xor": "ChaCha20 xor twice",
             "wire": "wire frames (nonce||BE32||ChaCha20(m||HMAC)) seal+open",
             "store": "chunk store (SHA-256 id + ChaCha20) + fetch (decrypt + SHA-256 check)"}
METRICS = {  # the headline is `aead`; the others are SURVEY 8d/8f side measurements
    "aead": METRIC,
    "xor": "GiB/s ChaCha20 xor pass pair (device-resident)",
    "wire": "GiB/s session wire frames seal+open (device-resident)",
    "store": "GiB/s chunk store+fetch pipeline, SHA-256 + ChaCha20 (device-resident)",
}
PMC_FILE = os.path.join(ROOT, "profiles", "pmc_r06.json")
VALU_CEILING_FILE = os.path.join(ROOT, "profiles", "valu_ceiling_r02.json")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--warmup", type=int, default=50,
                    help="untimed steps; MI355X clocks ramp over the first ~10 ms of sustained load")
    ap.add_argument("--records", type=int, default=None,
                    help="records per GPU (default 65 536; --c5: 524 288, BASELINE config 5)")
    ap.add_argument("--record-bytes", type=int, default=4096)
    ap.add_argument("--lanes", type=int, default=0, help="force lanes per record (0 = scheduler)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-power", action="store_true",
                    help="skip the rocm-smi package power / sclk sample after the timed region")
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="approximate wall budget of the CPU baseline sample")
    ap.add_argument("--e2e", action="store_true",
                    help="host-resident path through the library's host pipeline: pinned host "
                         "buffers, H2D -> kernel -> D2H overlapped over --streams streams in "
                         "--chunk-mib chunks (recorded in DESIGN.md, never `value`)")
    ap.add_argument("--chunk-mib", type=int, default=0, help="host pipeline chunk size (0 = runtime default)")
    ap.add_argument("--streams", type=int, default=0, help="host pipeline slots / streams (0 = runtime default)")
    # internal: one host-resident leg in a child process (host_child_main)
    ap.add_argument("--host-child", choices=["c2", "c5"], default=None, help=argparse.SUPPRESS)
    ap.add_argument("--host-device", type=int, default=0, help=argparse.SUPPRESS)
    for k in ("--c5-all", "--c5-lo", "--c5-hi", "--c5-rank"):
        ap.add_argument(k, type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--c5-steps", type=int, default=1, help=argparse.SUPPRESS)
    ap.add_argument("--no-pin", action="store_true",
                    help="do not pin this rank (and its host children) to its GPU's NUMA node CPUs")
    ap.add_argument("--no-long", action="store_true",
                    help="skip the long-record side leg (1 x 32 MiB, 8 x 1 MiB)")
    ap.add_argument("--long-only", action="store_true",
                    help="print only the long-record side leg (device-resident) and exit")
    ap.add_argument("--no-e2e", action="store_true",
                    help="host-resident keys: only the C5 share (no C2 e2e child) -- the one-GPU N = 8 "
                         "rehearsal, where 8 ranks + 8 children already use the box's 16 GPU process slots")
    ap.add_argument("--no-host", action="store_true",
                    help="default line: skip the host-resident extra keys (C2 e2e, C5 per-GPU share)")
    ap.add_argument("--c5-chunk-mib", type=int, default=0,
                    help="host pipeline chunk size for --c5 (one lane hashes a whole record, so "
                         "mixed batches with HMAC want big chunks)")
    ap.add_argument("--c5-streams", type=int, default=0,
                    help="host pipeline streams for --c5 (a chunk's kernel lasts as long as its "
                         "longest record's serial HMAC, so more chunks in flight)")
    ap.add_argument("--c5", action="store_true",
                    help="SURVEY 8d C5: log-uniform 512 B-64 KiB records, AEAD + fused HMAC-SHA256, "
                         "host-resident (H2D + kernels + D2H), records per GPU = --records")
    ap.add_argument("--c5-device", action="store_true",
                    help="C5 shape device-resident (inputs in HBM, one-pass duplex kernel); "
                         "--c5-order sorted|none picks the record order the kernel walks")
    ap.add_argument("--c5-overlap", action="store_true",
                    help="--c5-device: overlap step k+1's seal with step k's open (two streams)")
    ap.add_argument("--c5-order", default="sorted", choices=["sorted", "none"],
                    help="--c5-device: length-sorted (descending) record order, sort timed inside the step")
    ap.add_argument("--pow-jobs", type=int, default=65536, help="--mode pow: jobs per GPU")
    ap.add_argument("--pow-attempts", type=int, default=4096,
                    help="--mode pow: attempts per job (difficulty 24 = the store clamp, so nearly "
                         "every job scans all of them)")
    ap.add_argument("--pow-schedule", type=int, default=1, choices=[0, 1],
                    help="--mode pow: 1 = store PoW (mt19937_64 candidates, 44-byte prefix), "
                         "0 = handshake PoW (start + attempt, 88-byte prefix)")
    ap.add_argument("--prewarm-s", type=float, default=0.3,
                    help="untimed clock-ramp seal/open pairs before the warmup steps (seconds, 0 = off)")
    ap.add_argument("--sessions", type=int, default=0,
                    help="--mode wire: frames filed round-robin under this many session keys (a key "
                         "table + HMAC midstates computed inside every step, "
                         "enet_wire_*_batch_sessions); 0 = a key per frame")
    ap.add_argument("--store-ids", default="given", choices=["given", "content"],
                    help="store mode: caller-given chunk ids (fused kernel) or content-derived")
    ap.add_argument("--mode", default="aead", choices=["aead", "xor", "wire", "store", "pow"],
                    help="aead = seal+open (headline); xor = ChaCha20-only pass pair (roofline "
                         "probe); wire = session wire frames seal+open (SURVEY 8f row 1, messages "
                         "of --record-bytes); store = chunk store+fetch pipeline (8f row 2)")
    a = ap.parse_args()
    a.records_given = a.records is not None
    if a.records is None:
        a.records = 65536
    return a


def affinity_cpus() -> int:
    """CPUs in this process's affinity mask (on the GPU box: the whole machine, 256)."""
    try:
        return max(1, len(os.sched_getaffinity(0)))
    except AttributeError:
        return max(1, os.cpu_count() or 1)


def cgroup_cpus() -> int | None:
    """CPUs the cgroup quota grants (cpu.max "quota period" -> ceil(quota / period)), None when
    unlimited or unreadable.  The GPU box: "1600000 100000" = 16 CPUs of a 256-CPU machine."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
    except (OSError, ValueError):
        return None
    if quota == "max":
        return None
    q, p = int(quota), int(period)
    return max(1, -(-q // p)) if q > 0 and p > 0 else None


def host_threads() -> int:
    """Threads for the CPU baselines = the CPUs this process can actually use: the affinity mask
    capped by the cgroup CPU quota (all host cores, the count stated in the line).
    Round 3 ran 256 threads under a 16-CPU quota and reported 256 cores."""
    q = cgroup_cpus()
    return min(affinity_cpus(), q) if q else affinity_cpus()


def host_cpu_info() -> dict:
    """nproc, the affinity mask size, the lscpu model name and the cgroup CPU quota (cpu.max),
    recorded beside every CPU number so the baseline's hardware is explicit."""
    info = {"nproc": os.cpu_count(), "affinity": affinity_cpus(), "cgroup_cpus": cgroup_cpus(),
            "effective_cpus": host_threads(), "model": None, "cgroup_cpu_max": None}
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name:"):
                info["model"] = line.split(":", 1)[1].strip()
                break
    except Exception:
        pass
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            info["cgroup_cpu_max"] = f.read().strip()
    except OSError:
        pass
    return info


def cpu_baseline(record_bytes: int, budget_s: float) -> dict:
    """The CPU oracle (oracle/enet_oracle.c: byte-wise ChaCha20 like src/crypto/ChaCha20.cpp,
    RFC 8439 Poly1305) on a bounded sample of the same workload, all host threads of this rank's
    affinity mask (every core this rank may run on), same metric: sum L / (t_seal + t_open)."""
    import ctypes as C

    import numpy as np

    import oracle

    threads = host_threads()
    L = record_bytes
    n = max(512 * 16, 64 * threads)
    rng = np.random.default_rng(1)
    pt = rng.integers(0, 256, n * L, dtype=np.uint8)
    keys = rng.integers(0, 256, n * 32, dtype=np.uint8)
    nonces = rng.integers(0, 256, n * 12, dtype=np.uint8)
    ct = np.empty_like(pt)
    back = np.empty_like(pt)
    tags = np.empty(16 * n, dtype=np.uint8)
    secs = (C.c_double * 2)()
    lib = oracle.lib()
    p = lambda a: a.ctypes.data_as(C.c_void_p)
    total_s = 0.0
    total_b = 0
    reps = 0
    t_start = time.perf_counter()
    while True:
        fails = lib.orc_bench_aead(p(pt), p(ct), p(back), p(keys), p(nonces), p(tags), n, L,
                                   threads, secs)
        assert fails == 0 and np.array_equal(back[:L], pt[:L])
        total_s += secs[0] + secs[1]
        total_b += n * L
        reps += 1
        if time.perf_counter() - t_start > budget_s or reps >= 64:
            break
    # the same kernel on one core (SURVEY.md 8d asks for both numbers)
    n1 = min(n, max(64, (64 << 20) // max(L, 1) // 8))
    fails = lib.orc_bench_aead(p(pt), p(ct), p(back), p(keys), p(nonces), p(tags), n1, L, 1, secs)
    assert fails == 0
    one_core = n1 * L / (secs[0] + secs[1]) / 2**30
    return {
        "value": round(total_b / total_s / 2**30, 4),
        "unit": "GiB/s",
        "cores": threads,
        "one_core_value": round(one_core, 4),
        "host": host_cpu_info(),
        "kind": "port",
        "sample": f"{reps} x {n} records x {L} B AEAD seal+open (oracle/enet_oracle.c, "
                  f"byte-wise like src/crypto/ChaCha20.cpp, -O2), {threads} threads",
    }


def ref_lib():
    """oracle/_ref/libenet_ref.so: the reference's own src/crypto + StoreProof.cpp compiled in the
    build container (oracle/Makefile ref) -- travels with the tree; None when absent."""
    import ctypes as C
    path = os.path.join(ROOT, "oracle", "_ref", "libenet_ref.so")
    if not os.path.exists(path):
        return None
    lib = C.CDLL(path)
    lib.ref_bench_frames.argtypes = [C.c_void_p] * 3 + [C.c_size_t, C.c_size_t, C.c_int, C.c_void_p]
    lib.ref_bench_store_pow.argtypes = [C.c_void_p, C.c_size_t, C.c_uint64, C.c_uint8, C.c_uint64,
                                        C.c_int, C.POINTER(C.c_uint64)]
    lib.ref_bench_store_pow.restype = C.c_double
    return lib


def cpu_reference_frames(record_bytes: int, budget_s: float) -> dict | None:
    """The reference itself (oracle/_ref: src/crypto ChaCha20 + HmacSha256 as compiled from
    /root/reference) running its own record construction -- encode_signed's HMAC + ChaCha20 at
    counter 0 and the inverse with verification (Message.cpp:305-328, SessionManager.cpp:362-374,
    815-822) -- over records of the same length on the host cores.  Reported next to the AEAD
    baseline because the reference has no Poly1305."""
    import ctypes as C

    import numpy as np
    lib = ref_lib()
    if lib is None:
        return None
    threads = host_threads()
    L = record_bytes
    n = max(128 * 16, 16 * threads)
    rng = np.random.default_rng(3)
    pt = rng.integers(0, 256, n * L, dtype=np.uint8)
    keys = rng.integers(0, 256, n * 32, dtype=np.uint8)
    nonces = rng.integers(0, 256, n * 12, dtype=np.uint8)
    secs = (C.c_double * 2)()
    total_s, reps = 0.0, 0
    t_start = time.perf_counter()
    while True:
        fails = lib.ref_bench_frames(pt.ctypes.data, keys.ctypes.data, nonces.ctypes.data, n, L,
                                     threads, secs)
        assert fails == 0
        total_s += secs[0] + secs[1]
        reps += 1
        if time.perf_counter() - t_start > budget_s or reps >= 64:
            break
    return {"value": round(reps * n * L / total_s / 2**30, 4), "unit": "GiB/s", "cores": threads,
            "host": host_cpu_info(), "kind": "reference",
            "sample": f"{reps} x {n} records x {L} B, reference frame seal+open (HMAC-SHA256 + "
                      f"ChaCha20, oracle/_ref compiled from src/crypto), {threads} threads"}


# Where this rank's host work runs (ephemeralnet_amd/topo.py, set by place_rank() before any GPU
# call): its GPU's NUMA node, that node's CPUs within the affinity mask, and its share of the CPU
# budget (cgroup quota / ranks on the node, handed to the library as ENET_HOST_CPUS).  Host
# children inherit both.
PLACEMENT: dict = {}


def place_rank(args) -> None:
    from ephemeralnet_amd import topo
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("WORLD_SIZE", "1")))
    pl = topo.rank_placement(local, local_world)
    if not args.no_pin:
        topo.apply_placement(pl)
    PLACEMENT.update({"numa_node": pl["numa_node"], "cpus": topo.format_cpulist(pl["cpus"]),
                      "ncpus": len(pl["cpus"]), "cpu_budget": pl["cpu_budget"], "pinned": not args.no_pin,
                      "numa_nodes": len(topo.numa_nodes())})


def PLACEMENT_SHORT() -> dict:
    return {k: PLACEMENT.get(k) for k in ("numa_node", "cpus", "cpu_budget", "pinned")}


def gather_placement(world: int, info: dict):
    """N > 1: every rank's placement and host stats (all_gather_object), None for one process."""
    if world <= 1:
        return None
    import torch.distributed as dist
    got = [None] * dist.get_world_size()
    dist.all_gather_object(got, info)
    return [{"rank": i, **g} for i, g in enumerate(got)]


_PINNED = []  # enet_host_alloc blocks of this process (freed at exit by the OS)


def pinned_empty(nbytes: int):
    """A uint8 CPU tensor over pinned host memory from the library's allocator (enet_host_alloc =
    hipHostMalloc), the buffer pools INTEGRATION.md gives socket / relay code."""
    import ctypes as C

    import torch

    import ephemeralnet_amd as E
    p = E.lib().enet_host_alloc(max(nbytes, 1))
    if not p:
        raise SystemExit("enet_host_alloc failed")
    _PINNED.append(p)
    return torch.frombuffer((C.c_uint8 * max(nbytes, 1)).from_address(p), dtype=torch.uint8)[:nbytes]


def pinned_release(mark: int) -> None:
    """Free the enet_host_alloc blocks taken since len(_PINNED) was `mark` (their tensors must be
    dead by now)."""
    import ephemeralnet_amd as E
    E.lib().enet_host_free.argtypes = [__import__("ctypes").c_void_p]
    while len(_PINNED) > mark:
        E.lib().enet_host_free(_PINNED.pop())


def pinned_copy(t):
    out = pinned_empty(t.numel() * t.element_size())
    out.copy_(t.contiguous().view(-1).view(torch_uint8()))
    return out


def torch_uint8():
    import torch
    return torch.uint8


def host_c2(dev_index: int, n: int, L: int, reps: int = 3, chunk_mib: int = 0, streams: int = 0) -> dict:
    """C2 shape starting and ending in pinned host memory (the reference's socket / relay path),
    through the library's host pipeline (enet_pipeline_aead_*, host_batch.cpp runtime): seal then
    open, `reps` each, every tag verified and the plaintext back byte for byte.  Keys, nonces and
    tags live on the host too.  Returns GiB/s of plaintext (sum L / (t_seal + t_open))."""
    import torch

    import ephemeralnet_amd as E

    mark = len(_PINNED)
    g = torch.Generator().manual_seed(7)
    pt_h = pinned_copy(torch.randint(0, 256, (n * L,), dtype=torch.uint8, generator=g))
    keys_h = pinned_copy(torch.randint(0, 256, (n * 32,), dtype=torch.uint8, generator=g))
    nonces_h = pinned_copy(torch.randint(0, 256, (n * 12,), dtype=torch.uint8, generator=g))
    offs_h = pinned_copy(torch.arange(0, (n + 1) * L, L, dtype=torch.int64)).view(torch.int64)
    ct_h = pinned_empty(n * L)
    back_h = pinned_empty(n * L)
    tags_h = pinned_empty(16 * n)
    ok_h = pinned_empty(n)
    seal_b = E.Batch(pt_h, offs_h, keys_h, nonces_h, total_bytes_hint=n * L, max_len_hint=L)
    open_b = E.Batch(ct_h, offs_h, keys_h, nonces_h, total_bytes_hint=n * L, max_len_hint=L)
    pipe = E.Pipeline(dev_index, chunk_mib << 20, streams)
    pipe.aead_seal(seal_b, ct_h, tags_h)  # warm-up (grows the pipeline's buffers)
    pipe.aead_open(open_b, back_h, tags_h, ok_h)
    auto_mode_warmup(dev_index, lambda: (pipe.aead_seal(seal_b, ct_h, tags_h),
                                         pipe.aead_open(open_b, back_h, tags_h, ok_h)))
    t0 = time.perf_counter()
    for _ in range(reps):
        pipe.aead_seal(seal_b, ct_h, tags_h)
    t1 = time.perf_counter()
    for _ in range(reps):
        pipe.aead_open(open_b, back_h, tags_h, ok_h)
    t2 = time.perf_counter()
    st = host_stats(pipe)
    pipe.close()
    good = int(ok_h.sum()) == n and torch.equal(back_h, pt_h)
    del pt_h, keys_h, nonces_h, offs_h, ct_h, back_h, tags_h, ok_h, seal_b, open_b
    pinned_release(mark)
    if not good:
        raise SystemExit("host-resident C2: round trip failed")
    gib = n * L * reps / 2**30
    return {"gibs": gib / (t2 - t0), "seal_gibs": gib / (t1 - t0), "open_gibs": gib / (t2 - t1), "host": st}


def host_stats(pipe) -> dict:
    """Where the pipeline's host side ran (enet_pipeline_stats) and the process's pinned bytes."""
    import ephemeralnet_amd as E
    st = pipe.stats()
    keep = ("device_node", "target_node", "staging_node", "workers", "cpu_budget", "spin", "mode",
            "pinned_bytes")
    out = {k: st[k] for k in keep}
    out["process_pinned_bytes"] = E.host_pinned_bytes()
    return out


def e2e(args) -> dict:
    """--e2e: the C2 shape host-resident (host_c2), one line; the library is loaded before torch
    (the system HIP runtime, see HOST_RUNTIME)."""
    import ephemeralnet_amd as E
    E.lib()
    r = host_c2(0, args.records, args.record_bytes, 3, args.chunk_mib, args.streams)
    return {
        "metric": "GiB/s ChaCha20-Poly1305 seal+open, host-resident (H2D + kernel + D2H)",
        "value": round(r["gibs"], 2),
        "unit": "GiB/s",
        "seal_GiBs": round(r["seal_gibs"], 2),
        "open_GiBs": round(r["open_gibs"], 2),
        "pcie_bytes_per_plaintext_byte": 2.0,
        "host": r["host"],
        "placement": PLACEMENT,
        "numa_policy": os.environ.get("ENET_HOST_NUMA", "auto"),
        "config": {"records": args.records, "record_bytes": args.record_bytes, "chunk_mib": args.chunk_mib,
                   "streams": args.streams, "host_buffers": "pinned", "host_mode": HOST_MODES[r["host"]["mode"]],
                   "hip_runtime": "system ROCm HIP runtime (library loaded before torch)",
                   "path": "enet_pipeline_aead_seal/open (libenet_crypto.so)"},
    }


def under_profiler() -> bool:
    """rocprofv3 preloads its library (and initialises the GPU) before the program starts."""
    pre = os.environ.get("LD_PRELOAD", "")
    return "rocprof" in pre or any(k.startswith(("ROCPROF", "ROCP_")) for k in os.environ)


def start_power_sampler():
    """Fork the rocm-smi sampler BEFORE this process touches the GPU: the child waits on its stdin,
    then runs rocm-smi three times; this process never starts a program after GPU initialisation.
    None when unwanted (N > 1, --no-power, other modes, under a profiler) or unavailable."""
    import subprocess
    cmd = "read go || exit 0; sleep 0.8; for i in 1 2 3; do rocm-smi --showpower --showclocks; sleep 0.3; done"
    try:
        return subprocess.Popen(["bash", "-c", cmd], stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                                stderr=subprocess.DEVNULL, text=True)
    except OSError:
        return None


def sample_power(proc, step, sync, secs: float = 2.5) -> dict | None:
    """Package power and shader clock while the step runs back to back (after the timed region):
    the pre-forked sampler (start_power_sampler) reads rocm-smi a few times, the busiest GPU's
    readings are reported (the kernels are power-capped, DESIGN.md 4 / profiles/r02_power.txt)."""
    import re
    import subprocess
    import statistics
    try:
        proc.stdin.write("go\n")
        proc.stdin.flush()
    except OSError:
        return None
    t0 = time.perf_counter()
    while proc.poll() is None and time.perf_counter() - t0 < secs + 4:
        for _ in range(64):  # ~18 ms of queued work per host sync: no idle gaps in the sample
            step()
        sync()
    try:
        txt = proc.communicate(timeout=5)[0]
    except subprocess.TimeoutExpired:
        proc.kill()
        return None
    pw, clk = {}, {}
    for line in txt.splitlines():
        m = re.search(r"GPU\[(\d+)\].*Package Power \(W\):\s*([0-9.]+)", line)
        if m:
            pw.setdefault(int(m.group(1)), []).append(float(m.group(2)))
        m = re.search(r"GPU\[(\d+)\].*sclk clock level:.*\((\d+)Mhz\)", line)
        if m:
            clk.setdefault(int(m.group(1)), []).append(float(m.group(2)))
    if not pw:
        return None
    g = max(pw, key=lambda k: statistics.median(pw[k]))
    return {"package_w": statistics.median(pw[g]),
            "sclk_mhz": statistics.median(clk[g]) if g in clk else None,
            "samples": len(pw[g]),
            "source": "rocm-smi while seal/open pairs run back to back after the timed region "
                      "(busiest GPU); idle sclk 2.4 GHz, package cap ~1.4 kW"}


def rank_report(world: int, red_dev, local_bytes: int, local_s: float, local_ok: bool):
    """N > 1: every rank's own rate and round-trip verdict, all-gathered, plus what the process
    group itself says (backend, world size), so a SCALE record shows that N ranks each did the
    same work.  None for a single process."""
    if world <= 1:
        return None
    import torch
    import torch.distributed as dist
    mine = torch.tensor([float(local_bytes), local_s, 1.0 if local_ok else 0.0],
                        dtype=torch.float64, device=red_dev)
    got = [torch.zeros_like(mine) for _ in range(dist.get_world_size())]
    dist.all_gather(got, mine)
    return [{"rank": i, "gibs": round(g[0].item() / g[1].item() / 2**30, 2),
             "bytes": int(g[0].item()), "ok": bool(g[2].item())} for i, g in enumerate(got)]


def dist_init(local: int):
    """One process per GPU over nccl (= RCCL on ROCm).  ENET_BENCH_BACKEND=gloo rehearses the
    N > 1 path on a one-GPU box: the ranks share cuda:(LOCAL_RANK mod device_count) and the
    barrier / max-reduce run on the host.  Returns (device, device for the reduce tensor)."""
    import torch
    import torch.distributed as dist
    backend = os.environ.get("ENET_BENCH_BACKEND", "nccl")
    dev = torch.device("cuda", local % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=dev)
        return dev, dev
    dist.init_process_group(backend)
    return dev, torch.device("cpu")


def c5_lengths(n_all: int):
    """SURVEY 8d C5 record lengths: log-uniform on [512, 65 536] B, seed 5."""
    import numpy as np
    rng = np.random.default_rng(5)
    return np.exp(rng.uniform(np.log(512), np.log(65536), n_all)).astype(np.int64)


def auto_mode_warmup(dev_index: int, step) -> None:
    """Auto host mode: the device's first large in-place-output jobs sample modes 3 and 4 (two
    each).  Let them run before a timed region, as a long-running process would have."""
    import ephemeralnet_amd as E
    for _ in range(4):
        if E.host_mode() != -1 or E.host_mode_auto(dev_index)["mode"] != -1:
            return
        step()


def host_c5_rank(dev_index: int, lens, seed: int, chunk_mib: int, streams: int, steps: int = 1):
    """One rank's share of C5 host-resident: AEAD + fused HMAC-SHA256 seal then open of `lens`
    records from and to pinned host memory (enet_pipeline_aead_hmac_*).  Returns (step(),
    check(), bytes): step() runs one seal+open, check() verifies the last round trip."""
    import numpy as np
    import torch

    import ephemeralnet_amd as E

    n = len(lens)
    mark = len(_PINNED)
    offs_h = pinned_copy(torch.from_numpy(np.concatenate([[0], np.cumsum(lens)]).astype(np.int64))).view(torch.int64)
    total = int(offs_h[-1])
    g = torch.Generator().manual_seed(seed)
    pt_h = pinned_copy(torch.randint(0, 256, (total,), dtype=torch.uint8, generator=g))
    keys_h = pinned_copy(torch.randint(0, 256, (n * 32,), dtype=torch.uint8, generator=g))
    nonces_h = pinned_copy(torch.randint(0, 256, (n * 12,), dtype=torch.uint8, generator=g))
    ct_h = pinned_empty(total)
    back_h = pinned_empty(total)
    tags_h = pinned_empty(16 * n)
    macs_h = pinned_empty(32 * n)
    ok_h = pinned_empty(n)
    mx = int(lens.max()) if n else 0
    seal_b = E.Batch(pt_h, offs_h, keys_h, nonces_h, total_bytes_hint=total, max_len_hint=mx)
    open_b = E.Batch(ct_h, offs_h, keys_h, nonces_h, total_bytes_hint=total, max_len_hint=mx)
    pipe = E.Pipeline(dev_index, chunk_mib << 20, streams)

    def step():
        pipe.aead_hmac_seal(seal_b, ct_h, tags_h, macs_h)
        pipe.aead_hmac_open(open_b, back_h, tags_h, macs_h, ok_h)

    def check():
        nonlocal pt_h, back_h, ct_h
        good = int(ok_h.sum()) == n and torch.equal(back_h, pt_h)
        check.host = host_stats(pipe)
        pipe.close()
        pt_h = back_h = ct_h = None
        seal_b.arena = open_b.arena = None
        pinned_release(mark)
        return good

    return step, check, total


def c5_host_timed(world: int, rank: int, dev_index: int, red_dev, n_per_rank: int, chunk_mib: int,
                  streams: int, steps: int = 1) -> dict:
    """C5 host-resident over all ranks: the n_per_rank * world records are split into byte-balanced
    contiguous shares (shard.py, no collective on the data path); every rank seals and opens its
    share, barrier + max-over-ranks time; GiB/s = all ranks' plaintext bytes / that time."""
    import torch
    import torch.distributed as dist

    from ephemeralnet_amd.shard import shard_ranges

    lens_all = c5_lengths(n_per_rank * world)
    lo, hi = shard_ranges(lens_all.tolist(), world)[rank]
    step, check, mine = host_c5_rank(dev_index, lens_all[lo:hi], 11 + rank, chunk_mib, streams)
    step()  # warm-up: grows the pipeline's staging
    auto_mode_warmup(dev_index, step)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    ok = check()
    if world > 1:
        t = torch.tensor([el, 0.0 if ok else 1.0], dtype=torch.float64, device=red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el, bad = float(t[0].item()), float(t[1].item())
        ok = bad == 0.0
    if not ok:
        raise SystemExit(f"rank {rank}: C5 host-resident round trip failed")
    return {"gibs": int(lens_all.sum()) * steps / el / 2**30, "records_total": len(lens_all),
            "bytes_total": int(lens_all.sum()), "seconds": el}


# ---------------------------------------------------------------- host legs in a child process
# The host pipelines are measured in a child process that loads the library BEFORE torch, so the
# library runs on the system ROCm HIP runtime it links against -- the runtime of a C / C++ / Go
# host calling the C ABI, the deployment INTEGRATION.md describes.  In a process that imported
# torch first, the library resolves libamdhip64 to torch's bundled copy instead, whose SDMA copies
# measured 12.3 vs 18.9 GiB/s for the same C2 pipeline on the same box
# (profiles/r04_e2e_probe_hip_runtime.jsonl); that in-process figure is reported beside it.
HOST_RUNTIME = "system ROCm HIP runtime (child process: libenet_crypto loaded before torch)"


def host_child_main(args) -> None:
    """--host-child c2|c5 (internal): one host-resident measurement, JSON on stdout.  c5 prints
    "ready" after its warm-up and starts its timed steps when a line arrives on stdin, so the
    parents can line up every rank's timed region behind a barrier."""
    import ephemeralnet_amd as E
    E.lib()  # before torch: the system HIP runtime
    if args.host_child == "c2":
        r = host_c2(args.host_device, args.records, args.record_bytes, 3, args.chunk_mib, args.streams)
        r["host_mode"] = r["host"]["mode"]
        r["mode_auto"] = E.host_mode_auto(args.host_device)  # what picked it (system runtime)
        print(json.dumps(r), flush=True)
        return
    lens = c5_lengths(args.c5_all)[args.c5_lo:args.c5_hi]
    step, check, mine = host_c5_rank(args.host_device, lens, 11 + args.c5_rank, args.c5_chunk_mib,
                                     args.c5_streams)
    step()  # warm-up: grows the pipeline's staging
    auto_mode_warmup(args.host_device, step)
    print("ready", flush=True)
    sys.stdin.readline()
    t0 = time.perf_counter()
    for _ in range(args.c5_steps):
        step()
    el = time.perf_counter() - t0
    ok = bool(check())
    host = getattr(check, "host", None) or {}
    print(json.dumps({"seconds": el, "ok": ok, "bytes": int(mine), "host_mode": host.get("mode", 3),
                      "host": host or None}), flush=True)


def host_child(kind: str, dev_index: int, extra: list):
    """Start `bench.py --host-child kind` on device dev_index (a child process: this process may
    have initialised the GPU, so it never replaces itself by another program)."""
    cmd = [sys.executable, os.path.abspath(__file__), "--host-child", kind, "--host-device", str(dev_index)] + extra
    return subprocess.Popen(cmd, stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)


def frame_queue_leg(dev_index: int) -> dict | None:
    """SURVEY 8f row 1, side keys (never `value`): the cross-session frame queues through
    tools/queue_bench (built beside the library; skipped when it is not there) -- 16 session
    threads, 256 MTU frames in flight each, zero-copy collection -- on the device queue and on the
    host engine, frames/s each way and process CPU per frame; and the device queue with 1 024 in
    flight each (`device_1024`: past AUTO's crossover, large passes staged in device memory).
    Each run has an untimed 0.3 s leg each way first (steady state).  Runs as a child process on
    this rank's CPUs (the placement above), ~8 s."""
    exe = os.path.join(ROOT, "tools", "queue_bench")
    if not os.access(exe, os.X_OK):
        return None
    if dev_index != 0:  # queue_bench drives device 0 of this process's visible set
        return None
    res = {}
    for key, pol, window in (("device", "device", "256"), ("host", "host", "256"), ("device_1024", "device", "1024")):
        try:
            r = subprocess.run([exe, pol, "view", "16", window, "0.8"], capture_output=True, text=True,
                               timeout=120, env=dict(os.environ, QUEUE_BENCH_WARMUP="0.3"))
            d = json.loads(r.stdout.strip().splitlines()[-1])
        except (subprocess.TimeoutExpired, ValueError, IndexError) as e:
            return {"error": f"queue_bench {key}: {e}"}
        res[key] = {"seal_frames_per_s": d["seal_frames_per_s"], "open_frames_per_s": d["open_frames_per_s"],
                    "cpu_us_per_frame": round((d["seal_cpu_us_per_frame"] + d["open_cpu_us_per_frame"]) / 2, 3),
                    "frames_per_pass": round((d["tx_frames_per_pass"] + d["rx_frames_per_pass"]) / 2, 1),
                    "ok": d["ok"]}
    res["cpu_ratio_device_to_host"] = round(res["device"]["cpu_us_per_frame"] / res["host"]["cpu_us_per_frame"], 3)
    res["is"] = ("FrameQueue / FrameReceiveQueue: 16 threads x 256 frames of 1 500 B in flight, submit + "
                 "FrameTicket::view; host = the same calls served on the threads' host engine; device_1024 = "
                 "the device queue with 1 024 in flight per thread")
    return res


def host_c2_child(dev_index: int, n: int, L: int, chunk_mib: int, streams: int) -> dict:
    proc = host_child("c2", dev_index, ["--records", str(n), "--record-bytes", str(L),
                                        "--chunk-mib", str(chunk_mib), "--streams", str(streams)])
    out, _ = proc.communicate(timeout=600)
    if proc.returncode != 0:
        raise SystemExit(f"host-resident C2 child failed (exit {proc.returncode})")
    return json.loads(out.strip().splitlines()[-1])


def c5_host_child_timed(world: int, rank: int, dev_index: int, red_dev, n_per_rank: int, chunk_mib: int,
                        streams: int, steps: int = 1) -> dict:
    """c5_host_timed with each rank's share run by a child process on the system HIP runtime:
    every child warms up, the parents barrier, then all children run their timed steps; the time
    is the max over ranks."""
    import torch
    import torch.distributed as dist

    from ephemeralnet_amd.shard import shard_ranges

    n_all = n_per_rank * world
    lens_all = c5_lengths(n_all)
    lo, hi = shard_ranges(lens_all.tolist(), world)[rank]
    proc = host_child("c5", dev_index, ["--c5-all", str(n_all), "--c5-lo", str(lo), "--c5-hi", str(hi),
                                        "--c5-rank", str(rank), "--c5-steps", str(steps),
                                        "--c5-chunk-mib", str(chunk_mib), "--c5-streams", str(streams)])
    ready = proc.stdout.readline().strip() == "ready"
    if world > 1:
        flag = torch.tensor([0.0 if ready else 1.0], dtype=torch.float64, device=red_dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MAX)
        ready = ready and flag.item() == 0.0
        dist.barrier()
    if not ready:
        proc.kill()
        raise SystemExit(f"rank {rank}: C5 host-resident child did not start")
    out, _ = proc.communicate("go\n", timeout=600)
    res = json.loads(out.strip().splitlines()[-1]) if proc.returncode == 0 else {"seconds": 0.0, "ok": False}
    el, ok = float(res["seconds"]), bool(res["ok"])
    if world > 1:
        t = torch.tensor([el, 0.0 if ok else 1.0], dtype=torch.float64, device=red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el, ok = float(t[0].item()), t[1].item() == 0.0
    if not ok:
        raise SystemExit(f"rank {rank}: C5 host-resident round trip failed")
    return {"gibs": int(lens_all.sum()) * steps / el / 2**30, "records_total": len(lens_all),
            "bytes_total": int(lens_all.sum()), "seconds": el, "host_mode": res.get("host_mode", 3),
            "host": res.get("host")}


def c5(args) -> dict:
    """mixed log-uniform 512 B-64 KiB records with the fused HMAC-SHA256 tag,
    starting and ending in pinned host memory, through the library's host pipeline
    (enet_pipeline_aead_hmac_*).  Multi-GPU: each rank takes a byte-balanced contiguous share
    (shard.py), no collective."""
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = red_dev = torch.device("cuda", local)
    if world > 1:
        dev, red_dev = dist_init(local)
    # BASELINE config 5: n = 524 288 records (~7 GB) unless --records says otherwise
    n_per = args.records if args.records_given else 524288
    r = c5_host_child_timed(world, rank, dev.index, red_dev, n_per, args.c5_chunk_mib, args.c5_streams)
    placements = gather_placement(world, {**PLACEMENT_SHORT(), "host": r.get("host")})
    res = None
    if rank == 0:
        res = {
            "metric": "GiB/s AEAD + fused HMAC-SHA256 seal+open, mixed 512 B-64 KiB, "
                      "host-resident (H2D + kernels + D2H)",
            "value": round(r["gibs"], 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "config": {"workload": "C5", "records_total": r["records_total"], "bytes_total": r["bytes_total"],
                       "chunk_mib": args.c5_chunk_mib, "streams": args.c5_streams,
                       "host_buffers": "pinned", "host_mode": HOST_MODES[r["host_mode"]],
                       "hip_runtime": HOST_RUNTIME,
                       "path": "enet_pipeline_aead_hmac_seal/open (libenet_crypto.so)"},
            "host": r.get("host"),
            "placement": PLACEMENT,
            "numa_policy": os.environ.get("ENET_HOST_NUMA", "auto"),
        }
        if placements is not None:
            res["dist"] = {"backend": dist.get_backend(), "world_size": world, "per_rank": placements}
    if world > 1:
        dist.destroy_process_group()
    return res


def c5_device(args) -> dict:
    """C5 shape with the batch already in HBM: log-uniform 512 B-64 KiB records, AEAD seal +
    HMAC-SHA256 then open + verify of both, each direction ONE duplex launch (duplex.hip).  The
    length sort that balances workgroups (--c5-order sorted) runs on the device inside the timed
    step.  Single GPU; --records records."""
    import numpy as np
    import torch

    import ephemeralnet_amd as E
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(5)
    n = args.records
    lens = np.exp(rng.uniform(np.log(512), np.log(65536), n)).astype(np.int64)
    offs = torch.from_numpy(np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)).to(dev)
    total = int(lens.sum())
    g = torch.Generator(device=dev).manual_seed(11)
    pt = torch.randint(0, 256, (total,), dtype=torch.uint8, device=dev, generator=g)
    keys = torch.randint(0, 256, (n * 32,), dtype=torch.uint8, device=dev, generator=g)
    nonces = torch.randint(0, 256, (n * 12,), dtype=torch.uint8, device=dev, generator=g)
    dl = offs[1:] - offs[:-1]
    mx = int(lens.max())  # host-known hints, as a caller that built the batch has them
    # --c5-overlap: consecutive steps overlap -- step k+1's seal runs beside step k's open (two
    # streams; an open waits only for its own seal), so the serial HMAC chain of one step's
    # longest records (~2.8 ms for 64 KiB, one lane) hides under the other direction's work.
    # Each step still seals and opens its whole batch; buffers alternate by step parity.
    nb = 2 if args.c5_overlap else 1
    ct = [torch.empty_like(pt) for _ in range(nb)]
    back = [torch.empty_like(pt) for _ in range(nb)]
    tags = [torch.empty(16 * n, dtype=torch.uint8, device=dev) for _ in range(nb)]
    macs = [torch.empty(32 * n, dtype=torch.uint8, device=dev) for _ in range(nb)]
    ok = [torch.empty(n, dtype=torch.uint8, device=dev) for _ in range(nb)]
    s_seal = torch.cuda.Stream(dev) if args.c5_overlap else torch.cuda.current_stream(dev)
    s_open = torch.cuda.Stream(dev) if args.c5_overlap else s_seal
    main = torch.cuda.current_stream(dev)
    s_seal.wait_stream(main)
    s_open.wait_stream(main)
    order_holder = {}

    def step(k):
        b = k % nb
        with torch.cuda.stream(s_seal):
            order = (torch.argsort(dl, descending=True).to(torch.int32)
                     if args.c5_order == "sorted" else None)
            E.aead_hmac_seal(E.Batch(pt, offs, keys, nonces, order=order, total_bytes_hint=total,
                                     max_len_hint=mx), ct[b], tags[b], macs[b])
            sealed = torch.cuda.Event()
            sealed.record(s_seal)
        if order is not None:
            order.record_stream(s_open)
        order_holder[b] = order  # keep the order tensor alive until the open has run
        with torch.cuda.stream(s_open):
            s_open.wait_event(sealed)
            E.aead_hmac_open(E.Batch(ct[b], offs, keys, nonces, order=order, total_bytes_hint=total,
                                     max_len_hint=mx), back[b], tags[b], macs[b], ok[b])

    # parity buffers: seal k+2 rewrites ct[b] / tags[b] / macs[b], which open k reads -- each
    # seal waits for the open two steps back
    opened = [None] * nb

    def step_safe(k):
        b = k % nb
        if opened[b] is not None:
            s_seal.wait_event(opened[b])
        step(k)
        ev = torch.cuda.Event()
        ev.record(s_open)
        opened[b] = ev

    for k in range(max(1, args.warmup)):
        step_safe(k)
    torch.cuda.synchronize()
    for b in range(nb):
        assert int(ok[b].sum()) == n and torch.equal(back[b], pt)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    main.wait_stream(s_seal)
    main.wait_stream(s_open)
    e0.record(main)
    s_seal.wait_stream(main)
    s_open.wait_stream(main)
    for k in range(args.steps):
        step_safe(k)
    main.wait_stream(s_seal)
    main.wait_stream(s_open)
    e1.record(main)
    torch.cuda.synchronize()
    for b in range(nb):
        assert int(ok[b].sum()) == n and torch.equal(back[b], pt)
    ms = e0.elapsed_time(e1) / args.steps
    return {
        "metric": "GiB/s AEAD + fused HMAC-SHA256 seal+open, mixed 512 B-64 KiB, device-resident",
        "value": round(total / (ms / 1e3) / 2**30, 2),
        "unit": "GiB/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(ms, 4), "higher_is_better": True, "data": "synthetic",
        "config": {"workload": "C5 device-resident", "records": n, "bytes_total": total,
                   "order": args.c5_order, "overlap_steps": bool(args.c5_overlap),
                   "path": "enet_aead_hmac_seal/open_batch -> duplex_kernel"},
    }


def pow_bench(args) -> dict:
    """batched proof-of-work search on the device.  --pow-jobs jobs per GPU,
    each scanning --pow-attempts candidates at difficulty 24 (StoreProof.cpp's clamp: nearly
    never found, so every job does the full scan), prefixes resident in HBM.  value = candidate
    SHA-256 evaluations per second over all ranks.  CPU baseline: the oracle's search loop (the
    reference's algorithm, StoreProof.cpp:123-146 / Node.cpp:269-292) on the host cores."""
    import numpy as np
    import torch
    import torch.distributed as dist

    import ephemeralnet_amd as E

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = red_dev = torch.device("cuda", local)
    if world > 1:
        dev, red_dev = dist_init(local)
    n, A, sched = args.pow_jobs, args.pow_attempts, args.pow_schedule
    plen = 44 if sched == 1 else 88  # store prefix (empty hint) / handshake prefix
    g = torch.Generator(device=dev).manual_seed(77 + rank)
    pre = torch.randint(0, 256, (n * plen,), dtype=torch.uint8, device=dev, generator=g)
    offs = torch.arange(0, (n + 1) * plen, plen, dtype=torch.int64, device=dev)
    diff = torch.full((n,), 24, dtype=torch.uint8, device=dev)
    nonces = torch.empty(n, dtype=torch.int64, device=dev)
    atts = torch.empty(n, dtype=torch.int64, device=dev)
    found = torch.empty(n, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)

    def step():
        E.pow_search(pre, offs, diff, sched, A, nonces, found, atts, stream=stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(args.steps):
        step()
    e1.record(stream)
    e1.synchronize()
    launch_ms = e0.elapsed_time(e1) / args.steps
    # hashes actually evaluated: attempts up to the found one (+1 seed digest per job)
    at = atts.cpu().numpy()
    hashed = int(np.minimum(at + 1, A).sum()) + n
    out = None
    if rank == 0:
        value = hashed * args.steps * world / el
        out = {
            "metric": "G SHA-256 PoW candidates/s (device-resident batch search)",
            "value": round(value / 1e9, 3),
            "unit": "G candidates/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "dtype": "u32",
            "data": "synthetic random prefixes (torch.randint on device)",
            "config": {"workload": f"{'store' if sched else 'handshake'} PoW: {n} jobs x {A} attempts, "
                                   f"{plen}-byte prefixes, difficulty 24",
                       "jobs_per_gpu": n, "attempts": A, "schedule": sched,
                       "found": int(found.sum().item())},
            "launch_ms": round(launch_ms, 4),
            "compressions_per_candidate": 1,
            "sha_rounds_per_candidate": 64 - plen % 64 // 4,
        }
        if not args.no_cpu_baseline and world == 1:
            import ctypes as C

            threads = host_threads()
            m = 64 * threads
            cpu_att = max(256, int(args.cpu_seconds * 2e6 / m))  # ~2 M hashes/s per thread budget
            lib = ref_lib() if sched == 1 else None
            if lib is not None:  # the reference's own compute_store_pow (StoreProof.cpp:123-146)
                found = C.c_uint64()
                secs = lib.ref_bench_store_pow(os.urandom(32 * m), m, 4096, 24, cpu_att, threads,
                                               C.byref(found))
                hashes = m * (cpu_att + 1)  # not-found jobs (found ~1e-4) scan every attempt
                kind, what = "reference", ("security::compute_store_pow from oracle/_ref (compiled "
                                           "src/security/StoreProof.cpp + src/crypto/Sha256.cpp)")
            else:
                import oracle
                pre_h = np.frombuffer(os.urandom(m * plen), dtype=np.uint8).copy()
                off_h = np.arange(0, (m + 1) * plen, plen, dtype=np.uint64)
                hh = C.c_uint64()
                secs = oracle.lib().orc_bench_pow(pre_h.ctypes.data_as(C.c_void_p),
                                                  off_h.ctypes.data_as(C.c_void_p), m, 24, cpu_att,
                                                  threads, C.byref(hh))
                hashes = hh.value
                kind, what = "port", ("oracle/enet_oracle.c orc_pow_search, byte-wise SHA-256 like "
                                      "src/crypto/Sha256.cpp, -O2")
            out["cpu_baseline"] = {
                "value": round(hashes / secs / 1e9, 5), "unit": "G candidates/s", "cores": threads,
                "host": host_cpu_info(), "kind": kind,
                "sample": f"{m} {'store' if sched else 'handshake'}-PoW jobs x {cpu_att} attempts at "
                          f"difficulty 24 ({what})"}
    if world > 1:
        dist.destroy_process_group()
    return out


def chunk_leg(E, dev, stream, pt, offs, keys, nonces, lens, reps: int = 3) -> dict:
    """Chunk store + fetch (caller-given ids) of the long records through the C ABI, device-resident
    -- the hash chains on host threads, the cipher on the tiles (capi.cpp chunk_*_host_hash) --
    against the host engine doing the same on the calling thread's core (enet_host_sha256 +
    enet_host_chacha20_xor per chunk, store then fetch: Node.cpp:1414-1417, 1644-1655).  ms per
    store+fetch pair, best of `reps`."""
    import ctypes as C
    import time
    import numpy as np
    import torch
    n, tot = len(lens), sum(lens)
    g = torch.Generator(device=dev).manual_seed(91)
    ids = torch.randint(0, 256, (32 * n,), dtype=torch.uint8, device=dev, generator=g)
    ct, back = torch.empty_like(pt), torch.empty_like(pt)
    hashes = torch.empty(32 * n, dtype=torch.uint8, device=dev)
    ok = torch.zeros(n, dtype=torch.uint8, device=dev)
    sb = E.Batch(pt, offs, keys, nonces, total_bytes_hint=tot, max_len_hint=max(lens))
    ob = E.Batch(ct, offs, keys, nonces, total_bytes_hint=tot, max_len_hint=max(lens))
    best = None
    good = True
    for _ in range(reps + 1):  # the first pair warms the pinned buffers and worker streams
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        E.chunk_store(sb, ct, hashes, chunk_ids=ids, stream=stream)
        E.chunk_fetch(ob, back, ids, hashes, ok, stream=stream)
        torch.cuda.synchronize(dev)
        ms = (time.perf_counter() - t0) * 1e3
        best = ms if best is None or ms < best else best
        good = good and int(ok.sum()) == n and torch.equal(back, pt)
    L = E.lib()
    L.enet_host_sha256.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p]
    L.enet_host_chacha20_xor.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_uint64]
    hp = pt.cpu().numpy()
    hk, hn, hid = keys.cpu().numpy(), nonces.cpu().numpy(), ids.cpu().numpy()
    ho = np.empty_like(hp)
    hb = np.empty_like(hp)
    dg = np.empty(32, np.uint8)
    o = offs.cpu().tolist()
    host_best = None
    for _ in range(reps):
        t0 = time.perf_counter()
        for i in range(n):
            a, L_ = o[i], o[i + 1] - o[i]
            ctr = int.from_bytes(hid[32 * i:32 * i + 4].tobytes(), "little")
            L.enet_host_sha256(hp[a:].ctypes.data, L_, dg.ctypes.data)
            L.enet_host_chacha20_xor(hk[32 * i:].ctypes.data, hn[12 * i:].ctypes.data, ctr, hp[a:].ctypes.data,
                                     ho[a:].ctypes.data, L_)
            L.enet_host_chacha20_xor(hk[32 * i:].ctypes.data, hn[12 * i:].ctypes.data, ctr, ho[a:].ctypes.data,
                                     hb[a:].ctypes.data, L_)
            L.enet_host_sha256(hb[a:].ctypes.data, L_, dg.ctypes.data)
        ms = (time.perf_counter() - t0) * 1e3
        host_best = ms if host_best is None or ms < host_best else host_best
    return {"chunk_store_fetch_ms": round(best, 3), "chunk_store_fetch_ok": bool(good),
            "chunk_host_engine_ms": round(host_best, 3), "chunk_host_threads": E.host_cpu_budget(),
            "chunk_vs_host_engine": round(host_best / best, 2)}


def long_records_leg(dev, reps: int = 20) -> dict:
    """Side leg (never `value`): the reference's real chunk sizes, device-resident -- a stored file
    is ONE chunk of up to 32 MiB (Config.hpp:62, Node.cpp:1414-1417) and session payloads go up
    to 1 MiB (SessionManager.cpp:87).  AEAD seal+open and ChaCha20 (XOR, both directions) GiB/s =
    plaintext bytes per seal+open pair / its HIP-event time, on the sequence-parallel tiles
    (segments.hip) and, for comparison, on the record engine alone (16 lanes per record)."""
    import numpy as np
    import torch
    import ephemeralnet_amd as E
    stream = torch.cuda.current_stream(dev)
    res = {}
    for name, lens in (("1x32MiB", [32 << 20]), ("8x1MiB", [1 << 20] * 8)):
        n, tot = len(lens), sum(lens)
        g = torch.Generator(device=dev).manual_seed(77)
        pt = torch.randint(0, 256, (tot,), dtype=torch.uint8, device=dev, generator=g)
        keys = torch.randint(0, 256, (32 * n,), dtype=torch.uint8, device=dev, generator=g)
        nonces = torch.randint(0, 256, (12 * n,), dtype=torch.uint8, device=dev, generator=g)
        offs = torch.tensor([0] + list(np.cumsum(lens)), dtype=torch.int64, device=dev)
        ct, back = torch.empty_like(pt), torch.empty_like(pt)
        tags = torch.empty(16 * n, dtype=torch.uint8, device=dev)
        ok = torch.zeros(n, dtype=torch.uint8, device=dev)
        sb = E.Batch(pt, offs, keys, nonces, total_bytes_hint=tot, max_len_hint=max(lens))
        ob = E.Batch(ct, offs, keys, nonces, total_bytes_hint=tot, max_len_hint=max(lens))
        row = {}
        for path, seg in (("tiles", -1), ("record_engine", E.SEG_NEVER)):
            E.set_seg_min(seg)
            for mode in ("aead", "xor"):
                def pair():
                    if mode == "aead":
                        E.aead_seal(sb, ct, tags, stream=stream)
                        E.aead_open(ob, back, tags, ok, stream=stream)
                    else:
                        E.chacha20_xor(sb, ct, stream=stream)
                        E.chacha20_xor(ob, back, stream=stream)
                r_ = reps if path == "tiles" else max(2, reps // 10)
                for _ in range(3):
                    pair()
                torch.cuda.synchronize(dev)
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
                ev[0].record(stream)
                for _ in range(r_):
                    pair()
                ev[1].record(stream)
                ev[1].synchronize()
                ms = ev[0].elapsed_time(ev[1]) / r_
                good = torch.equal(back, pt) and not torch.equal(ct, pt) and (
                    mode == "xor" or int(ok.sum()) == n)
                row[f"{mode}_{path}_gibs"] = round(tot / (ms * 1e-3) / 2**30, 1)
                row[f"{mode}_{path}_ms"] = round(ms, 4)
                row[f"{mode}_{path}_ok"] = bool(good)
        E.set_seg_min(-1)
        row.update(chunk_leg(E, dev, stream, pt, offs, keys, nonces, lens))
        res[name] = row
    res["is"] = ("device-resident, per-record (key, nonce); GiB/s = plaintext bytes / (seal + open) "
                 "time; tiles = 64 KiB tiles over every CU (default), record_engine = at most 16 lanes "
                 "per record (enet_set_seg_min(INT64_MAX)); chunk_store_fetch_ms = one chunk store + fetch pair "
                 "through the C ABI (hash chains on host threads, cipher on the tiles, wall clock), "
                 "chunk_host_engine_ms = the host engine doing both on one core")
    return res


def main():
    args = parse()
    if args.host_child:
        host_child_main(args)
        return
    place_rank(args)  # before any GPU call: this rank and its host children on its GPU's node
    if args.mode == "pow":
        r = pow_bench(args)
        if r:
            print(json.dumps(r), flush=True)
        return
    if args.c5_device:
        print(json.dumps(c5_device(args)))
        return
    if args.c5:
        r = c5(args)
        if r:
            print(json.dumps(r), flush=True)
        return
    if args.e2e:
        print(json.dumps(e2e(args)), flush=True)
        return
    if args.long_only:
        import torch
        import ephemeralnet_amd as E
        E.lib()
        print(json.dumps({"long_records": long_records_leg(torch.device("cuda", 0))}), flush=True)
        return
    sampler = None
    if (int(os.environ.get("WORLD_SIZE", "1")) == 1 and not args.no_power
            and args.mode in ("aead", "xor") and not under_profiler()):
        sampler = start_power_sampler()  # before any GPU initialisation in this process
    import torch
    import torch.distributed as dist

    import ephemeralnet_amd as E

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = red_dev = torch.device("cuda", local)
    if world > 1:
        dev, red_dev = dist_init(local)
    E.lib()
    if args.lanes:
        E.set_lanes_per_record(args.lanes)

    n, L = args.records, args.record_bytes
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    pt = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device=dev, generator=g)
    keys = torch.randint(0, 256, (n * 32,), dtype=torch.uint8, device=dev, generator=g)
    nonces = torch.randint(0, 256, (n * 12,), dtype=torch.uint8, device=dev, generator=g)
    offs = torch.arange(0, (n + 1) * L, L, dtype=torch.int64, device=dev)
    ct = torch.empty_like(pt)
    back = torch.empty_like(pt)
    tags = torch.empty(16 * n, dtype=torch.uint8, device=dev)
    ok = torch.zeros(n, dtype=torch.uint8, device=dev)
    seal_b = E.Batch(pt, offs, keys, nonces, total_bytes_hint=n * L, max_len_hint=L)
    open_b = E.Batch(ct, offs, keys, nonces, total_bytes_hint=n * L, max_len_hint=L)
    stream = torch.cuda.current_stream(dev)
    if args.mode == "wire":
        F = L + 48  # nonce(12) || BE32 || m || HMAC(32)
        foffs = torch.arange(0, (n + 1) * F, F, dtype=torch.int64, device=dev)
        frames = torch.empty(n * F, dtype=torch.uint8, device=dev)
        macs = torch.empty(32 * n, dtype=torch.uint8, device=dev)
        wire_b = E.Batch(frames, foffs, keys, None, total_bytes_hint=n * F, max_len_hint=F)
        if args.sessions:
            K = args.sessions
            if not 0 < K <= n:
                raise SystemExit("--sessions must be in [1, records]")
            sess_tbl = keys[:32 * K]  # session key table; frame i belongs to session i mod K
            sess_idx = (torch.arange(n, dtype=torch.int32, device=dev) % K).contiguous()
            sess_mid = torch.empty(16 * K, dtype=torch.int32, device=dev)
            seal_b = E.Batch(pt, offs, sess_tbl, nonces, total_bytes_hint=n * L, max_len_hint=L)
            wire_b = E.Batch(frames, foffs, sess_tbl, None, total_bytes_hint=n * F, max_len_hint=F)
    if args.mode == "store":
        hashes = torch.empty(32 * n, dtype=torch.uint8, device=dev)
        # Node::store_chunk(chunk_id, data) takes the id from its caller (ControlServer.cpp:1101
        # derives it beforehand): "given" ids take the fused one-pass kernel; "content" ids
        # (counter from the fresh digest) need the digest first, i.e. two passes
        ids = (torch.randint(0, 256, (32 * n,), dtype=torch.uint8, device=dev)
               if args.store_ids == "given" else None)

    def seal():
        if args.mode == "aead":
            E.aead_seal(seal_b, ct, tags, stream=stream)
        elif args.mode == "wire" and args.sessions:
            E.hmac_midstates(sess_tbl, args.sessions, sess_mid, stream=stream)
            E.wire_seal_sessions(seal_b, frames, foffs, sess_idx, args.sessions, sess_mid, stream=stream)
        elif args.mode == "wire":
            E.wire_seal(seal_b, frames, foffs, stream=stream)
        elif args.mode == "store":
            E.chunk_store(seal_b, ct, hashes, chunk_ids=ids, stream=stream)
        else:
            E.chacha20_xor(seal_b, ct, stream=stream)

    def open_():
        if args.mode == "aead":
            E.aead_open(open_b, back, tags, ok, stream=stream)
        elif args.mode == "wire" and args.sessions:
            E.wire_open_sessions(wire_b, back, offs, sess_idx, args.sessions, sess_mid, macs, ok, stream=stream)
        elif args.mode == "wire":
            E.wire_open(wire_b, back, offs, macs, ok, stream=stream)
        elif args.mode == "store":
            E.chunk_fetch(open_b, back, hashes if ids is None else ids, hashes, ok, stream=stream)
        else:
            E.chacha20_xor(open_b, back, stream=stream)

    # clock ramp: untimed seal/open pairs for >= --prewarm-s of wall time (bounded), so a short
    # --warmup still leaves the GPU at its steady-state clock when the timed region starts
    prewarm_steps = 0
    tp = time.perf_counter()
    while args.prewarm_s > 0 and prewarm_steps < 20000:
        for _ in range(16):
            seal()
            open_()
        prewarm_steps += 16
        torch.cuda.synchronize(dev)
        if time.perf_counter() - tp >= args.prewarm_s:
            break
    for _ in range(args.warmup):
        seal()
        open_()
    torch.cuda.synchronize(dev)

    # timed region: exactly K steps, no per-kernel markers in the stream
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        seal()
        open_()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    elapsed_local = elapsed
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # per-kernel durations: HIP events on the launch stream bracketing back-to-back launches of
    # one kernel (separate from the timed region so the markers do not add kernel gaps there)
    # Timed in the same seal/open alternation as the timed region: each kernel reads what the
    # other just wrote.  (Back-to-back launches of one kernel re-read an input that the 256 MiB
    # Infinity Cache partly still holds, and read 4-6 % fast at C2.)
    def kernel_ms_alt(reps):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * reps + 1)]
        ev[0].record(stream)
        for i in range(reps):
            seal()
            ev[2 * i + 1].record(stream)
            open_()
            ev[2 * i + 2].record(stream)
        ev[-1].synchronize()
        s_ms = sum(ev[2 * i].elapsed_time(ev[2 * i + 1]) for i in range(reps)) / reps
        o_ms = sum(ev[2 * i + 1].elapsed_time(ev[2 * i + 2]) for i in range(reps)) / reps
        return s_ms, o_ms

    reps = max(4, args.steps)
    seal_ms, open_ms = kernel_ms_alt(reps)
    okh = int(ok.sum().item()) if args.mode != "xor" else n
    # the round trip must give the plaintext back, byte for byte (a keystream bug shared by seal
    # and open would still verify every tag), and the ciphertext must differ from it
    fail = None
    if okh != n:
        fail = f"rank {rank}: {n - okh} records failed to open"
    elif not torch.equal(back, pt):
        fail = f"rank {rank}: open(seal(x)) != x"
    elif args.mode in ("aead", "xor", "store") and torch.equal(ct, pt):
        fail = f"rank {rank}: ciphertext equals plaintext"
    ranks = rank_report(world, red_dev, n * L * args.steps, elapsed_local, fail is None)
    if fail is not None:
        raise SystemExit(fail)
    if ranks is not None and not all(r["ok"] for r in ranks):
        raise SystemExit(f"rank {rank}: round trip failed on rank(s) "
                         f"{[r['rank'] for r in ranks if not r['ok']]}")
    power = None
    if sampler is not None:
        power = sample_power(sampler, lambda: (seal(), open_()), lambda: torch.cuda.synchronize(dev))

    # Host-resident extra keys (never `value`): the reference's path starts and ends in host
    # memory (SessionManager.cpp:1049-1099), so the line also carries the C2 shape through the
    # host pipeline and BASELINE config 5 (mixed 512 B-64 KiB, AEAD + fused HMAC, H2D/D2H
    # included) at its per-GPU share, 524 288 / 8 = 65 536 records per rank, timed over all ranks
    host = None
    if args.mode == "aead" and not args.no_host and (n, L) == (65536, 4096):
        import ephemeralnet_amd as E2
        if args.no_e2e:
            hc2 = {"gibs": 0.0, "seal_gibs": 0.0, "open_gibs": 0.0}
        else:
            hc2 = host_c2_child(dev.index, n, L, args.chunk_mib, args.streams)
        hc5 = c5_host_child_timed(world, rank, dev.index, red_dev, 65536, args.c5_chunk_mib, args.c5_streams)
        hc2t = (host_c2(dev.index, n, L, 3, args.chunk_mib, args.streams) if not args.no_e2e  # torch's runtime
                else {"gibs": 0.0, "host": {"mode": 3}})
        host = {"e2e_gibs": round(hc2["gibs"], 2), "e2e_seal_gibs": round(hc2["seal_gibs"], 2),
                "e2e_open_gibs": round(hc2["open_gibs"], 2),
                "e2e_is": "C2 (65 536 x 4 KiB) seal+open from and to pinned host memory, this rank",
                "hip_runtime": HOST_RUNTIME,
                "e2e_gibs_torch_hip_runtime": round(hc2t["gibs"], 2),
                "host_mode_torch_hip_runtime": HOST_MODES[hc2t["host"]["mode"]],
                "mode_auto": hc2.get("mode_auto"),
                "mode_auto_torch_hip_runtime": E2.host_mode_auto(dev.index),
                "c5_host_gibs": round(hc5["gibs"], 2),
                "c5_host_is": f"BASELINE config 5 per-GPU share: {hc5['records_total']} log-uniform "
                              f"512 B-64 KiB records over {world} rank(s), AEAD + fused HMAC-SHA256 "
                              "seal+open, pinned host memory in and out, all ranks' bytes / max-over-ranks time",
                "host_mode": HOST_MODES[hc2.get("host_mode", 3)],
                "host": hc2.get("host"), "c5_host": hc5.get("host"),
                "path": "enet_pipeline_aead_* / enet_pipeline_aead_hmac_* (host_batch.cpp)"}
        if world == 1:
            fq = frame_queue_leg(dev.index)
            if fq is not None:
                host["frame_queue"] = fq
    long_recs = None
    if args.mode == "aead" and world == 1 and not args.no_long and (n, L) == (65536, 4096):
        long_recs = long_records_leg(dev)
    # every rank's placement (node, CPUs, CPU share) and its C5 share's pinned bytes / staging node
    placements = gather_placement(world, {**PLACEMENT_SHORT(), "c5_host": host.get("c5_host") if host else None})
    if ranks is not None and placements is not None:
        for r_, p_ in zip(ranks, placements):
            r_.update({k: v for k, v in p_.items() if k != "rank"})

    if rank == 0:
        total_bytes = n * L * args.steps * world
        value = total_bytes / elapsed / 2**30
        # algorithmic HBM bytes per launch: seal 2L+64, open 2L+65 per record
        # (xor: 2L + key/nonce/counter 48; wire: frames carry 48 more bytes; store: hashes/ids)
        seal_bytes = n * (2 * L + {"aead": 64, "xor": 48, "wire": 92, "store": 76}[args.mode]
                          + (4 if args.mode == "store" and args.store_ids == "given" else 0))
        open_bytes = n * (2 * L + {"aead": 65, "xor": 48, "wire": 81, "store": 109}[args.mode])
        seal_gbs = seal_bytes / (seal_ms * 1e-3) / 1e9
        open_gbs = open_bytes / (open_ms * 1e-3) / 1e9
        dom = "seal" if seal_ms >= open_ms else "open"
        dom_gbs = seal_gbs if dom == "seal" else open_gbs
        traffic = None
        pmc_note = None
        valu = None
        dom_s = (seal_ms if dom == "seal" else open_ms) * 1e-3
        blocks = n * ((L + 63) // 64)
        if args.mode in ("aead", "xor") and os.path.exists(VALU_CEILING_FILE):
            with open(VALU_CEILING_FILE) as f:
                ceil = json.load(f)
            key = "seal_open_Gblocks_per_s" if args.mode == "aead" else "xor_Gblocks_per_s"
            peak = ceil["isa_bound"][key]
            comp = ceil["compute_only"][key]
            achieved = blocks / dom_s / 1e9
            valu = {
                "achieved": round(achieved, 2),
                "peak": peak,
                "unit": "G ChaCha20 blocks/s (64 B) incl. Poly1305" if args.mode == "aead"
                        else "G ChaCha20 blocks/s (64 B)",
                "frac": round(achieved / peak, 4),
                "peak_is": "ISA bound of the instruction mix at 2.4 GHz, two waves per SIMD "
                           "(" + os.path.relpath(VALU_CEILING_FILE, ROOT) + " isa_bound)",
                "compute_only": comp,
                "frac_of_compute_only": round(achieved / comp, 4),
                "compute_only_is": "the same kernel with its memory waves idle "
                                   "(ENET_STREAM_DBG=257, " + os.path.relpath(VALU_CEILING_FILE, ROOT) + ")",
            }
        if os.path.exists(PMC_FILE):
            with open(PMC_FILE) as f:
                pmc = json.load(f)
            lanes = E.lanes_per_record(n, n * L, L)
            lg, md = lanes.bit_length() - 1, 1 if dom == "seal" else 2
            # the lockstep kernel (default for 64-byte-multiple records), else the 256-thread one
            k = None
            for want in (f"stream_kernel<{lg}, {md}, 0>", f"records_kernel_l<{lg}, {md}, 5>",
                         f"records_kernel<{lg}, {md}, 0, 1>"):
                k = k or next((v for name, v in pmc.get("kernels", {}).items() if want in name), None)
            if k and args.mode == "aead" and pmc.get("config") == {"records": n, "record_bytes": L}:
                traffic = k.get("hbm_bytes_per_launch")
                pmc_note = os.path.relpath(PMC_FILE, ROOT)
                if "SQ_INSTS_VALU" in k and valu is not None:
                    # wave64 VALU instructions per launch (PMC) over the kernel time measured
                    # live above: lane-ops/s against the full-rate issue peak, and cycles per
                    # instruction per SIMD (2.0 = every slot full-rate and paired)
                    ops = k["SQ_INSTS_VALU"] * 64
                    valu["lane_ops_Tps"] = round(ops / dom_s / 1e12, 2)
                    valu["issue_peak_Tps"] = VALU_ISSUE_PEAK_TOPS
                    valu["instr_per_64B_block"] = round(ops / blocks, 1)  # lane instructions
                    valu["cycles_per_instr_per_simd_at_2.4GHz"] = round(
                        dom_s * 2.4e9 * 1024 / k["SQ_INSTS_VALU"], 2)
                    valu["pmc_source"] = pmc_note
        out = {
            "metric": METRICS[args.mode],
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "prewarm_steps": prewarm_steps,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (torch.randint on device; random per-record keys and nonces)",
            "config": {
                "workload": f"{WORKLOADS.get((n, L), 'custom')}: {n} x {L} B records, "
                            + (f"{args.sessions} session keys (round-robin), per-record nonce"
                               if args.mode == "wire" and args.sessions else "per-record (key, nonce)")
                            + f", {MODE_DESC[args.mode]}, device-resident",
                "records_per_gpu": n,
                "record_bytes": L,
                "lanes_per_record": E.lanes_per_record(n, n * L, L),
                "parallelism": f"records split over {world} GPU(s), no collective",
                **({"chunk_ids": args.store_ids} if args.mode == "store" else {}),
            },
            "seal_ms": round(seal_ms, 4),
            "open_ms": round(open_ms, 4),
            "seal_gibs": round(n * L / (seal_ms * 1e-3) / 2**30, 1),
            "open_gibs": round(n * L / (open_ms * 1e-3) / 2**30, 1),
            "roofline": {
                "bound": "hbm",
                "kernel": (f"stream_kernel ({dom})" if args.mode in ("aead", "xor")
                           else f"{args.mode} {dom} kernel sequence"),
                "achieved": round(dom_gbs, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(dom_gbs / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "traffic_source": pmc_note,
                "algorithmic_bytes_per_launch": seal_bytes if dom == "seal" else open_bytes,
                "note": "power-capped: with the keystream and HBM streaming together the package sits "
                        "at ~1.38 kW and the shader clock drops to ~2.08 GHz (2.39 GHz with either alone); "
                        "in shader cycles the kernel is within 5 % of its compute-only form "
                        "(profiles/r02_power.txt); VALU work: see valu_roofline",
            },
            "valu_roofline": valu,
        }
        if power:
            out["power"] = power
        if long_recs:
            long_recs["vs_c2_value"] = {k: round(v["aead_tiles_gibs"] / value, 3)
                                        for k, v in long_recs.items() if isinstance(v, dict)}
            out["long_records"] = long_recs
        if host:
            out["host_resident"] = host
        out["placement"] = PLACEMENT
        if ranks is not None:
            out["dist"] = {"backend": dist.get_backend(), "world_size": dist.get_world_size(),
                           "per_rank": ranks}
        if not args.no_cpu_baseline and world == 1:
            if args.mode == "wire":  # the same workload through the reference itself
                ref = cpu_reference_frames(L, args.cpu_seconds)
                if ref is not None:
                    out["cpu_baseline"] = ref
            else:
                out["cpu_baseline"] = cpu_baseline(L, args.cpu_seconds)
                ref = cpu_reference_frames(L, args.cpu_seconds / 2)
                if ref is not None:
                    out["cpu_reference"] = ref
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
