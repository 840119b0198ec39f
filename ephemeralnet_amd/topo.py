"""Where a rank's host work runs, read from sysfs WITHOUT initialising the GPU (bench.py pins each
rank and its host children before its first HIP call): the NUMA node of every GPU from the KFD
topology (HIP's device order) and its PCI function, the CPUs of a node, the process's affinity
mask and cgroup CPU quota.  The library reads the same facts through HIP (enet_device_numa_node,
csrc/host_topo.cpp); tests/test_gpu_host_topology.py checks that the two agree on the box."""
from __future__ import annotations

import os


def _read(path: str) -> str | None:
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def parse_cpulist(s: str | None) -> list[int]:
    out: set[int] = set()
    for part in (s or "").split(","):
        part = part.strip()
        if not part:
            continue
        a, _, b = part.partition("-")
        try:
            lo, hi = int(a), int(b or a)
        except ValueError:
            continue
        out.update(range(lo, hi + 1))
    return sorted(out)


def format_cpulist(cpus) -> str:
    cpus = sorted(set(cpus))
    parts, i = [], 0
    while i < len(cpus):
        j = i
        while j + 1 < len(cpus) and cpus[j + 1] == cpus[j] + 1:
            j += 1
        parts.append(str(cpus[i]) if i == j else f"{cpus[i]}-{cpus[j]}")
        i = j + 1
    return ",".join(parts)


def _visible(n: int) -> list[int]:
    """Indices of the KFD GPUs HIP exposes, in HIP's order (ROCR_/HIP_/CUDA_VISIBLE_DEVICES as
    plain index lists; anything else: all)."""
    idx = list(range(n))
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is None:
            continue
        try:
            sel = [int(x) for x in v.split(",") if x.strip() != ""]
        except ValueError:
            continue
        idx = [idx[i] for i in sel if 0 <= i < len(idx)]
    return idx


def gpu_pci_functions() -> list[str]:
    """PCI functions ("0000:75:00.0") of the GPUs in KFD node order (HIP device order)."""
    base = "/sys/class/kfd/kfd/topology/nodes"
    try:
        nodes = sorted((int(d) for d in os.listdir(base) if d.isdigit()))
    except OSError:
        return []
    out = []
    for nd in nodes:
        props = {}
        for line in (_read(f"{base}/{nd}/properties") or "").splitlines():
            k, _, v = line.partition(" ")
            props[k] = v.strip()
        try:
            if int(props.get("simd_count", "0")) <= 0:
                continue  # a CPU node
            loc, dom = int(props.get("location_id", "0")), int(props.get("domain", "0"))
        except ValueError:
            continue
        out.append(f"{dom:04x}:{loc >> 8:02x}:{(loc >> 3) & 0x1f:02x}.{loc & 7:x}")
    return [out[i] for i in _visible(len(out))]


def gpu_numa_node(index: int) -> int:
    """NUMA node of HIP device `index` (-1 unknown)."""
    fns = gpu_pci_functions()
    if not 0 <= index < len(fns):
        return -1
    try:
        v = int(_read(f"/sys/bus/pci/devices/{fns[index]}/numa_node") or "-1")
    except ValueError:
        return -1
    return v if v >= 0 else -1


def numa_nodes() -> list[int]:
    return parse_cpulist(_read("/sys/devices/system/node/online")) or [0]


def node_cpus(node: int) -> list[int]:
    return parse_cpulist(_read(f"/sys/devices/system/node/node{node}/cpulist")) if node >= 0 else []


def allowed_cpus() -> list[int]:
    try:
        return sorted(os.sched_getaffinity(0))
    except AttributeError:
        return list(range(os.cpu_count() or 1))


def cgroup_quota_cpus() -> int | None:
    """cgroup v2 cpu.max of this process's cgroup and its ancestors (the least), None = unlimited."""
    best = None
    path = ""
    for line in (_read("/proc/self/cgroup") or "").splitlines():
        if line.startswith("0::"):
            path = line[3:]
    cands = []
    p = path
    while True:
        cands.append(f"/sys/fs/cgroup{p}/cpu.max")
        if not p or p == "/":
            break
        p = p.rsplit("/", 1)[0]
    cands.append("/sys/fs/cgroup/cpu.max")
    for c in cands:
        v = _read(c)
        if not v:
            continue
        q, _, per = v.partition(" ")
        try:
            if q != "max" and int(q) > 0 and int(per) > 0:
                n = max(1, -(-int(q) // int(per)))
                best = n if best is None else min(best, n)
        except ValueError:
            pass
    return best


def rank_placement(local_rank: int, local_world: int) -> dict:
    """Where rank `local_rank` of `local_world` ranks on this node should run: its GPU's node
    CPUs within the affinity mask (the whole mask when the node is unknown or outside it) and
    its share of the CPU budget (min(mask, quota) / ranks, at least 1)."""
    allowed = allowed_cpus()
    # the rank's GPU: cuda:(local_rank mod GPUs), as bench.py binds it (ranks share the card when
    # there are fewer GPUs than ranks -- the one-GPU rehearsal of N = 2 / 8)
    fns = gpu_pci_functions()
    node = gpu_numa_node(local_rank % len(fns) if fns else local_rank)
    cpus = sorted(set(node_cpus(node)) & set(allowed)) or allowed
    q = cgroup_quota_cpus()
    budget = min(len(allowed), q) if q else len(allowed)
    share = max(1, budget // max(1, local_world))
    return {"numa_node": node, "cpus": cpus, "cpu_budget": share}


def apply_placement(pl: dict) -> None:
    """Pin this process (and the children it starts afterwards) to pl["cpus"] and hand the
    library its CPU share (ENET_HOST_CPUS, read when its first engine plans its threads)."""
    try:
        os.sched_setaffinity(0, pl["cpus"])
    except (AttributeError, OSError):
        pass
    os.environ["ENET_HOST_CPUS"] = str(pl["cpu_budget"])
