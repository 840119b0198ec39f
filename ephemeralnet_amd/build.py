"""Build libenet_crypto.so in-tree with hipcc for gfx950 (no JIT cache: the .so travels with
the repo snapshot to the GPU box).  Each translation unit compiles to its own object in
parallel (the device code of one TU never calls into another), then one link step."""
from __future__ import annotations

import hashlib
import json
import os
import platform
import subprocess
import sys
import time
from concurrent.futures import ThreadPoolExecutor

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "libenet_crypto.so")
OBJ = os.path.join(PKG, "build")
# tools build: the host TUs that read -DENET_TOOLS_BUILD (the frame queue's stand-in device and
# stall hooks, per-phase profile, A/B knobs) recompiled with it and linked with the product's
# kernel objects; loaded only through ENET_LIB_PATH by tools/ and the queue's stand-in-device
# tests.  probes=True also recompiles the kernels (stream-kernel probes and schedule variants).
LIB_TOOLS = os.path.join(PKG, "libenet_crypto_tools.so")
OBJ_TOOLS = os.path.join(PKG, "build_tools")
SOURCES = ["records.hip", "segments.hip", "stream.hip", "sha.hip", "pow.hip", "duplex.hip", "duplex_split.hip",
           "capi.cpp", "chunk_hybrid.cpp", "crypto_api.cpp", "pipeline.cpp", "host_engine.cpp", "frame_queue.cpp", "host_batch.cpp",
           "host_topo.cpp"]
HEADERS = ["enet_device.hpp", "enet_internal.hpp", "records_body.hpp", "stream_common.hpp", "host_engine.hpp",
           "scalar.hpp", "host_batch.hpp", "host_topo.hpp"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CFLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++20", "-fPIC",
          "-fvisibility=hidden", "-Wall", "-Wno-unused-function",
          "-I" + os.path.join(ROOT, "include")]
LDFLAGS = ["--offload-arch=gfx950", "-fPIC", "-shared"]


DEVICE_HEADERS = ["enet_device.hpp", "enet_internal.hpp", "records_body.hpp", "stream_common.hpp",
                  "chacha_lockstep_asm.hpp"]


def _headers(src: str = "") -> list[str]:
    """Headers a source depends on: kernels (.hip) only the device headers; host C++ (.cpp) those,
    the host engine's and everything under include/."""
    if src.endswith(".hip"):
        return [os.path.join(CSRC, f) for f in DEVICE_HEADERS if os.path.exists(os.path.join(CSRC, f))]
    deps = [os.path.join(CSRC, f) for f in HEADERS + ["chacha_lockstep_asm.hpp"]]
    for dp, _, fs in os.walk(os.path.join(ROOT, "include")):
        deps += [os.path.join(dp, f) for f in fs]
    return [d for d in deps if os.path.exists(d)]


def _obj(src: str, obj_dir: str = OBJ) -> str:
    return os.path.join(obj_dir, os.path.splitext(src)[0] + ".o")


def tools_tus(probes: bool = False) -> list[str]:
    """TUs the tools build compiles with -DENET_TOOLS_BUILD (the others are the product's)."""
    out = []
    for f in SOURCES:
        if f.endswith(".hip") and not probes:
            continue
        with open(os.path.join(CSRC, f)) as fh:
            if "ENET_TOOLS_BUILD" in fh.read():
                out.append(f)
    return out


def source_digest(tools: bool = False) -> str:
    """SHA-256 over the compiler, the flags and the bytes of every source and header the library
    is built from (csrc/ and include/): what the built .so claims to be in its stamp file."""
    h = hashlib.sha256()
    # flags with the checkout's absolute include path made relative: the GPU box runs the same
    # tree from another directory and must compute the same digest
    flags = [f.replace(ROOT, ".") for f in CFLAGS + LDFLAGS] + (["-DENET_TOOLS_BUILD"] if tools else [])
    h.update(" ".join([os.path.basename(HIPCC)] + flags).encode())
    files = [os.path.join(CSRC, f) for f in SOURCES] + _headers()
    for f in sorted(set(files)):
        h.update(os.path.relpath(f, ROOT).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def tu_digest(src: str, tools: bool = False) -> str:
    """SHA-256 of one translation unit as compiled: flags, its source and the headers it depends
    on.  A TU is recompiled exactly when this differs from the stamp's record of it."""
    h = hashlib.sha256()
    flags = [f.replace(ROOT, ".") for f in CFLAGS] + (["-DENET_TOOLS_BUILD"] if tools else [])
    h.update(" ".join([os.path.basename(HIPCC)] + flags).encode())
    for f in [os.path.join(CSRC, src)] + sorted(_headers(src)):
        h.update(os.path.relpath(f, ROOT).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def stamp_path(lib: str = LIB) -> str:
    return lib + ".stamp.json"


def read_stamp(lib: str = LIB) -> dict | None:
    try:
        with open(stamp_path(lib)) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def build(force: bool = False, verbose: bool = True, jobs: int | None = None,
          tools: bool = False, probes: bool = False) -> str:
    obj_dir, lib = (OBJ_TOOLS, LIB_TOOLS) if tools else (OBJ, LIB)
    cflags = CFLAGS + (["-DENET_TOOLS_BUILD"] if tools else [])
    mine = tools_tus(probes) if tools else list(SOURCES)
    if tools:
        build(force=False, verbose=verbose, jobs=jobs)  # the product objects the rest links from
    objs = {s: _obj(s, obj_dir if s in mine else OBJ) for s in SOURCES}
    os.makedirs(obj_dir, exist_ok=True)
    digest = source_digest(tools) + ("+probes" if probes else "")
    stamp = read_stamp(lib) or {}
    # content, not mtimes, decides (a pushed .so beside edited sources, a checkout that reset
    # mtimes): a TU is recompiled when its own digest (flags + source + headers) differs from the
    # one the stamp recorded for the object, or the object is missing
    tus = {s: tu_digest(s, tools and s in mine) for s in SOURCES}
    old = stamp.get("tu_sha256", {}) if stamp.get("sources_sha256") else {}
    todo = [s for s in mine if force or old.get(s) != tus[s] or not os.path.exists(objs[s])]
    if not todo and os.path.exists(lib) and stamp.get("sources_sha256") == digest:
        print(f"[build] {os.path.relpath(lib, ROOT)} up to date (sources {digest[:12]}, nothing "
              "recompiled)", file=sys.stderr)
        return lib

    def cc(src: str) -> None:
        o = _obj(src, obj_dir)
        cmd = [HIPCC] + cflags + ["-c", os.path.join(CSRC, src), "-o", o + ".tmp"]
        if verbose:
            print("[build]", " ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        os.replace(o + ".tmp", o)

    n = jobs or min(len(todo) or 1, max(1, min(8, os.cpu_count() or 1)))
    with ThreadPoolExecutor(max_workers=n) as ex:
        for f in [ex.submit(cc, s) for s in todo]:
            f.result()
    tmp = lib + ".tmp"
    cmd = [HIPCC] + LDFLAGS + [objs[s] for s in SOURCES] + ["-o", tmp]
    if verbose:
        print("[build]", " ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, lib)
    with open(lib, "rb") as fh:
        lib_sha = hashlib.sha256(fh.read()).hexdigest()
    rec = {"sources_sha256": digest, "lib_sha256": lib_sha, "recompiled": todo, "tu_sha256": tus,
           "built_at": time.strftime("%Y-%m-%dT%H:%M:%S%z"), "host": platform.node()}
    with open(stamp_path(lib) + ".tmp", "w") as f:
        json.dump(rec, f, indent=1)
    os.replace(stamp_path(lib) + ".tmp", stamp_path(lib))
    print(f"[build] {os.path.relpath(lib, ROOT)} rebuilt: recompiled {len(todo)} of {len(SOURCES)} "
          f"TUs ({', '.join(todo)}), sources {digest[:12]}, lib {lib_sha[:12]}", file=sys.stderr)
    return lib


if __name__ == "__main__":
    build(force="--force" in sys.argv, tools="--tools" in sys.argv, probes="--probes" in sys.argv)
