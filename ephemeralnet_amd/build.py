"""Build libenet_crypto.so in-tree with hipcc for gfx950 (no JIT cache: the .so travels with
the repo snapshot to the GPU box).  Each translation unit compiles to its own object in
parallel (the device code of one TU never calls into another), then one link step."""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "libenet_crypto.so")
OBJ = os.path.join(PKG, "build")
SOURCES = ["records.hip", "stream.hip", "sha.hip", "pow.hip", "duplex.hip", "capi.cpp", "crypto_api.cpp", "pipeline.cpp"]
HEADERS = ["enet_device.hpp", "enet_internal.hpp", "records_body.hpp"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CFLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++20", "-fPIC",
          "-fvisibility=hidden", "-Wall", "-Wno-unused-function",
          "-I" + os.path.join(ROOT, "include")]
LDFLAGS = ["--offload-arch=gfx950", "-fPIC", "-shared"]


def _headers() -> list[str]:
    deps = [os.path.join(CSRC, f) for f in HEADERS]
    for dp, _, fs in os.walk(os.path.join(ROOT, "include")):
        deps += [os.path.join(dp, f) for f in fs]
    return [d for d in deps if os.path.exists(d)]


def _obj(src: str) -> str:
    return os.path.join(OBJ, os.path.splitext(src)[0] + ".o")


def _stale_obj(src: str, hdr_t: float) -> bool:
    o = _obj(src)
    if not os.path.exists(o):
        return True
    t = os.path.getmtime(o)
    return os.path.getmtime(os.path.join(CSRC, src)) > t or hdr_t > t


def build(force: bool = False, verbose: bool = True, jobs: int | None = None) -> str:
    os.makedirs(OBJ, exist_ok=True)
    hdr_t = max((os.path.getmtime(h) for h in _headers()), default=0.0)
    todo = [s for s in SOURCES if force or _stale_obj(s, hdr_t)]
    if not todo and os.path.exists(LIB) and \
            os.path.getmtime(LIB) >= max(os.path.getmtime(_obj(s)) for s in SOURCES):
        return LIB

    def cc(src: str) -> None:
        cmd = [HIPCC] + CFLAGS + ["-c", os.path.join(CSRC, src), "-o", _obj(src) + ".tmp"]
        if verbose:
            print("[build]", " ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        os.replace(_obj(src) + ".tmp", _obj(src))

    n = jobs or min(len(todo) or 1, max(1, min(8, os.cpu_count() or 1)))
    with ThreadPoolExecutor(max_workers=n) as ex:
        for f in [ex.submit(cc, s) for s in todo]:
            f.result()
    tmp = LIB + ".tmp"
    cmd = [HIPCC] + LDFLAGS + [_obj(s) for s in SOURCES] + ["-o", tmp]
    if verbose:
        print("[build]", " ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
