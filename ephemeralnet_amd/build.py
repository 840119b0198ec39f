"""Build libenet_crypto.so in-tree with hipcc for gfx950 (no JIT cache: the .so travels with
the repo snapshot to the GPU box)."""
from __future__ import annotations

import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "libenet_crypto.so")
SOURCES = ["records.hip", "sha.hip", "pow.hip", "frames.hip", "capi.cpp", "crypto_api.cpp", "pipeline.cpp"]
HEADERS = ["enet_device.hpp", "enet_internal.hpp"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++20", "-fPIC", "-shared",
         "-fvisibility=hidden", "-Wall", "-Wno-unused-function",
         "-I" + os.path.join(ROOT, "include")]


def _stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS]
    inc = os.path.join(ROOT, "include")
    for dp, _, fs in os.walk(inc):
        deps += [os.path.join(dp, f) for f in fs]
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(force: bool = False, verbose: bool = True) -> str:
    if not force and not _stale():
        return LIB
    srcs = [os.path.join(CSRC, f) for f in SOURCES if os.path.exists(os.path.join(CSRC, f))]
    tmp = LIB + ".tmp"
    cmd = [HIPCC] + FLAGS + srcs + ["-o", tmp]
    if verbose:
        print("[build]", " ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
