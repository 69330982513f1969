"""In-tree build of libpsf.so (HIP, gfx950) -- no JIT cache, no pip install.

`python -m parameter_server_amd.build` or __graft_entry__.build() compiles every
csrc/*.hip kernel file and the csrc/host/*.cc C++ host layer into
parameter_server_amd/libpsf.so with one hipcc invocation per object.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
OBJ = os.path.join(PKG, "build")
LIB = os.path.join(PKG, "libpsf.so")
ARCH = "gfx950"


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found")


def sources():
    out = []
    for d in (CSRC, os.path.join(CSRC, "host")):
        for f in sorted(os.listdir(d)):
            if f.endswith((".hip", ".cc")):
                out.append(os.path.join(d, f))
    return out


# -ffp-contract=off: the reference's double arithmetic must not be fused into
# FMAs (bit-parity).
COMMON = ["-O3", "-fPIC", "-std=c++17", "-ffp-contract=off", "-Wall", "-Wno-unused-function",
          "-I", os.path.join(os.path.dirname(PKG), "include")]


def _compile(src: str) -> str:
    rel = os.path.relpath(src, CSRC).replace(os.sep, "_")
    obj = os.path.join(OBJ, rel + ".o")
    deps = [src] + [os.path.join(CSRC, h) for h in os.listdir(CSRC) if h.endswith(".h")] + \
        [os.path.join(CSRC, "host", h) for h in os.listdir(os.path.join(CSRC, "host")) if h.endswith(".h")]
    if os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(d) for d in deps):
        return obj
    cmd = [_hipcc(), *COMMON, "-c", src, "-o", obj]
    if src.endswith(".hip"):
        cmd[1:1] = ["-x", "hip", f"--offload-arch={ARCH}"]
    subprocess.check_call(cmd)
    return obj


def build(verbose: bool = False) -> str:
    os.makedirs(OBJ, exist_ok=True)
    srcs = sources()
    with cf.ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(_compile, srcs))
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(o) for o in objs):
        cmd = [_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB, *objs]
        subprocess.check_call(cmd)
    if verbose:
        print(LIB)
    return LIB


if __name__ == "__main__":
    build(verbose=True)
    sys.exit(0)
