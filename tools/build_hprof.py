#!/usr/bin/env python3
"""Diagnostic build: libpsf.so with -DPSF_HOST_PROF (host time per code
section, read by tools/host_prof.py) into tools/variants/hprof/ (git-ignored)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from parameter_server_amd import build as b  # noqa: E402

out = os.path.join(ROOT, "tools", "variants", "hprof")
os.makedirs(out, exist_ok=True)
b.build()
objs = []
for src in b.sources():
    rel = os.path.relpath(src, b.CSRC).replace(os.sep, "_")
    if src.endswith(".cc"):
        o = os.path.join(out, rel + ".o")
        subprocess.check_call([b._hipcc(), *b.COMMON, "-DPSF_HOST_PROF", "-c", src, "-o", o])
        objs.append(o)
    else:
        objs.append(os.path.join(b.OBJ, rel + ".o"))
subprocess.check_call([b._hipcc(), f"--offload-arch={b.ARCH}", "-shared", "-fPIC", "-o",
                       os.path.join(out, "libpsf.so"), *objs])
print(os.path.join(out, "libpsf.so"))
