#!/usr/bin/env python3
"""Diagnostic: tests/test_gpu_batch.py's 48-message batch through
encode_many with ff_fused_batch, timed per call, and the fused counter lines
after each."""
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
os.environ.setdefault("PSF_FF_FUSED", "1")
import torch  # noqa: E402

from parameter_server_amd import filter as F  # noqa: E402
from parameter_server_amd._lib import lib  # noqa: E402
import test_gpu_batch as T  # noqa: E402

L = lib()
L.psf_debug_fused_ctl.argtypes = [C.c_void_p, C.POINTER(C.c_uint32), C.c_int]
ctx = F.Context(0)


def lines(k=8):
    buf = (C.c_uint32 * (32 * 64))()
    assert L.psf_debug_fused_ctl(ctx.h, buf, 32 * 64) == 0
    return [tuple(buf[32 * j:32 * j + 3]) for j in range(k)]


F.set_clock(987654)
cases = T._cases()
if len(sys.argv) > 1:  # the first k cases
    cases = cases[:int(sys.argv[1])]
print("start", lines(), flush=True)
for rep in range(3):
    snd = [F.RemoteNode(ctx) for _ in cases]
    mb = [T._message(F, *c, ch=i) for i, c in enumerate(cases)]
    t0 = time.perf_counter()
    F.RemoteNode.encode_many(snd, mb)
    t1 = time.perf_counter()
    ctx.sync()
    t2 = time.perf_counter()
    print(rep, f"encode_many {1e3 * (t1 - t0):.1f} ms, sync {1e3 * (t2 - t1):.1f} ms", lines(), flush=True)
    try:
        print("fixed points", [mb[i].fixed_points(1 if cases[i][3] is not None else 0) for i in range(3)], flush=True)
    except Exception as e:  # noqa: BLE001
        print("settle error", e, flush=True)
