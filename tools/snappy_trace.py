#!/usr/bin/env python3
"""Phase timeline of the snappy compress kernel (diagnostic).

Builds a libpsf variant with -DPSF_SNAPPY_TRACE (tools/variants/trace/) and
loads it: python tools/snappy_trace.py --build (here, on CPU), then on the GPU
box python tools/snappy_trace.py --run [--mib 128] [--kind codes|keys|random].
Prints per-fragment statistics of the compress pipeline: the probe (0->4),
the placement (2->3), and the spans of both launches.
"""
import argparse
import ctypes as C
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VAR = os.path.join(ROOT, "tools", "variants", "trace")


def build(src=None):
    sys.path.insert(0, ROOT)
    from parameter_server_amd import build as b
    b.build()
    os.makedirs(VAR, exist_ok=True)
    objs = [os.path.join(b.OBJ, f) for f in sorted(os.listdir(b.OBJ)) if f.endswith(".o") and f != "snappy.hip.o"]
    obj = os.path.join(VAR, "snappy.o")
    subprocess.check_call([b._hipcc(), "-x", "hip", f"--offload-arch={b.ARCH}", *b.COMMON, "-DPSF_SNAPPY_TRACE",
                           "-I", b.CSRC, "-c", src or os.path.join(b.CSRC, "snappy.hip"), "-o", obj])
    subprocess.check_call([b._hipcc(), f"--offload-arch={b.ARCH}", "-shared", "-fPIC", "-o",
                           os.path.join(VAR, "libpsf.so"), *objs, obj])
    print(os.path.join(VAR, "libpsf.so"))


def run(mib, kind, dfrag=False):
    os.environ["PSF_LIBRARY_VARIANT"] = os.path.join(VAR, "libpsf.so")
    sys.path.insert(0, ROOT)
    import numpy as np
    import torch

    from parameter_server_amd import filter as F
    from parameter_server_amd._lib import lib
    n = mib << 20
    g = torch.Generator(device="cuda").manual_seed(3)
    if kind == "codes":
        x = (torch.randn(n, device="cuda", generator=g) * 30 + 128).clamp(0, 255).to(torch.uint8)
    elif kind == "keys":
        x = torch.sort(torch.randint(0, 10**9, (n // 8,), device="cuda", generator=g))[0].view(torch.uint8)
    elif kind == "ff":  # FIXING_FLOAT nb=1 codes of N(0, 1) values, as C5's
        v = torch.randn(n, device="cuda", generator=g)
        x = ((v - v.min()) / (v.max() - v.min()) * 255 + 0.5).floor().to(torch.uint8)
    else:
        x = torch.randint(0, 256, (n,), device="cuda", dtype=torch.uint8, generator=g)
    ctx = F.Context(0)
    for _ in range(3):
        ctx.snappy_compress(x)
    torch.cuda.synchronize()
    nfrag = (n + 65535) // 65536
    buf = np.zeros(nfrag * 6, np.uint64)
    L = lib()
    L.psf_debug_snappy_trace.argtypes = [C.c_void_p, C.c_size_t]
    assert L.psf_debug_snappy_trace(buf.ctypes.data, buf.nbytes) == 0
    if dfrag:
        s = ctx.snappy_compress(x)
        for _ in range(2):
            ctx.snappy_uncompress(s)
        torch.cuda.synchronize()
        L.psf_debug_dfrag_trace.argtypes = [C.c_void_p, C.c_size_t]
        db = np.zeros(nfrag * 4, np.uint64)
        assert L.psf_debug_dfrag_trace(db.ctypes.data, db.nbytes) == 0
        d = db.reshape(nfrag, 4).astype(np.int64)
        t0 = d[:, 0].min()
        work = np.nonzero(d[:, 1] >= t0)[0]
        dur = (d[:, 2] - d[:, 0]) * 10.0 / 1000
        print(json.dumps({"dfrag_span_us": round(float((d[:, 2].max() - t0) * 10 / 1000), 1),
                          "working": int(work.size), "first_working": int(work.min()) if work.size else None,
                          "slowest": [(int(i), round(float(dur[i]), 1)) for i in np.argsort(-dur)[:5]],
                          "start_spread_us": round(float((np.sort(d[:, 0])[-1] - t0) * 10 / 1000), 1)}))
        return
    t = buf.reshape(nfrag, 6).astype(np.int64)
    ns = lambda a: a * 10.0  # noqa: E731  (100 MHz clock)
    q = lambda a: {p: round(float(np.percentile(a, p)) / 1000, 2) for p in (10, 50, 90, 99)}  # noqa: E731
    t0 = t[:, 0].min()
    probe = ns(t[:, 4] - t[:, 0])
    place = ns(t[:, 3] - t[:, 2])
    mt = t[:, 1] > t[:, 4]  # slot 1 after the probe: the fragment was parsed
    split = {"parsed_frags": int(mt.sum()),
             "parse_us": sorted(round(float(a) / 1000, 1) for a in ns(t[mt, 1] - t[mt, 4]))[-8:],
             "parse_end_us": round(ns(t[mt, 1].max() - t0) / 1000, 1)} if mt.any() else {}
    print(json.dumps({"kind": kind, "mib": mib, "frags": nfrag,
                      "probe_span_us": round(ns(t[:, 4].max() - t0) / 1000, 1),
                      "probe_start_spread_us": round(ns(t[:, 0].max() - t0) / 1000, 1),
                      "probe_us": q(probe),
                      "probe_to_place_us": round(ns(t[:, 2].min() - t[:, 4].max()) / 1000, 1),
                      "place_span_us": round(ns(t[:, 3].max() - t[:, 2].min()) / 1000, 1),
                      "place_us": q(place),
                      "place_start_spread_us": round(ns(t[:, 2].max() - t[:, 2].min()) / 1000, 1), **split}))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--run", action="store_true")
    ap.add_argument("--mib", type=int, default=128)
    ap.add_argument("--kind", default="codes")
    ap.add_argument("--dfrag", action="store_true", help="per-fragment times of the decoder's K4")
    ap.add_argument("--name", default="trace", help="variant directory under tools/variants")
    ap.add_argument("--src", default=None, help="build: snappy.hip to trace (default: csrc/snappy.hip)")
    a = ap.parse_args()
    VAR = os.path.join(ROOT, "tools", "variants", a.name)
    if a.build:
        build(a.src)
    if a.run:
        run(a.mib, a.kind, a.dfrag)
