#!/usr/bin/env python3
"""Phase timeline of C5 + COMPRESSING's compress (diagnostic): bench.py's C5
workload (hits, or --miss) run a few steps against the -DPSF_SNAPPY_TRACE
variant (python tools/snappy_trace.py --build first), then the last compress
launch's per-fragment phases: probe (0 -> 4), parse end (1, parsed fragments
only), placement (2 -> 3)."""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["PSF_LIBRARY_VARIANT"] = os.path.join(ROOT, "tools", "variants", "trace", "libpsf.so")
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch

    import bench
    from parameter_server_amd import filter as F
    from parameter_server_amd._lib import lib
    args = bench.parse(["--config", "c5", "--compress"] + sys.argv[1:])
    ctx = F.Context(0)
    g = torch.Generator(device="cuda").manual_seed(1)
    run, *_ = bench.build_workload(args, F, ctx, 0, 1, torch.device("cuda:0"), g, 0)
    run(4)
    torch.cuda.synchronize()
    nfrag = 1 << 14
    buf = np.zeros(nfrag * 6, np.uint64)
    L = lib()
    L.psf_debug_snappy_trace.argtypes = [C.c_void_p, C.c_size_t]
    assert L.psf_debug_snappy_trace(buf.ctypes.data, buf.nbytes) == 0
    t = buf.reshape(nfrag, 6).astype(np.int64)
    t = t[t[:, 0] > 0]
    t0 = t[:, 0].max() - 5000  # the last launch: its probes start within 50 us
    t = t[t[:, 0] > t0]
    t0 = t[:, 0].min()
    us = lambda a: round(float(a) * 10 / 1000, 1)  # noqa: E731  (100 MHz clock)
    probe = (t[:, 4] - t[:, 0]) * 10 / 1000
    mt = t[:, 1] > t[:, 4]
    out = {"frags": int(len(t)), "probe_span_us": us(t[:, 4].max() - t0),
           "probe_us_p50_p99": [round(float(np.percentile(probe, p)), 2) for p in (50, 99)],
           "parsed": int(mt.sum()),
           "parsed_frags": [{"probe_end_us": us(a[4] - t0), "parse_us": us(a[1] - a[4]), "wg": int(a[5])} for a in t[mt]],
           "place_start_us": us(t[:, 2].min() - t0) if (t[:, 2] > t0).any() else None,
           "place_end_us": us(t[:, 3].max() - t0) if (t[:, 3] > t0).any() else None}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
