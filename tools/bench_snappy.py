#!/usr/bin/env python3
"""COMPRESSING codec throughput on one GPU (diagnostic, not the bench.py line).

For each synthetic payload: device compress / uncompress wall time (synchronous
C-ABI calls, HBM-resident), the compressor kernel time from the libpsf event
profiler, and the reference's snappy 1.1.8 on one host core (the library, when
present) on a bounded sample.  Prints one JSON line per payload.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def payloads(mib):
    n = mib << 20
    g = torch.Generator(device="cuda").manual_seed(3)
    keys = torch.sort(torch.randint(0, 10**9, (n // 8,), device="cuda", generator=g))[0]
    codes = (torch.randn(n, device="cuda", generator=g) * 30 + 128).clamp(0, 255).to(torch.uint8)
    rnd = torch.randint(0, 256, (n,), device="cuda", dtype=torch.uint8, generator=g)
    zeros = torch.zeros(n, dtype=torch.uint8, device="cuda")
    return {"sorted_keys_1e9": keys.view(torch.uint8), "ff_codes_nb1": codes, "random": rnd, "zeros": zeros}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=64)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--cpu-mib", type=int, default=8)
    ap.add_argument("--only", default=None, help="comma-separated payload names")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-check", action="store_true", help="diagnostic builds that emit nothing")
    ap.add_argument("--no-verify", action="store_true", help="diagnostic decoders: time the uncompress, skip the comparison")
    a = ap.parse_args()
    from parameter_server_amd import filter as F
    ctx = F.Context(0)
    ref = None
    try:
        if a.no_cpu:
            raise ImportError
        import oracle
        ref = oracle.Snappy118()  # the library the reference links, where the image has it
    except Exception:
        pass
    for name, x in payloads(a.mib).items():
        if a.only and name not in a.only.split(","):
            continue
        nbytes = x.numel()
        s = ctx.snappy_compress(x)  # warm
        if not a.no_check:
            back = ctx.snappy_uncompress(s)
            assert a.no_verify or torch.equal(back, x.view(torch.uint8))
        ctx.profile(True, ["snappy_compress", "snappy_decompress"])
        ctx.profile_reset()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            s = ctx.snappy_compress(x)
        torch.cuda.synchronize()
        tc = (time.perf_counter() - t0) / a.reps
        t0 = time.perf_counter()
        for _ in range(0 if a.no_check else a.reps):
            back = ctx.snappy_uncompress(s)
        torch.cuda.synchronize()
        td = max(time.perf_counter() - t0, 1e-9) / a.reps
        prof = ctx.profile_read()
        ctx.profile(False)
        rec = {"payload": name, "bytes": nbytes, "compressed": int(s.numel()),
               "ratio": round(s.numel() / nbytes, 4),
               "gpu_compress_GBps": round(nbytes / tc / 1e9, 2),
               "gpu_uncompress_GBps": None if a.no_check else round(nbytes / td / 1e9, 2)}
        for k, (nl, ms, _) in prof.items():
            rec[f"{k}_kernel_ms"] = round(ms / nl, 3)
        if ref is not None:
            cpu_n = min(nbytes, a.cpu_mib << 20)
            xb = x.view(torch.uint8)[:cpu_n].cpu().numpy().tobytes()
            t0 = time.perf_counter()
            cs = ref.snappy_compress(xb)
            t1 = time.perf_counter()
            st, _ = ref.snappy_uncompress(cs, cap=cpu_n)
            t2 = time.perf_counter()
            rec["cpu_ref_compress_GBps"] = round(cpu_n / (t1 - t0) / 1e9, 3)
            rec["cpu_ref_uncompress_GBps"] = round(cpu_n / (t2 - t1) / 1e9, 3)
            rec["cpu_sample_bytes"] = cpu_n
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
