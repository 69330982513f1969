"""C3-shape probe: where the single-array FIXING_FLOAT step's time goes.

Cases (10M f32 values + 10M uint64 keys, [KEY_CACHING, FIXING_FLOAT nb=1],
the bench's psf_node_roundtrip driver): min/max computed (the C3 line) or
preset on the filter (no min/max pass, no partials fold in the encode), with
3 rotating messages or 1.  Prints one JSON line per case: us per step and the
per-kernel averages from the evented diagnostic pass.

    python tools/c3_probe.py [--m 10000000] [--steps 200]
"""
import argparse
import json
import time

import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import parameter_server_amd.filter as F
from parameter_server_amd._lib import FIXING_FLOAT, KEY_CACHING


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=10_000_000)
    ap.add_argument("--steps", type=int, default=200)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    ctx = F.Context(0)
    m = a.m
    keys = torch.sort(torch.unique(torch.randint(0, 10**9, (m + m // 8,), device=dev, generator=g))[:m])[0]
    vals = [torch.randn(m, device=dev, generator=g, dtype=torch.float32) for _ in range(3)]
    for preset in (False, True):
        for nbuf in (3, 1):
            tmpls = []
            for i in range(nbuf):
                t = F.Message(request=True, push=True, key_channel=0, key_range=(0, 10**9))
                t.set_key(keys)
                t.add_value(vals[i])
                t.add_filter(KEY_CACHING)
                fp = [(float(vals[i].min()), float(vals[i].max()))] if preset else None
                t.add_filter(FIXING_FLOAT, num_bytes=1, fixed_point=fp)
                tmpls.append(t)
            worker, server = F.RemoteNode(ctx), F.RemoteNode(ctx)
            worker.roundtrip(server, tmpls, 20)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            worker.roundtrip(server, tmpls, a.steps)
            torch.cuda.synchronize()
            us = (time.perf_counter() - t0) / a.steps * 1e6
            ctx.profile(True)
            ctx.profile_reset()
            worker.roundtrip(server, tmpls, 20)
            torch.cuda.synchronize()
            prof = ctx.profile_read()
            ctx.profile(False)
            print(json.dumps({"preset": preset, "bufs": nbuf, "us_per_step": round(us, 2),
                              "kernels_us": {k: round(v[1] / v[0] * 1e3, 2) for k, v in prof.items()}}),
                  flush=True)


if __name__ == "__main__":
    main()
