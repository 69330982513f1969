#!/usr/bin/env python3
"""Does FIXING_FLOAT encode on one stream overlap with snappy compress on
another?  C5's shape: 8 slices of 2^24 f32 values; baseline = all on one
stream; overlapped = encodes queued on stream A, each slice's compress on
stream B behind an event.  Prints both times (GPU box)."""
import time

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from parameter_server_amd import filter as F


def main():
    n, S = 1 << 24, 8
    g = torch.Generator(device="cuda").manual_seed(5)
    xs = [torch.randn(n, device="cuda", generator=g) for _ in range(S)]
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    A, B = F.Context(0, sa), F.Context(0, sb)
    codes = [torch.empty(n, dtype=torch.uint8, device="cuda") for _ in range(S)]
    rng = [torch.empty(4, dtype=torch.float32, device="cuda") for _ in range(S)]
    cap = 32 + n + n // 6
    comp = [torch.empty(cap, dtype=torch.uint8, device="cuda") for _ in range(S)]

    def seq():
        for i in range(S):
            A.ff_encode_async(xs[i], 1, 7, codes[i], rng[i])
        for i in range(S):
            A.snappy_compress(codes[i], comp[i])

    def ovl():
        evs = []
        for i in range(S):
            A.ff_encode_async(xs[i], 1, 7, codes[i], rng[i])
            e = torch.cuda.Event()
            e.record(sa)
            evs.append(e)
        for i in range(S):
            sb.wait_event(evs[i])
            B.snappy_compress(codes[i], comp[i])

    for name, fn in (("sequential", seq), ("overlapped", ovl), ("sequential", seq), ("overlapped", ovl)):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        print(name, round((time.perf_counter() - t0) / 5 * 1e6, 1), "us per 8 slices", flush=True)


if __name__ == "__main__":
    main()
