#!/usr/bin/env python3
"""Per-kernel HIP-event timings of the FIXING_FLOAT kernels under variants of
the call (computed vs preset range, nb), 2^27 f32 values over rotating
buffers.  Diagnostic only."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    from parameter_server_amd import filter as F
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 27
    dev = "cuda:0"
    ctx = F.Context(0)
    xs = [torch.randn(n, device=dev) for _ in range(3)]
    out = {}
    for nb in (1, 2, 3):
        codes = torch.empty(n * nb, dtype=torch.uint8, device=dev)
        rng = torch.empty(2, dtype=torch.float32, device=dev)
        dec = torch.empty(n, device=dev)
        for preset in (False, True):
            kw = dict(mn=-5.0, mx=5.0) if preset else {}
            for i in range(6):
                ctx.ff_encode_async(xs[i % 3], nb, 12345, codes, rng, **kw)
            torch.cuda.synchronize()
            ctx.profile(True)
            ctx.profile_reset()
            for i in range(30):
                ctx.ff_encode_async(xs[i % 3], nb, 12345, codes, rng, **kw)
                ctx.ff_decode_async(codes, nb, rng, dec)
            torch.cuda.synchronize()
            r = ctx.profile_read()
            ctx.profile(False)
            out[f"nb{nb}_{'preset' if preset else 'computed'}"] = {
                k: {"us": round(v[1] / v[0] * 1e3, 2), "GBps": round(v[2] / v[1] * 1e-6, 1)} for k, v in r.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
