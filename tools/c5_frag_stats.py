#!/usr/bin/env python3
"""Diagnostic: the fragments of bench.py's C5 slices whose snappy 1.1.8 parse
is not one literal (the port's compressor on the port's codes), and how many
bytes each one gains or loses against the stored literal.  Same data as
`bench.py --config c5` (torch generator seed 1, device values)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle  # noqa: E402
from bench import splitmix64_keys  # noqa: E402
from parameter_server_amd import shard  # noqa: E402

port = oracle.Port()
M, DIM, S = 1 << 20, 128, 8
g = torch.Generator(device="cuda:0")
g.manual_seed(1)
keys = splitmix64_keys(M, 4)
vals = torch.randn(keys.size * DIM, device="cuda:0", generator=g, dtype=torch.float32).cpu().numpy()
ranges = shard.server_ranges(S)
b = np.array([r[0] for r in ranges] + [ranges[-1][1]], dtype=np.uint64)
pos = np.searchsorted(keys, b)
for d in range(S):
    v = vals[pos[d] * DIM:pos[d + 1] * DIM]
    st, codes, mn, mx = port.ff_encode(v, 1, 12345)
    nf = (codes.size + 65535) // 65536
    out = []
    for k in range(nf):
        fr = codes[k * 65536:(k + 1) * 65536].tobytes()
        if len(fr) < 65536:
            continue
        c = port.snappy_compress(fr)
        if len(c) != 3 + 3 + 65536:
            out.append((k, len(c) - 65542))
    print(d, nf, out, flush=True)
