"""Device FIXING_FLOAT codes against the C restatement at large sizes (a
diagnostic for grid-shape variants: PSF_LIBRARY_VARIANT=... python
tools/grid_check.py [log2 sizes...])."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle  # noqa: E402
from parameter_server_amd import filter as F  # noqa: E402

ctx = F.Context(0)
port = oracle.Port()
for lg in [int(a) for a in sys.argv[1:]] or [24, 26, 28]:
    n = 1 << lg
    torch.manual_seed(lg)
    xd = torch.randn(n, device="cuda:0")
    x = xd.cpu().numpy()
    codes, mn, mx = ctx.ff_encode(xd, 1, 12345)
    st, pc, pmn, pmx = port.ff_encode(x, 1, 12345)
    c = codes.cpu().numpy()
    bad = np.nonzero(c != pc)[0]
    print(lg, "mismatch", bad.size, (mn, mx) == (pmn, pmx), bad[:5], c[bad[:5]], pc[bad[:5]], flush=True)
