"""FIXING_FLOAT encode at 2^28: repeat the encode of one input several times
(codes must be identical every time and equal the C restatement's), and
compare the reference's floor((x - min) / bin * 254) computed with a true
division against torch's scalar division (which multiplies by a reciprocal)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle  # noqa: E402
from parameter_server_amd import filter as F  # noqa: E402

ctx = F.Context(0)
n = 1 << 28
torch.manual_seed(int(sys.argv[1]) if len(sys.argv) > 1 else 0)
x = torch.randn(n, device="cuda:0")
ref = None
for k in range(5):
    codes, mn, mx = ctx.ff_encode(x, 1, 12345)
    c = codes.clone()
    if ref is None:
        ref = c
    else:
        d = (c != ref).nonzero().flatten()
        print("run", k, "differs from run 0 at", d.numel(), "positions", d[:8].tolist(), flush=True)
mn64, mx64 = np.float64(mn), np.float64(mx)
xd = x.double().clamp(mn64, mx64) - mn64
t_scalar = torch.floor(xd / (mx64 - mn64) * 254.0).long()
t_true = torch.floor(xd / torch.tensor(mx64 - mn64, dtype=torch.float64, device="cuda:0") * 254.0).long()
bs, bt = ref.long() - t_scalar, ref.long() - t_true
print("scalar-division bit range", int(bs.min()), int(bs.max()), "true-division bit range", int(bt.min()), int(bt.max()),
      "floors differ at", int((t_scalar != t_true).sum()), flush=True)
st, pc, pmn, pmx = oracle.Port().ff_encode(x.cpu().numpy(), 1, 12345)
print("vs port: mismatches", int((ref.cpu().numpy() != pc).sum()), (mn, mx) == (pmn, pmx), flush=True)
