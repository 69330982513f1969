"""Debug: compare the device standard-normal table against the port."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import oracle  # noqa: E402
from parameter_server_amd import NOISE  # noqa: E402
from parameter_server_amd import filter as F  # noqa: E402

P = oracle.Port()
ctx = F.Context(0)
node = F.RemoteNode(ctx)
for dt in (np.float32, np.float64):
    n = 100000
    x = np.zeros(n, dt)
    t = torch.from_numpy(x.copy()).cuda()
    m = F.Message()
    m.add_value(t)
    m.add_filter(NOISE, noise=(0.0, 1.0))
    node.encode(m)
    ctx.sync()
    got = t.cpu().numpy()
    want = P.add_noise(x, 0.0, 1.0)
    it = np.int32 if dt == np.float32 else np.int64
    d = got.view(it).astype(np.int64) - want.view(it).astype(np.int64)
    bad = np.nonzero(d)[0]
    print(dt.__name__, "mismatch frac", len(bad) / n, "first", bad[:10], "ulp", d[bad[:10]])
    print(" got", got[bad[:5]], "want", want[bad[:5]])
    print(" first 6 got", got[:6], "want", want[:6])
