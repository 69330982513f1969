"""Debug: isolate the filter-level path (RemoteNode) vs the kernel API."""
import faulthandler
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
faulthandler.enable()
import oracle  # noqa: E402
from parameter_server_amd import FIXING_FLOAT, KEY_CACHING  # noqa: E402
from parameter_server_amd import filter as F  # noqa: E402

P = oracle.Port()
ctx = F.Context(0)
print("ctx stream", ctx.stream.cuda_stream, flush=True)
F.set_clock(12345)
n = 100_003
x = np.random.default_rng(1).standard_normal(n).astype(np.float32)
xt = torch.from_numpy(x).cuda()
torch.cuda.synchronize()

# 1: kernel API
codes, mn, mx = ctx.ff_encode(xt, 1, 12345)
st, pc, pmn, pmx = P.ff_encode(x, 1, 12345)
print("kernel api equal:", np.array_equal(codes.cpu().numpy(), pc), mn, mx, pmn, pmx, flush=True)

# 2: FF-only message through a node
node = F.RemoteNode(ctx)
m = F.Message()
m.add_value(xt)
fi = m.add_filter(FIXING_FLOAT, num_bytes=1)
node.encode(m)
print("encoded; fixed points", m.fixed_points(fi), flush=True)
p, nb, loc = m.value_ptr(0)
print("value ptr", hex(p), nb, loc, flush=True)
ctx.sync()
got = node.value(m, 0).cpu().numpy()
print("node path equal:", np.array_equal(got, pc), "ndiff", int((got != pc).sum()), got[:8], pc[:8], flush=True)

# 3: KC with device keys
keys = torch.arange(1000, dtype=torch.int64, device="cuda") * 7
print("key sig kernel api", ctx.key_signature(keys), P.key_signature(keys.cpu().numpy()), flush=True)
m2 = F.Message(request=True, push=True, key_channel=1, key_range=(0, 1 << 40))
m2.set_key(keys)
m2.add_filter(KEY_CACHING)
print("kc encode...", flush=True)
node.encode(m2)
print("kc sig", m2.signature(0), flush=True)
