"""GPU: SliceKOFVMessage with keys/values resident in HBM (device lower_bound),
against the numpy restatement, then each slice through a FIXING_FLOAT +
KEY_CACHING RemoteNode pair (the per-server encode of executor.cc:131-146)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _keys(n, seed):
    rng = np.random.default_rng(seed)
    return np.unique(rng.integers(0, (1 << 64) - 1, size=n + 64, dtype=np.uint64))[:n]


@pytest.mark.parametrize("nserv", [1, 2, 5, 8])
@pytest.mark.parametrize("n", [0, 1, 3000, 200000])
def test_slice_device_keys(ctx, nserv, n):
    from oracle import slicing
    from parameter_server_amd import filter as F
    from parameter_server_amd import shard
    keys = _keys(n, nserv + n)
    v1 = np.random.default_rng(1).standard_normal(n).astype(np.float32)
    v2 = np.random.default_rng(2).standard_normal(2 * n).astype(np.float64)
    mr = shard.KEY_ALL if n < 10 else (int(keys[n // 10]), int(keys[-n // 10]))
    m = F.Message(request=True, push=True, key_range=mr)
    m.set_key(torch.from_numpy(keys.view(np.int64).copy()).cuda())
    m.add_value(torch.from_numpy(v1).cuda())
    m.add_value(torch.from_numpy(v2).cuda())
    ranges = shard.server_ranges(nserv)
    parts = shard.slice_message(ctx, m, ranges)
    want = slicing.slice_kofv(keys, [v1, v2], mr, ranges)
    torch.cuda.synchronize()
    for p, w in zip(parts, want):
        assert (p is None) == (w is None)
        if w is None:
            continue
        ptr, nb, loc = p.key_ptr()
        got = F.copy_out(ptr, nb, loc, "cpu").numpy()
        assert got.tobytes() == w[0].tobytes()
        for j, wv in enumerate(w[1]):
            vp, vb, vl = p.value_ptr(j)
            assert F.copy_out(vp, vb, vl, "cpu").numpy().tobytes() == wv.tobytes()


def test_slice_then_encode_per_server(ctx, port):
    """Each slice is encoded by its own sender node and decoded by the owner:
    the decoded values equal the port's FIXING_FLOAT round trip of that slice."""
    from oracle import slicing
    from parameter_server_amd import filter as F
    from parameter_server_amd import shard
    from parameter_server_amd._lib import FIXING_FLOAT, KEY_CACHING
    F.set_clock(1700000000)
    try:
        n, nserv = 100000, 4
        keys = _keys(n, 77)
        v = np.random.default_rng(3).standard_normal(n).astype(np.float32)
        m = F.Message(request=True, push=True, key_range=shard.KEY_ALL)
        m.set_key(torch.from_numpy(keys.view(np.int64).copy()).cuda())
        m.add_value(torch.from_numpy(v).cuda())
        parts = shard.slice_message(ctx, m, shard.server_ranges(nserv))
        want = slicing.slice_kofv(keys, [v], shard.KEY_ALL, shard.server_ranges(nserv))
        for p, w in zip(parts, want):
            snd, rcv = F.RemoteNode(ctx), F.RemoteNode(ctx)
            p.add_filter(KEY_CACHING)
            p.add_filter(FIXING_FLOAT, num_bytes=1)
            snd.encode(p)
            q = p.clone()
            rcv.decode(q)
            got = rcv.value(q, 0).cpu().numpy().view(np.float32)
            xs = w[1][0].view(np.float32)
            st, codes, mn, mx = port.ff_encode(xs, 1, 1700000000)
            assert st == 0
            st, dec = port.ff_decode(codes, 1, mn, mx, np.float32)
            assert got.tobytes() == dec.tobytes()
            assert rcv.key(q).cpu().numpy().view(np.uint64).tobytes() == w[0].tobytes()
    finally:
        F.set_clock(None)
