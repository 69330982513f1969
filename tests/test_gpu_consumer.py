"""GPU: the server-side consumers through the C ABI
against the C restatements in oracle/psf_port.c:

* ParallelOrderedMatch (parallel_ordered_match.h:7-83) -- bit-exact, every op,
  k = 1 / 3 / 128, repeated keys, LDS-staged and global dst windows;
* the fused FIXING_FLOAT dequantise + match and the deferred decode path
  (RemoteNode decode leaves codes pending, the consumer dequantises);
* KVMap<Key, float, FTRLEntry> (kv_map.h:69-91, async_sgd.h:137-151) -- weights
  bit-exact after several pushes with table growth, nnz exact, the float sums
  within summation-order error; fused push of deferred codes.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _t(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def _keys(rng, n, hi):
    return np.unique(rng.integers(0, hi, int(n * 1.2) + 8).astype(np.uint64))[:n]


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("op", [0, 1, 2, 3, 4])
@pytest.mark.parametrize("shape", ["dense", "sparse"])
def test_ordered_match_vs_port(ctx, port, dtype, op, shape):
    rng = np.random.default_rng(op + (10 if shape == "dense" else 20))
    if shape == "dense":  # dst window per workgroup fits LDS
        dk = _keys(rng, 300_000, 1_000_000)
        sk = _keys(rng, 100_000, 1_000_000)
    else:  # src keys sparse in a huge dst: global-memory windows
        dk = _keys(rng, 2_000_000, 1 << 40)
        sk = np.sort(np.concatenate([dk[rng.choice(dk.size, 20_000, replace=False)],
                                     _keys(rng, 5_000, 1 << 40)]))
        sk = np.unique(sk)
    sv = (rng.standard_normal(sk.size) + 2).astype(dtype)
    dv = (rng.standard_normal(dk.size) + 2).astype(dtype)
    want = dv.copy()
    n_want = port.ordered_match(sk, sv, dk, want, 1, op)
    got = _t(dv)
    n = ctx.ordered_match(_t(sk.view(np.int64)), _t(sv), _t(dk.view(np.int64)), got, 1, op)
    assert n == n_want
    assert got.cpu().numpy().tobytes() == want.tobytes()


@pytest.mark.parametrize("k", [3, 128])
def test_ordered_match_rows(ctx, port, k):
    rng = np.random.default_rng(k)
    dk = _keys(rng, 20_000, 100_000)
    sk = _keys(rng, 8_000, 100_000)
    sv = rng.standard_normal(sk.size * k).astype(np.float32)
    dv = rng.standard_normal(dk.size * k).astype(np.float32)
    want = dv.copy()
    n_want = port.ordered_match(sk, sv, dk, want, k, 1)
    got = _t(dv)
    n = ctx.ordered_match(_t(sk.view(np.int64)), _t(sv), _t(dk.view(np.int64)), got, k, 1)
    assert n == n_want
    assert got.cpu().numpy().tobytes() == want.tobytes()


def test_ordered_match_repeated_keys_and_empty(ctx, port):
    rng = np.random.default_rng(5)
    dk = np.sort(rng.integers(0, 3000, 10_000).astype(np.uint64))  # many repeats
    sk = np.sort(rng.integers(0, 3000, 7_000).astype(np.uint64))
    sv = rng.standard_normal(sk.size).astype(np.float32)
    dv = np.zeros(dk.size, np.float32)
    want = dv.copy()
    n_want = port.ordered_match(sk, sv, dk, want, 1, 1)
    got = _t(dv)
    assert ctx.ordered_match(_t(sk.view(np.int64)), _t(sv), _t(dk.view(np.int64)), got, 1, 1) == n_want
    assert got.cpu().numpy().tobytes() == want.tobytes()
    e = torch.zeros(0, dtype=torch.int64, device=DEV)
    assert ctx.ordered_match(e, torch.zeros(0, device=DEV), _t(dk.view(np.int64)), got, 1, 1) == 0


@pytest.mark.parametrize("nb", [1, 2, 3])
def test_ff_decode_match_vs_port(ctx, port, nb):
    rng = np.random.default_rng(nb)
    dk = _keys(rng, 500_000, 10**9)
    sk = np.unique(np.concatenate([dk[::3], _keys(rng, 1000, 10**9)]))
    x = rng.standard_normal(sk.size).astype(np.float32)
    st, codes, mn, mx = port.ff_encode(x, nb, 99)
    st, dec = port.ff_decode(codes, nb, mn, mx, np.float32)
    dv = rng.standard_normal(dk.size).astype(np.float32)
    want = dv.copy()
    n_want = port.ordered_match(sk, dec, dk, want, 1, 1)
    got = _t(dv)
    n = ctx.ff_decode_match(_t(sk.view(np.int64)), _t(codes), nb, mn, mx, _t(dk.view(np.int64)), got, 1, 1)
    assert n == n_want
    assert got.cpu().numpy().tobytes() == want.tobytes()


def _push_message(F, keys, x, nb, channel=3):
    from parameter_server_amd import FIXING_FLOAT, KEY_CACHING
    m = F.Message(request=True, push=True, key_channel=channel, key_range=(0, 1 << 62))
    m.set_key(_t(keys.view(np.int64)))
    m.add_value(_t(x))
    m.add_filter(KEY_CACHING)
    m.add_filter(FIXING_FLOAT, num_bytes=nb)
    return m


def test_deferred_decode_and_message_match(ctx, port):
    """Worker encodes [KEY_CACHING, FIXING_FLOAT]; the server decodes with the
    dequantise deferred; KVVector::SetValue's merge consumes the codes; a
    materialised copy equals the normal decode."""
    from parameter_server_amd import filter as F
    F.set_clock(1234)
    try:
        rng = np.random.default_rng(11)
        keys = _keys(rng, 200_000, 1 << 62)
        x = rng.standard_normal(keys.size).astype(np.float32)
        worker, server, plain = F.RemoteNode(ctx), F.RemoteNode(ctx), F.RemoteNode(ctx)
        server.set_defer_dequant(True)
        m = _push_message(F, keys, x, 1)
        worker.encode(m)
        w1, w2 = m.clone(), m.clone()
        server.decode(w1)
        plain.decode(w2)
        nb, mn, mx = w1.pending(0)
        assert nb == 1 and w2.pending(0) is None
        dk = np.unique(np.concatenate([keys[::2], _keys(rng, 50_000, 1 << 62)]))
        dv = np.zeros(dk.size, np.float32)
        got = _t(dv)
        n = w1.ordered_match(ctx, 0, _t(dk.view(np.int64)), got, 1, 1)
        dec = plain.value(w2, 0).cpu().numpy().view(np.float32)
        want = dv.copy()
        assert n == port.ordered_match(keys, dec, dk, want, 1, 1)
        assert got.cpu().numpy().tobytes() == want.tobytes()
        w1.materialize(ctx)
        assert w1.pending(0) is None
        assert server.value(w1, 0).cpu().numpy().tobytes() == dec.tobytes()
    finally:
        F.set_clock(None)


def test_defer_rules(ctx, port):
    """[FIXING_FLOAT, COMPRESSING]: snappy decodes first, the codes can be left
    pending.  [NOISE, FIXING_FLOAT]: a value filter is listed before
    FIXING_FLOAT, so the dequantise is not deferred."""
    from parameter_server_amd import COMPRESSING, FIXING_FLOAT, NOISE
    from parameter_server_amd import filter as F
    x = torch.randn(10_000, device=DEV)
    for chain, deferred in (([FIXING_FLOAT, COMPRESSING], True), ([NOISE, FIXING_FLOAT], False)):
        m = F.Message(request=True, push=True)
        m.add_value(x.clone())
        for f in chain:
            m.add_filter(f, num_bytes=2 if f == FIXING_FLOAT else None)
        snd, rcv, plain = F.RemoteNode(ctx), F.RemoteNode(ctx), F.RemoteNode(ctx)
        rcv.set_defer_dequant(True)
        snd.encode(m)
        w, w2 = m.clone(), m.clone()
        rcv.decode(w)
        plain.decode(w2)
        assert (w.pending(0) is not None) == deferred
        w.materialize(ctx)
        assert rcv.value(w, 0).cpu().numpy().tobytes() == plain.value(w2, 0).cpu().numpy().tobytes()


@pytest.mark.parametrize("cfg", [(2, 0.05, 1.0, 1.0, 0.5), (2, 0.01, 10.0, 10.0, 1.0), (1, 0.1, 0.0, 0.0, 0.0)])
def test_kvmap_ftrl_vs_port(ctx, port, cfg):
    import oracle
    from parameter_server_amd import filter as F
    lr_type, alpha, beta, l1, l2 = cfg
    model = oracle.FtrlModel(port, lr_type, alpha, beta, l1, l2)
    kv = F.KVMap(ctx, capacity=1000, lr_type=lr_type, alpha=alpha, beta=beta, lambda1=l1, lambda2=l2)
    rng = np.random.default_rng(int(alpha * 1000))
    universe = _keys(rng, 60_000, 1 << 50)
    for step in range(5):  # overlapping key sets; the table grows past 1000
        keys = np.sort(rng.choice(universe, 25_000, replace=False))
        g = (rng.standard_normal(keys.size) * 2).astype(np.float32)
        assert model.push(keys, g) == 0
        kv.push(_t(keys.view(np.int64)), _t(g))
    probe = np.concatenate([universe, _keys(rng, 100, 1 << 50) + np.uint64(1 << 51)])
    got = kv.pull(_t(probe.view(np.int64))).cpu().numpy()
    assert got.tobytes() == model.pull(probe).tobytes()
    nnz, ws, ds, size = kv.stats()
    assert nnz == model.nnz.value
    assert size == len(model.index)
    w = model.pull(np.array(sorted(model.index), np.uint64)).astype(np.float64)
    assert ws >= 0 and abs(ws - float(model.weight_sum.value)) <= 1e-3 * max(1.0, ws)
    assert abs(ds - float(model.delta_sum.value)) <= 1e-3 * max(1.0, ds)
    assert (w != 0).sum() == nnz


def test_kvmap_fused_push_messages(ctx, port):
    """The async-SGD server path: push messages [KEY_CACHING, FIXING_FLOAT nb=1]
    decoded with the dequantise deferred into KVMap::SetValue, then a pull
    message answered by KVMap::GetValue."""
    import oracle
    from parameter_server_amd import filter as F
    F.set_clock(777)
    try:
        model = oracle.FtrlModel(port, 2, 0.01, 10.0, 0.5, 0.1)
        kv = F.KVMap(ctx, capacity=1 << 16, lr_type=2, alpha=0.01, beta=10.0, lambda1=0.5, lambda2=0.1)
        worker, server = F.RemoteNode(ctx), F.RemoteNode(ctx)
        server.set_defer_dequant(True)
        rng = np.random.default_rng(3)
        for step in range(4):
            keys = _keys(rng, 30_000, 1 << 40)
            x = (rng.standard_normal(keys.size) * 3).astype(np.float32)
            m = _push_message(F, keys, x, 1, channel=step)
            worker.encode(m)
            w = m.clone()
            server.decode(w)
            assert w.pending(0) is not None
            kv.set_value(w)
            st, codes, mn, mx = port.ff_encode(x, 1, 777)
            st, dec = port.ff_decode(codes, 1, mn, mx, np.float32)
            assert model.push(keys, dec) == 0
        allk = np.array(sorted(model.index), np.uint64)
        pull = F.Message(request=True, push=False)
        pull.set_key(_t(allk.view(np.int64)))
        kv.get_value(pull)
        assert pull.num_values() == 1
        got = server.value(pull, 0).cpu().numpy().view(np.float32)
        assert got.tobytes() == model.pull(allk).tobytes()
        assert kv.stats()[0] == model.nnz.value
    finally:
        F.set_clock(None)
