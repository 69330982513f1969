"""GPU: the batched FIXING_FLOAT encode on C4's shape -- hundreds of slices
of ~2^18 values (64 or 65 tiles each) starting at unaligned offsets of one
buffer, computed, half-preset and preset ranges, nb 1-3, f32 / f64, and the
stored layout COMPRESSING reads.  Codes, side-info and decoded values must
equal the C restatement (fixing_float.h:50-101)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
SEED = 4242


def _slices(rng, count, base_n, dt=np.float32):
    total = count * (base_n + 600) + 16
    buf = (rng.standard_normal(total) * 3).astype(dt)
    out, at = [], 1
    for k in range(count):
        n = base_n + int(rng.integers(-520, 520))  # 64 or 65 tiles around 2^18
        out.append((at, n))
        at += n + int(rng.integers(0, 3))
    return buf, out


def _encode(F, ctx, buf_t, sl, nb, presets, compress=False):
    from parameter_server_amd import COMPRESSING, FIXING_FLOAT
    msgs = []
    for i, (at, n) in enumerate(sl):
        m = F.Message(request=True, push=True, key_channel=i)
        m.add_value(buf_t[at:at + n])
        p = presets(i)
        m.add_filter(FIXING_FLOAT, num_bytes=nb, fixed_point=None if p is None else [p])
        if compress:
            m.add_filter(COMPRESSING)
        msgs.append(m)
    snd = [F.RemoteNode(ctx) for _ in msgs]
    F.RemoteNode.encode_many(snd, msgs)
    return snd, msgs


def _presets(i):
    return [None, None, None, (-1.0, None), (None, 2.5), (-4.0, 4.0)][i % 6]


@pytest.mark.parametrize("count,nb,dt", [(512, 1, np.float32), (200, 2, np.float32), (96, 3, np.float64),
                                         (64, 1, np.float32)])
def test_c4_shaped_batch(count, nb, dt):
    import oracle
    from parameter_server_amd import filter as F
    F.set_clock(SEED)
    port = oracle.Port()
    try:
        ctx = F.Context(0)
        rng = np.random.default_rng(count + nb)
        base = 1 << 18 if dt == np.float32 else 1 << 17
        buf, sl = _slices(rng, count, base, dt)
        buf_t = torch.from_numpy(buf).to(DEV)
        snd, msgs = _encode(F, ctx, buf_t, sl, nb, _presets)
        rcv = [F.RemoteNode(ctx) for _ in msgs]
        dec = [m.clone() for m in msgs]
        F.RemoteNode.decode_many(rcv, dec)
        ctx.sync()
        for i, (at, n) in enumerate(sl):
            x = buf[at:at + n]
            p = _presets(i)
            mn, mx = (None, None) if p is None else p
            st, codes, pmn, pmx = port.ff_encode(x, nb, SEED, mn, mx)
            assert st == 0
            (hm, gmn, hx, gmx), = msgs[i].fixed_points(0)
            assert hm and hx and (gmn, gmx) == (pmn, pmx), i
            assert snd[i].value(msgs[i], 0).cpu().numpy().tobytes() == codes.tobytes(), i
            st, d = port.ff_decode(codes, nb, pmn, pmx, dt)
            assert rcv[i].value(dec[i], 0).cpu().numpy().tobytes() == d.tobytes(), i
    finally:
        F.set_clock(None)


def test_c4_shaped_batch_stored_layout():
    """[FIXING_FLOAT nb=1, COMPRESSING]: the batched encode writes the codes in
    the stored-stream layout the compressor leaves in place; the compressed
    arrays equal snappy 1.1.8 (restated) of the port's codes."""
    import oracle
    from parameter_server_amd import filter as F
    F.set_clock(SEED)
    port = oracle.Port()
    try:
        ctx = F.Context(0)
        rng = np.random.default_rng(7)
        buf, sl = _slices(rng, 100, 1 << 16)
        buf_t = torch.from_numpy(buf).to(DEV)
        snd, msgs = _encode(F, ctx, buf_t, sl, 1, lambda i: None, compress=True)
        ctx.sync()
        for i, (at, n) in enumerate(sl):
            st, codes, pmn, pmx = port.ff_encode(buf[at:at + n], 1, SEED)
            got = snd[i].value(msgs[i], 0).cpu().numpy().tobytes()
            assert got == port.snappy_compress(codes.tobytes()), i
    finally:
        F.set_clock(None)
