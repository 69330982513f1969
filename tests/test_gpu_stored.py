"""GPU: FIXING_FLOAT codes written straight into the stored snappy stream
layout when COMPRESSING follows (chain [..., FIXING_FLOAT, (KEY_CACHING,)
COMPRESSING]).  The compressor leaves a stream whose fragments all come out
stored where FIXING_FLOAT wrote it (header and tags included) and places the
others as usual, so every encoded stream must be byte-identical to the snappy
1.1.8 restatement of the restatement's codes (fixing_float.h:73-88, then
compressing.h:16-19 -> shared_array_inl.h:232-245), whatever the sizes: a
stream ending on a fragment / tile / group boundary or just past one, the
last fragment's tag of 1, 2 or 3 bytes, tiny arrays, num_bytes 1 and 2, f32
and f64, one message or a batch, and streams with a compressible fragment
(the fallback placement) or compressible throughout.  Decoding gives the
restatement's values."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

SEED = 424242
F64 = np.float64


def _values(kind, n, dt, seed, nb):
    x = np.random.default_rng(seed).standard_normal(n).astype(dt)
    per = 65536 // nb  # values per fragment
    if kind == "onecomp" and n > 3 * per:  # fragment 2 constant: codes with matches
        x[2 * per:3 * per] = 0.25
    elif kind == "lastcomp":  # the last fragment constant
        x[(n - 1) // per * per:] = -0.5
    elif kind == "allcomp":
        x[:] = 1.0
        x[::7] = -1.0  # (a range: bin > 0)
    return x


CASES = [  # kind, n values, nb, dtype
    ("random", 16 * 65536, 1, np.float32),
    ("random", 16 * 65536 + 1, 1, np.float32),
    ("random", 16 * 65536 + 3, 1, np.float32),
    ("random", 16 * 65536 + 4, 1, np.float32),
    ("random", 5 * 65536 + 60, 1, np.float32),
    ("random", 5 * 65536 + 61, 1, np.float32),
    ("random", 5 * 65536 + 256, 1, np.float32),
    ("random", 5 * 65536 + 257, 1, np.float32),
    ("random", 3 * 65536 + 4095, 1, np.float32),
    ("random", 3 * 65536 + 4096, 1, np.float32),
    ("random", 3 * 65536 + 4100, 1, np.float32),
    ("random", 65536, 1, np.float32),
    ("random", 65537, 1, np.float32),
    ("random", 4096, 1, np.float32),
    ("random", 1000, 1, np.float32),
    ("random", 15, 1, np.float32),
    ("random", 14, 1, np.float32),
    ("random", 1, 1, np.float32),
    ("random", 8 * 32768, 2, np.float32),
    ("random", 8 * 32768 + 1, 2, np.float32),
    ("random", 8 * 32768 + 30, 2, np.float32),
    ("random", 8 * 32768 + 31, 2, np.float32),
    ("random", 3 * 32768 + 2049, 2, np.float32),
    ("random", 7, 2, np.float32),
    ("random", 4 * 65536 + 5, 1, F64),
    ("random", 4 * 32768 + 2048, 2, F64),
    ("onecomp", 12 * 65536 + 333, 1, np.float32),
    ("onecomp", 9 * 32768 + 7, 2, np.float32),
    ("lastcomp", 6 * 65536 + 5000, 1, np.float32),
    ("allcomp", 4 * 65536 + 17, 1, np.float32),
]


def _msg(F, x, nb, kc_between=False):
    from parameter_server_amd import COMPRESSING, FIXING_FLOAT, KEY_CACHING
    m = F.Message(request=True, push=True, key_channel=3, key_range=(0, 1 << 40))
    if kc_between:
        m.set_key(torch.arange(1000, device="cuda:0", dtype=torch.int64) * 3)
    m.add_value(torch.from_numpy(x).cuda())
    m.add_filter(FIXING_FLOAT, num_bytes=nb)
    if kc_between:
        m.add_filter(KEY_CACHING)
    m.add_filter(COMPRESSING)
    return m


def _want(port, x, nb):
    st, codes, mn, mx = port.ff_encode(x, nb, SEED)
    assert st == 0
    st, dec = port.ff_decode(codes, nb, mn, mx, x.dtype)
    return port.snappy_compress(codes.tobytes()), dec.tobytes()


@pytest.mark.parametrize("batched", [False, True])
def test_stored_layout_streams_vs_port(ctx, port, batched):
    from parameter_server_amd import filter as F
    F.set_clock(SEED)
    try:
        xs = [_values(kind, n, dt, 50 + k, nb) for k, (kind, n, nb, dt) in enumerate(CASES)]
        msgs = [_msg(F, x, c[2], kc_between=(k % 5 == 1)) for k, (x, c) in enumerate(zip(xs, CASES))]
        snd = [F.RemoteNode(ctx) for _ in msgs]
        if batched:
            F.RemoteNode.encode_many(snd, msgs)
        else:
            for nd, m in zip(snd, msgs):
                nd.encode(m)
        ctx.sync()
        for k, (x, c, m) in enumerate(zip(xs, CASES, msgs)):
            stream, dec = _want(port, x, c[2])
            vp, vn, vl = m.value_ptr(0)
            got = F.copy_out(vp, vn, vl, "cuda:0").cpu().numpy().tobytes()
            assert got == stream, (c, len(got), len(stream))
            w = m.clone()
            rcv = F.RemoteNode(ctx)
            rcv.decode(w)
            assert rcv.value(w, 0).cpu().numpy().tobytes() == dec, c
    finally:
        F.set_clock(None)
