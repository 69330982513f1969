"""GPU: FIXING_FLOAT's decode fused into COMPRESSING's (decode_batch on a chain
[..., FIXING_FLOAT, COMPRESSING]: the uncompress writes dequantised values and
the codes never reach HBM).  The values must be bit-identical to the C
restatement's uncompress + FIXING_FLOAT decode (fixing_float.h:89-101,
compressing.h:20-37) and to the unfused single-message decode, for every way
the uncompress places a fragment: stored fragments where the fast path
assumes them, fragments a few bytes off (after a match), tag-dense fragments
(the window scan and the LDS decoder), the array's ragged end, num_bytes 1
and 2, f32 and f64, and a recorded size that disagrees with the stream's
header (the header decides; the message is decoded again unfused)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
DT_FLOAT, DT_DOUBLE = 9, 10


def _codes(kind, nval, nb, seed):
    rng = np.random.default_rng(seed)
    c = rng.integers(0, 256, nval * nb, dtype=np.uint8)
    if kind == "match":  # one 40-byte match: later fragments sit a few bytes off
        b = 5 * 65536 + 3000
        c[b + 100:b + 140] = c[b:b + 40]
    elif kind == "dense":  # every third fragment constant: tag-dense
        for f in range(0, c.size // 65536 + 1, 3):
            c[f * 65536:(f + 1) * 65536] = 17
    elif kind == "mixed":  # runs of repeats inside every fragment (a few tags each)
        c[::4096] = 0
        for f in range(c.size // 65536 + 1):
            c[f * 65536 + 500:f * 65536 + 900] = 3
    return c


def _message(F, s, nval, nb, vt, rng_mm, hint):
    from parameter_server_amd import COMPRESSING, FIXING_FLOAT, lib
    m = F.Message(request=True, push=True)
    m.add_value(torch.frombuffer(bytearray(s), dtype=torch.uint8).to(DEV), value_type=vt)
    m.add_filter(FIXING_FLOAT, num_bytes=nb, fixed_point=[rng_mm])
    idx = m.add_filter(COMPRESSING)
    assert lib().psf_fc_add_uncompressed(m.h, idx, hint) == 0
    return m


CASES = [  # kind, values, nb, dtype
    ("random", 40 * 65536 + 777, 1, np.float32),
    ("random", 20 * 65536 + 3, 2, np.float32),
    ("random", 9 * 65536 + 5, 1, np.float64),
    ("random", 7 * 32768 + 9, 2, np.float64),
    ("match", 40 * 65536 + 12345, 1, np.float32),
    ("match", 20 * 32768 + 11, 2, np.float32),
    ("dense", 12 * 65536 + 100, 1, np.float32),
    ("dense", 6 * 32768 + 1, 2, np.float64),
    ("mixed", 10 * 65536 + 1, 1, np.float32),
    ("random", 1, 1, np.float32),
    ("random", 3, 2, np.float32),
]


def test_fused_decode_matches_port_and_unfused(ctx, port):
    from parameter_server_amd import filter as F
    msgs, single, want = [], [], []
    for k, (kind, nval, nb, dt) in enumerate(CASES):
        codes = _codes(kind, nval, nb, 100 + k)
        s = port.snappy_compress(codes.tobytes())
        mm = (-1.25 - k, 2.5 + 0.5 * k)
        vt = DT_DOUBLE if dt == np.float64 else DT_FLOAT
        msgs.append(_message(F, s, nval, nb, vt, mm, codes.size))
        single.append(_message(F, s, nval, nb, vt, mm, codes.size))
        st, dec = port.ff_decode(codes, nb, mm[0], mm[1], dt)
        assert st == 0
        want.append(dec.tobytes())
    rcv = [F.RemoteNode(ctx) for _ in msgs]
    F.RemoteNode.decode_many(rcv, msgs)  # batched: fused
    for k in range(len(msgs)):
        got = rcv[k].value(msgs[k], 0).cpu().numpy().tobytes()
        assert got == want[k], CASES[k]
        nd = F.RemoteNode(ctx)
        nd.decode(single[k])  # one message at a time: unfused
        assert nd.value(single[k], 0).cpu().numpy().tobytes() == want[k], CASES[k]


def test_fused_decode_header_disagrees_with_record(ctx, port):
    """Two arrays in one message, the second's recorded size wrong: the stream
    header decides (UncompressFrom), both arrays come out as the unfused chain
    gives them."""
    from parameter_server_amd import COMPRESSING, FIXING_FLOAT, lib
    from parameter_server_amd import filter as F
    a = _codes("random", 3 * 65536 + 7, 1, 1)
    b = _codes("match", 8 * 65536 + 1, 1, 2)
    mm = [(-3.0, 3.0), (0.0, 10.0)]
    for wrong in (b.size - 1, b.size + 64, 7):
        m = F.Message(request=True, push=True)
        for c in (a, b):
            s = port.snappy_compress(c.tobytes())
            m.add_value(torch.frombuffer(bytearray(s), dtype=torch.uint8).to(DEV), value_type=DT_FLOAT)
        m.add_filter(FIXING_FLOAT, num_bytes=1, fixed_point=mm)
        idx = m.add_filter(COMPRESSING)
        assert lib().psf_fc_add_uncompressed(m.h, idx, a.size) == 0
        assert lib().psf_fc_add_uncompressed(m.h, idx, wrong) == 0
        nd = F.RemoteNode(ctx)
        F.RemoteNode.decode_many([nd], [m])
        for i, c in enumerate((a, b)):
            st, dec = port.ff_decode(c, 1, mm[i][0], mm[i][1], np.float32)
            assert nd.value(m, i).cpu().numpy().tobytes() == dec.tobytes(), (wrong, i)


def test_fused_decode_device_range_from_encode(ctx, port):
    """Computed min/max left on the device by a batched encode on the same
    context are read by the fused decode (no host wait), as the unfused
    decode reads them; KEY_CACHING between the two decodes."""
    from parameter_server_amd import COMPRESSING, FIXING_FLOAT, KEY_CACHING
    from parameter_server_amd import filter as F
    F.set_clock(4242)
    try:
        rng = np.random.default_rng(9)
        xs = [rng.standard_normal(n).astype(dt) for n, dt in
              ((3 << 20, np.float32), (1 << 20, np.float64), (70_001, np.float32))]
        ms = []
        for i, x in enumerate(xs):
            m = F.Message(request=True, push=True, key_channel=i, key_range=(0, 10**9))
            keys = np.arange(x.size, dtype=np.int64) * 3
            m.set_key(torch.from_numpy(keys).to(DEV))
            m.add_value(torch.from_numpy(x).to(DEV))
            m.add_filter(KEY_CACHING)
            m.add_filter(FIXING_FLOAT, num_bytes=1 + i % 2)
            m.add_filter(COMPRESSING)
            ms.append(m)
        snd = [F.RemoteNode(ctx) for _ in ms]
        rcv = [F.RemoteNode(ctx) for _ in ms]
        F.RemoteNode.encode_many(snd, ms)
        ws = [m.clone() for m in ms]
        F.RemoteNode.decode_many(rcv, ws)
        for i, x in enumerate(xs):
            st, codes, mn, mx = port.ff_encode(x, 1 + i % 2, 4242)
            st, dec = port.ff_decode(codes, 1 + i % 2, mn, mx, x.dtype)
            assert rcv[i].value(ws[i], 0).cpu().numpy().tobytes() == dec.tobytes(), i
            assert rcv[i].key(ws[i]).cpu().numpy().view(np.int64).tobytes() == \
                (np.arange(x.size, dtype=np.int64) * 3).tobytes(), i
    finally:
        F.set_clock(None)


def _tag_positions(s, p):
    out = []
    while p < len(s):
        out.append(p)
        c = s[p]
        if c & 3 == 0:
            ln, h = (c >> 2) + 1, 1
            if ln > 60:
                ln = int.from_bytes(s[p + 1:p + 1 + ln - 60], "little") + 1
                h += (c >> 2) - 59
            p += h + ln
        else:
            p += (2, 3, 5)[(c & 3) - 1]
    return out


@pytest.mark.parametrize("kind", ["random", "match", "dense", "mixed"])
def test_fused_decode_mutated_streams(ctx, port, kind):
    """A compressed code stream with a byte overwritten (a literal's or a
    tag's), deleted or inserted, or its tail cut: the fused decode (batched)
    and the unfused one (single message) both reject what RawUncompress
    rejects (snappy.cc's SnappyDecoder via oracle/snappy_port.c) and
    otherwise agree byte for byte
    — with the restatement's dequantised codes when the stream still holds
    the array's length."""
    from parameter_server_amd import PsfError
    from parameter_server_amd import filter as F
    rng = np.random.default_rng(500 + len(kind))
    nval, mm = 9 * 65536 + 321, (-2.0, 3.0)
    codes = _codes(kind, nval, 1, 7 + len(kind))
    s0 = port.snappy_compress(codes.tobytes())
    hdr = 1
    while s0[hdr - 1] & 0x80:
        hdr += 1
    tags = _tag_positions(s0, hdr)
    nbad = 0
    for t in range(15):
        s = bytearray(s0)
        i, op = int(rng.integers(hdr, len(s))), t % 5
        if op == 4:  # a tag byte (length, kind or offset change)
            i, op = int(tags[int(rng.integers(0, len(tags)))]), 0
        if op == 0:
            s[i] = (s[i] + int(rng.integers(1, 256))) & 255
        elif op == 1:
            del s[i]
        elif op == 2:
            s.insert(i, int(rng.integers(0, 256)))
        else:
            del s[i:]
        s = bytes(s)
        st, out = port.snappy_uncompress(s, cap=1 << 24)
        res = []
        for fused in (True, False):
            m = _message(F, s, nval, 1, DT_FLOAT, mm, codes.size)
            nd = F.RemoteNode(ctx)
            try:
                if fused:
                    F.RemoteNode.decode_many([nd], [m])
                else:
                    nd.decode(m)
                res.append(nd.value(m, 0).cpu().numpy().tobytes())
            except PsfError:
                res.append(None)
        if st != 0:
            assert res == [None, None], (kind, t, op)
            nbad += 1
            continue
        assert res[0] == res[1], (kind, t, op)
        if len(out) == codes.size:
            st2, dec = port.ff_decode(np.frombuffer(out, np.uint8), 1, mm[0], mm[1], np.float32)
            assert st2 == 0 and res[0] == dec.tobytes(), (kind, t, op)
    assert nbad > 0
