"""GPU: many messages through psf_nodes_encode / psf_nodes_decode (FIXING_FLOAT
batched across messages) give exactly what one-at-a-time RemoteNode calls and
the C restatement give: codes, side-info and decoded values bit-exact, for
mixed sizes (tiny, ragged, partial tiles), num_bytes 1-3, f32 / f64, preset
and computed ranges, chains with KEY_CACHING and COMPRESSING, deferred
dequantise."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _cases():
    rng = np.random.default_rng(42)
    sizes = [1, 3, 4, 5, 1023, 4096, 4099, 100_003, 262_144, 70_001]
    out = []
    for k in range(48):
        n = sizes[k % len(sizes)] + (k // len(sizes))
        dt = np.float64 if k % 7 == 3 else np.float32
        nb = 1 + k % 3
        preset = [None, (-1.5, 1.5), (None, 2.0)][k % 3 if k % 5 else 0]
        x = (rng.standard_normal(n) * (1 + k)).astype(dt)
        keys = np.unique(rng.integers(0, 10**9, n + 16).astype(np.uint64))[:n] if k % 4 else None
        out.append((x, nb, preset, keys))
    return out


def _message(F, x, nb, preset, keys, ch, compress=False):
    from parameter_server_amd import COMPRESSING, FIXING_FLOAT, KEY_CACHING
    m = F.Message(request=True, push=True, key_channel=ch, key_range=(0, 10**9))
    if keys is not None:
        m.set_key(torch.from_numpy(keys.view(np.int64)).to(DEV))
        m.add_filter(KEY_CACHING)
    m.add_value(torch.from_numpy(x).to(DEV))
    fp = None if preset is None else [preset]
    m.add_filter(FIXING_FLOAT, num_bytes=nb, fixed_point=fp)
    if compress:
        m.add_filter(COMPRESSING)
    return m


@pytest.mark.parametrize("compress", [False, True])
def test_batch_matches_single_and_port(ctx, port, compress):
    from parameter_server_amd import filter as F
    F.set_clock(987654)
    try:
        cases = _cases()
        snd_b = [F.RemoteNode(ctx) for _ in cases]
        rcv_b = [F.RemoteNode(ctx) for _ in cases]
        snd_s = [F.RemoteNode(ctx) for _ in cases]
        rcv_s = [F.RemoteNode(ctx) for _ in cases]
        mb = [_message(F, *c, ch=i, compress=compress) for i, c in enumerate(cases)]
        ms = [_message(F, *c, ch=i, compress=compress) for i, c in enumerate(cases)]
        F.RemoteNode.encode_many(snd_b, mb)
        for nd, m in zip(snd_s, ms):
            nd.encode(m)
        wb = [m.clone() for m in mb]
        ws = [m.clone() for m in ms]
        F.RemoteNode.decode_many(rcv_b, wb)
        for nd, m in zip(rcv_s, ws):
            nd.decode(m)
        ctx.sync()
        for i, (x, nb, preset, keys) in enumerate(cases):
            fi = 1 if keys is not None else 0
            assert mb[i].fixed_points(fi) == ms[i].fixed_points(fi), i
            vb, vs = snd_b[i].value(mb[i], 0), snd_s[i].value(ms[i], 0)
            assert vb.cpu().numpy().tobytes() == vs.cpu().numpy().tobytes(), i
            db, ds = rcv_b[i].value(wb[i], 0), rcv_s[i].value(ws[i], 0)
            assert db.cpu().numpy().tobytes() == ds.cpu().numpy().tobytes(), i
            # and the C restatement of the reference
            mn = None if preset is None else preset[0]
            mx = None if preset is None else preset[1]
            st, codes, pmn, pmx = port.ff_encode(x, nb, 987654, mn, mx)
            assert st == 0
            st, dec = port.ff_decode(codes, nb, pmn, pmx, x.dtype)
            assert db.cpu().numpy().tobytes() == dec.tobytes(), i
            if not compress:
                assert vb.cpu().numpy().tobytes() == codes.tobytes(), i
            if keys is not None:
                assert rcv_b[i].key(wb[i]).cpu().numpy().view(np.uint64).tobytes() == keys.tobytes(), i
    finally:
        F.set_clock(None)


@pytest.mark.parametrize("compress", [False, True])
def test_batch_guard_band_values(ctx, port, compress):
    """Batched f32 num_bytes=1 encodes (the fused small-batch launch and the
    stored-stream one) of values on and next to the quantisation grid, where
    every lane's band test fails and the rolled exact pass decides each code,
    in arrays whose last tile is partial: codes and decoded values against the
    C restatement."""
    from parameter_server_amd import filter as F
    F.set_clock(2024)
    try:
        rng = np.random.default_rng(77)
        cases = []
        for n, preset in ((4099, (-1.0, 1.0)), (70_001, None), (262_147, (-3.5, 12.25)), (5, None)):
            mn, mx = preset if preset else (-2.0, 3.0)
            k = rng.integers(0, 255, n)
            g = (np.float64(mn) + k * ((np.float64(mx) - np.float64(mn)) / 254.0)).astype(np.float32)
            side = rng.integers(0, 3, n)
            x = np.where(side == 0, g, np.where(side == 1, np.nextafter(g, np.float32(np.inf)),
                                                np.nextafter(g, np.float32(-np.inf)))).astype(np.float32)
            cases.append((x, 1, preset, None))
        snd = [F.RemoteNode(ctx) for _ in cases]
        rcv = [F.RemoteNode(ctx) for _ in cases]
        ms = [_message(F, *c, ch=i, compress=compress) for i, c in enumerate(cases)]
        F.RemoteNode.encode_many(snd, ms)
        ws = [m.clone() for m in ms]
        F.RemoteNode.decode_many(rcv, ws)
        ctx.sync()
        for i, (x, nb, preset, _) in enumerate(cases):
            mn = None if preset is None else preset[0]
            mx = None if preset is None else preset[1]
            st, codes, pmn, pmx = port.ff_encode(x, nb, 2024, mn, mx)
            assert st == 0
            if not compress:
                assert snd[i].value(ms[i], 0).cpu().numpy().tobytes() == codes.tobytes(), i
            st, dec = port.ff_decode(codes, nb, pmn, pmx, np.float32)
            assert rcv[i].value(ws[i], 0).cpu().numpy().tobytes() == dec.tobytes(), i
    finally:
        F.set_clock(None)


def test_batch_deferred_decode(ctx, port):
    from parameter_server_amd import filter as F
    F.set_clock(55)
    try:
        cases = _cases()[:20]
        snd = [F.RemoteNode(ctx) for _ in cases]
        rcv = [F.RemoteNode(ctx) for _ in cases]
        for r in rcv:
            r.set_defer_dequant(True)
        ms = [_message(F, *c, ch=i) for i, c in enumerate(cases)]
        F.RemoteNode.encode_many(snd, ms)
        ws = [m.clone() for m in ms]
        F.RemoteNode.decode_many(rcv, ws)
        for i, (x, nb, preset, keys) in enumerate(cases):
            pend = ws[i].pending(0)
            assert (pend is not None) == (x.dtype == np.float32), i
            ws[i].materialize(ctx)
            mn = None if preset is None else preset[0]
            mx = None if preset is None else preset[1]
            st, codes, pmn, pmx = port.ff_encode(x, nb, 55, mn, mx)
            st, dec = port.ff_decode(codes, nb, pmn, pmx, x.dtype)
            assert rcv[i].value(ws[i], 0).cpu().numpy().tobytes() == dec.tobytes(), i
    finally:
        F.set_clock(None)


def test_batch_roundtrip_driver(ctx):
    from parameter_server_amd import FIXING_FLOAT
    from parameter_server_amd import filter as F
    tm = []
    for i in range(40):
        m = F.Message(request=True, push=True, key_channel=i)
        m.add_value(torch.randn(100_000 + i, device=DEV))
        m.add_filter(FIXING_FLOAT, num_bytes=1)
        tm.append(m)
    snd = [F.RemoteNode(ctx) for _ in tm]
    rcv = [F.RemoteNode(ctx) for _ in tm]
    F.RemoteNode.roundtrip_many(snd, rcv, tm, 3)
    ctx.sync()


@pytest.mark.parametrize("wire", [False, True])
def test_batch_roundtrip_driver_c1_vs_port(ctx, port, wire):
    """The timed C1 driver (psf_nodes_roundtrip_opts in three phases, what
    `bench.py --config c1` runs): 64 ctr minibatch streams of 10^5 sorted keys,
    per step a pull request (keys), pull response (weights) and push
    (gradients) with the ctr filters (online_l1lr.conf:36-53), three steps.
    The last step's encoded messages (KEY_CACHING signature and elision,
    codes, side-info) and decoded messages (keys restored, values) of every
    stream against the C restatement.  wire: each encoded Task is serialised
    (side-info settled) and the receiver decodes a message parsed from it, as
    Van::Send / Recv do (van.cc:122-191, 244-269)."""
    from parameter_server_amd import FIXING_FLOAT, KEY_CACHING
    from parameter_server_amd import filter as F
    m, S, seed = 100_000, 64, 31337
    g = torch.Generator(device=DEV)
    g.manual_seed(7)
    wk = [F.RemoteNode(ctx) for _ in range(S)]
    sv = [F.RemoteNode(ctx) for _ in range(S)]
    req, resp, push, data = [], [], [], []
    for sid in range(S):
        keys = torch.sort(torch.unique(torch.randint(0, 10**9, (m + m // 8,), device=DEV, generator=g))[:m])[0]
        vals = []
        for lst, request, is_push, has_v, clear in ((req, True, False, False, None),
                                                    (resp, False, False, True, None),
                                                    (push, True, True, True, True)):
            t = F.Message(request=request, push=is_push, key_channel=sid, key_range=(0, 10**9))
            t.set_key(keys)
            if has_v:
                v = torch.randn(m, device=DEV, generator=g)
                t.add_value(v)
                vals.append(v.cpu().numpy())
            t.add_filter(KEY_CACHING, clear_cache_if_done=clear)
            t.add_filter(FIXING_FLOAT, num_bytes=1)
            lst.append(t)
        data.append((keys.cpu().numpy().view(np.uint64), vals))
    F.set_clock(seed)
    try:
        last = F.RemoteNode.roundtrip_many(wk + sv + wk, sv + wk + sv, req + resp + push, 3, keep_last=True,
                                           phase_end=[S, 2 * S, 3 * S], wire=wire)
    finally:
        F.set_clock(None)
    node = lambda msg: wk[0]  # noqa: E731  (any node of the context copies out)
    for sid, (keys, (w, x)) in enumerate(data):
        sig = port.key_signature(keys)
        (qe, qd), (re_, rd), (pe, pd_) = last[sid], last[S + sid], last[2 * S + sid]
        # pull request: the push of the previous step erased the cache -> miss
        assert qe.signature(0) == (True, sig) and qe.key_info()[0], sid
        assert node(qd).key(qd).cpu().numpy().view(np.uint64).tobytes() == keys.tobytes()
        for enc, dec, v in ((re_, rd, w), (pe, pd_, x)):  # response / push: hit, keys elided
            assert enc.signature(0) == (True, sig) and not enc.key_info()[0], sid
            st, pc, pmn, pmx = port.ff_encode(v, 1, seed)
            (hm, mn, hx, mx), = enc.fixed_points(1)
            assert hm and hx and (mn, mx) == (pmn, pmx), sid
            assert np.array_equal(node(enc).value(enc, 0).cpu().numpy(), pc), sid
            st, pdec = port.ff_decode(pc, 1, pmn, pmx, np.float32)
            assert node(dec).value(dec, 0).cpu().numpy().tobytes() == pdec.tobytes(), sid
            assert node(dec).key(dec).cpu().numpy().view(np.uint64).tobytes() == keys.tobytes(), sid


def test_batch_key_caching_order(ctx, port):
    """Two messages with the same keys and channel on ONE node in one batch:
    the first misses and caches, the second hits and drops its keys -- as
    sequential EncodeMessage calls would; a second batch hits for both; the
    receiver restores the keys."""
    from parameter_server_amd import filter as F
    rng = np.random.default_rng(9)
    keys = np.unique(rng.integers(0, 10**9, 5000).astype(np.uint64))
    snd, rcv = F.RemoteNode(ctx), F.RemoteNode(ctx)
    for rnd in range(2):
        ms = []
        for j in range(3):
            x = rng.standard_normal(keys.size).astype(np.float32)
            ms.append(_message(F, x, 1, None, keys, ch=7))
        F.RemoteNode.encode_many([snd] * 3, ms)
        has = [m.key_info()[0] for m in ms]
        assert has == ([True, False, False] if rnd == 0 else [False, False, False]), (rnd, has)
        ws = [m.clone() for m in ms]
        F.RemoteNode.decode_many([rcv] * 3, ws)
        for w in ws:
            assert rcv.key(w).cpu().numpy().view(np.uint64).tobytes() == keys.tobytes()


def test_batch_many_messages_slot_chunks(ctx, port):
    """300 messages [KEY_CACHING, FIXING_FLOAT] in one batch: more signatures
    than the deferred publish-slot range holds (the signatures are then waited
    for batch by batch) and more FIXING_FLOAT arrays than one slot chunk;
    results equal one-at-a-time encodes and the C restatement, and a second
    batch hits the key cache for every message."""
    from parameter_server_amd import filter as F
    F.set_clock(4242)
    try:
        rng = np.random.default_rng(11)
        cases = []
        for k in range(300):
            n = 50 + 37 * (k % 13)
            keys = np.unique(rng.integers(0, 10**9, n + 8).astype(np.uint64))[:n]
            cases.append((rng.standard_normal(keys.size).astype(np.float32), keys))
        snd_b = [F.RemoteNode(ctx) for _ in cases]
        snd_s = [F.RemoteNode(ctx) for _ in cases]
        for rnd in range(2):
            mb = [_message(F, x, 1, None, keys, ch=i) for i, (x, keys) in enumerate(cases)]
            ms = [_message(F, x, 1, None, keys, ch=i) for i, (x, keys) in enumerate(cases)]
            F.RemoteNode.encode_many(snd_b, mb)
            for nd, m in zip(snd_s, ms):
                nd.encode(m)
            ctx.sync()
            for i, (x, keys) in enumerate(cases):
                assert mb[i].key_info()[0] == ms[i].key_info()[0] == (rnd == 0), (rnd, i)
                assert mb[i].fixed_points(1) == ms[i].fixed_points(1), i
                vb = snd_b[i].value(mb[i], 0).cpu().numpy().tobytes()
                assert vb == snd_s[i].value(ms[i], 0).cpu().numpy().tobytes(), i
                if rnd == 0 and i % 37 == 0:
                    st, codes, _, _ = port.ff_encode(x, 1, 4242)
                    assert vb == codes.tobytes(), i
    finally:
        F.set_clock(None)


def test_batch_lazy_range_bin_check(ctx):
    """A batched encode leaves computed min/max on the device; the
    CHECK_GT(bin, 0) of an array whose max rounds onto its min is reported
    when the range is settled (a host read of the FilterConfig) or at the
    context's sync, not lost."""
    from parameter_server_amd import filter as F
    from parameter_server_amd import FIXING_FLOAT, PsfError
    def msgs():
        out = []
        for v in (1.0e4, None):
            m = F.Message(request=True, push=True, key_channel=0)
            x = torch.full((4096,), v, device=DEV) if v is not None else torch.randn(4096, device=DEV)
            m.add_value(x)
            m.add_filter(FIXING_FLOAT, num_bytes=1)
            out.append(m)
        return out
    ms = msgs()
    F.RemoteNode.encode_many([F.RemoteNode(ctx), F.RemoteNode(ctx)], ms)
    assert ms[1].fixed_points(0)[0][0]  # the good array settles fine
    with pytest.raises(PsfError):
        ms[0].fixed_points(0)
    ctx_err = None
    try:
        ctx.sync()
    except PsfError as e:  # the same batch is also reported once at sync
        ctx_err = e
    assert ctx_err is not None
    ctx.sync()  # reported once


def test_batch_lazy_ring_wraps(ctx, port):
    """More lazily encoded arrays than the host-mapped record ring holds
    (2^15): older batches are resolved before their records are reused, and
    every message's settled range equals the C restatement's."""
    from parameter_server_amd import FIXING_FLOAT
    from parameter_server_amd import filter as F
    rng = np.random.default_rng(5)
    node = F.RemoteNode(ctx)
    kept = []
    total = 0
    while total < (1 << 15) + 4096:
        xs = [rng.standard_normal(8).astype(np.float32) * (1 + i % 7) for i in range(256)]
        ms = []
        for x in xs:
            m = F.Message(request=True, push=True, key_channel=0)
            m.add_value(torch.from_numpy(x).to(DEV))
            m.add_filter(FIXING_FLOAT, num_bytes=1)
            ms.append(m)
        F.RemoteNode.encode_many([node] * len(ms), ms)
        kept.append((xs[::37], ms[::37]))
        total += len(ms)
    for xs, ms in kept:
        for x, m in zip(xs, ms):
            _, mn, _, mx = m.fixed_points(0)[0]
            _, _, pmn, pmx = port.ff_encode(x, 1, 1)
            assert (np.float32(mn), np.float32(mx)) == (np.float32(pmn), np.float32(pmx))
    ctx.sync()


def test_batch_lazy_range_cross_context(ctx, port):
    """Encoded on one context (stream), decoded on another: the decoding
    context cannot read the encode's device record in stream order, so it
    settles the range first (a sync of the encoding context); the decoded
    values equal the C restatement's."""
    from parameter_server_amd import filter as F
    F.set_clock(777)
    try:
        other = F.Context(0)
        cases = _cases()[:12]
        snd = [F.RemoteNode(ctx) for _ in cases]
        rcv = [F.RemoteNode(other) for _ in cases]
        ms = [_message(F, *c, ch=i) for i, c in enumerate(cases)]
        F.RemoteNode.encode_many(snd, ms)
        ws = [m.clone() for m in ms]
        F.RemoteNode.decode_many(rcv, ws)
        other.sync()
        for i, (x, nb, preset, keys) in enumerate(cases):
            mn = None if preset is None else preset[0]
            mx = None if preset is None else preset[1]
            st, codes, pmn, pmx = port.ff_encode(x, nb, 777, mn, mx)
            st, dec = port.ff_decode(codes, nb, pmn, pmx, x.dtype)
            assert rcv[i].value(ws[i], 0).cpu().numpy().tobytes() == dec.tobytes(), i
    finally:
        F.set_clock(None)


@pytest.mark.parametrize("count", [64, 70])
def test_batch_full_job_table(ctx, port, count):
    """A full 64-array job table (and one spilling into a second launch) of one
    (f32, num_bytes=1) group, with fully preset arrays (no min/max pass: empty
    ranges in the min/max workgroup table) between computed and half-preset
    ones and ragged sizes: codes, side-info and decoded values equal the
    one-at-a-time path and the C restatement."""
    from parameter_server_amd import filter as F
    F.set_clock(31337)
    try:
        rng = np.random.default_rng(count)
        cases = []
        for k in range(count):
            n = [1, 5, 4096, 4099, 65_537, 100_003][k % 6] + k
            preset = [None, (-2.0, 2.0), (None, 3.0), (-1.0, None)][k % 4] if k % 5 else (-0.5, 0.5)
            cases.append((rng.standard_normal(n).astype(np.float32) * (1 + k % 9), preset))
        snd_b = [F.RemoteNode(ctx) for _ in cases]
        rcv_b = [F.RemoteNode(ctx) for _ in cases]
        snd_s = [F.RemoteNode(ctx) for _ in cases]
        mb = [_message(F, x, 1, p, None, ch=i) for i, (x, p) in enumerate(cases)]
        ms = [_message(F, x, 1, p, None, ch=i) for i, (x, p) in enumerate(cases)]
        F.RemoteNode.encode_many(snd_b, mb)
        for nd, m in zip(snd_s, ms):
            nd.encode(m)
        wb = [m.clone() for m in mb]
        F.RemoteNode.decode_many(rcv_b, wb)
        ctx.sync()
        for i, (x, p) in enumerate(cases):
            assert mb[i].fixed_points(0) == ms[i].fixed_points(0), i
            vb = snd_b[i].value(mb[i], 0).cpu().numpy().tobytes()
            assert vb == snd_s[i].value(ms[i], 0).cpu().numpy().tobytes(), i
            mn, mx = (None, None) if p is None else p
            st, codes, pmn, pmx = port.ff_encode(x, 1, 31337, mn, mx)
            assert st == 0 and vb == codes.tobytes(), i
            st, dec = port.ff_decode(codes, 1, pmn, pmx, x.dtype)
            assert rcv_b[i].value(wb[i], 0).cpu().numpy().tobytes() == dec.tobytes(), i
    finally:
        F.set_clock(None)


@pytest.mark.parametrize("count", [600])
def test_batch_two_launches_of_large_table(ctx, port, count):
    """More arrays than one job table holds (512): two launches, the first
    with the 512-entry table; codes and decoded values equal the C
    restatement."""
    test_batch_full_job_table(ctx, port, count)


def test_batch_tile_edges_and_offsets(ctx, port):
    """One batch of arrays at tile edges (exactly 256 full tiles of 4096
    values, 256 tiles plus a 1-value tail, 256 tiles plus one group, a
    3-value array) and slices starting 1, 2 and 3 elements past a 16-byte
    boundary (the C4 slices), presets mixed in: codes, side-info and decoded
    values equal the C restatement and the one-at-a-time path."""
    from parameter_server_amd import filter as F
    F.set_clock(2024)
    try:
        rng = np.random.default_rng(3)
        base = torch.from_numpy(rng.standard_normal(300_000).astype(np.float32)).to(DEV)
        arrays = [torch.from_numpy(rng.standard_normal(n).astype(np.float32)).to(DEV)
                  for n in (1 << 20, (1 << 20) + 1, (1 << 20) + 4, 3)]
        arrays += [base[off:off + 100_000 + off] for off in (1, 2, 3)]
        presets = [None, (-1.0, None), None, None, (None, 2.5), None, (-3.0, 3.0)]
        snd_b = [F.RemoteNode(ctx) for _ in arrays]
        rcv_b = [F.RemoteNode(ctx) for _ in arrays]
        snd_s = [F.RemoteNode(ctx) for _ in arrays]

        def msg(i, a):
            from parameter_server_amd import FIXING_FLOAT
            m = F.Message(request=True, push=True, key_channel=i)
            m.add_value(a)
            m.add_filter(FIXING_FLOAT, num_bytes=1, fixed_point=None if presets[i] is None else [presets[i]])
            return m
        mb = [msg(i, a) for i, a in enumerate(arrays)]
        ms = [msg(i, a) for i, a in enumerate(arrays)]
        F.RemoteNode.encode_many(snd_b, mb)
        for nd, m in zip(snd_s, ms):
            nd.encode(m)
        wb = [m.clone() for m in mb]
        F.RemoteNode.decode_many(rcv_b, wb)
        ctx.sync()
        for i, a in enumerate(arrays):
            x = a.cpu().numpy()
            assert mb[i].fixed_points(0) == ms[i].fixed_points(0), i
            vb = snd_b[i].value(mb[i], 0).cpu().numpy().tobytes()
            assert vb == snd_s[i].value(ms[i], 0).cpu().numpy().tobytes(), i
            mn, mx = (None, None) if presets[i] is None else presets[i]
            st, codes, pmn, pmx = port.ff_encode(x, 1, 2024, mn, mx)
            assert st == 0 and vb == codes.tobytes(), i
            st, dec = port.ff_decode(codes, 1, pmn, pmx, x.dtype)
            assert rcv_b[i].value(wb[i], 0).cpu().numpy().tobytes() == dec.tobytes(), i
    finally:
        F.set_clock(None)


def test_small_batch_min_max_and_encode_in_one_launch(ctx, port):
    """A batch of small arrays with computed ranges runs its min/max pass and
    encode in one launch (ff_fused_batch: the min/max items folded by the
    encode workgroups themselves), with a held-back decode of the same
    num_bytes in front when the round-trip driver defers one -- and the codes
    and decoded values are still the restatement's."""
    import os

    from parameter_server_amd import FIXING_FLOAT
    from parameter_server_amd import filter as F
    if os.environ.get("PSF_FF_FUSED") == "0":
        pytest.skip("fused launch disabled (PSF_FF_FUSED=0)")
    F.set_clock(4242)
    try:
        rng = np.random.default_rng(5)
        xs = [(rng.standard_normal(n) * 3).astype(np.float32) for n in (1, 5, 4096, 9999, 100_003, 262_145)]
        msgs = []
        for i, x in enumerate(xs):
            m = F.Message(request=True, push=True, key_channel=i, key_range=(0, 10**9))
            m.add_value(torch.from_numpy(x).to(DEV))
            m.add_filter(FIXING_FLOAT, num_bytes=1)
            msgs.append(m)
        ctx.profile(True)
        ctx.profile_reset()
        F.RemoteNode.encode_many([F.RemoteNode(ctx) for _ in msgs], msgs)
        ctx.sync()
        prof = ctx.profile_read()
        ctx.profile(False)
        assert prof.get("ff_minmax_encode", (0,))[0] == 1, prof
        assert "ff_minmax_partials" not in prof and "ff_encode" not in prof, prof
        for i, (x, m) in enumerate(zip(xs, msgs)):
            st, codes, mn, mx = port.ff_encode(x, 1, 4242)
            assert st == 0
            fp = m.fixed_points(0)
            assert len(fp) == 1 and fp[0][0] and fp[0][2], i
            assert np.float32(fp[0][1]) == np.float32(mn) and np.float32(fp[0][3]) == np.float32(mx), i
            vp, vn, vl = m.value_ptr(0)
            got = F.copy_out(vp, vn, vl, DEV).cpu().numpy().tobytes()
            assert got == codes.tobytes(), i
    finally:
        F.set_clock(None)


def test_fused_batches_back_to_back(ctx, port):
    """Twenty batched encodes in a row on one context, each a random mix of
    small arrays (sizes, num_bytes, f32/f64, computed or half-preset ranges):
    the fused launch's counter lines are zeroed by each launch for the next,
    so every batch's codes and ranges equal the restatement's."""
    from parameter_server_amd import FIXING_FLOAT
    from parameter_server_amd import filter as F
    F.set_clock(777)
    try:
        rng = np.random.default_rng(11)
        for it in range(20):
            nmsg = int(rng.integers(2, 12))
            nb = int(rng.integers(1, 4))
            cases, msgs = [], []
            for i in range(nmsg):
                n = int(rng.integers(1, 60_000))
                dt = np.float64 if rng.random() < 0.3 else np.float32
                x = (rng.standard_normal(n) * (1 + i)).astype(dt)
                preset = (None, float(x.max()) + 1.0) if rng.random() < 0.2 else None
                m = F.Message(request=True, push=True, key_channel=i, key_range=(0, 10**9))
                m.add_value(torch.from_numpy(x).to(DEV))
                m.add_filter(FIXING_FLOAT, num_bytes=nb, fixed_point=None if preset is None else [preset])
                cases.append((x, preset))
                msgs.append(m)
            F.RemoteNode.encode_many([F.RemoteNode(ctx) for _ in msgs], msgs)
            ctx.sync()
            for i, ((x, preset), m) in enumerate(zip(cases, msgs)):
                st, codes, mn, mx = port.ff_encode(x, nb, 777, None, None if preset is None else preset[1])
                assert st == 0
                vp, vn, vl = m.value_ptr(0)
                got = F.copy_out(vp, vn, vl, DEV).cpu().numpy().tobytes()
                assert got == codes.tobytes(), (it, i)
    finally:
        F.set_clock(None)


def test_batch_tag_dense_key_streams(ctx, port):
    """Five messages decoded in one batch, each with 2^17 sorted keys (1 MiB,
    tag-dense once compressed: the window scan, the three-launch linker with
    several 16-window blocks per stream, the index and the fragment decoder,
    all over a multi-stream grid) and one value array: keys and values come
    back exactly, and each compressed key stream is snappy 1.1.8's."""
    from parameter_server_amd import filter as F
    rng = np.random.default_rng(31)
    F.set_clock(4242)
    try:
        cases = []
        for k in range(5):
            n = (1 << 17) + 977 * k
            keys = np.unique(rng.integers(0, 10**9, n + n // 8).astype(np.uint64))[:n]
            x = rng.standard_normal(n).astype(np.float32)
            cases.append((x, 1, None, keys))
        snd = [F.RemoteNode(ctx) for _ in cases]
        rcv = [F.RemoteNode(ctx) for _ in cases]
        ms = [_message(F, *c, ch=i, compress=True) for i, c in enumerate(cases)]
        F.RemoteNode.encode_many(snd, ms)
        ws = [m.clone() for m in ms]
        F.RemoteNode.decode_many(rcv, ws)
        ctx.sync()
        for i, (x, nb, preset, keys) in enumerate(cases):
            kz = snd[i].key(ms[i]).cpu().numpy().tobytes()
            assert kz == port.snappy_compress(keys.tobytes()), i
            assert rcv[i].key(ws[i]).cpu().numpy().view(np.uint64).tobytes() == keys.tobytes(), i
            st, codes, pmn, pmx = port.ff_encode(x, nb, 4242)
            st, dec = port.ff_decode(codes, nb, pmn, pmx, x.dtype)
            assert rcv[i].value(ws[i], 0).cpu().numpy().tobytes() == dec.tobytes(), i
    finally:
        F.set_clock(None)
