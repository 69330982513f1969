"""GPU parity: libpsf's HIP kernels (through the C ABI) against the golden
fixtures generated from the reference and against the C restatement
(oracle/psf_port.c) on large seeded inputs.  Integer/byte outputs (codes,
CRCs, side-info bits) must be bit-exact; decoded floats must be bit-exact too
(the reference's double arithmetic is reproduced without FMA contraction)."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _dt(tag):
    return np.float32 if tag == "f32" else np.float64


def _bits(x):
    return int(np.float32(x).view(np.uint32))


def test_ff_golden_cases_kernel_api(ctx, ff_golden):
    from parameter_server_amd import PsfError
    meta, arrs = ff_golden
    for i, m in enumerate(meta):
        x = torch.from_numpy(arrs[f"x{i}"]).to(DEV)
        try:
            codes, mn, mx = ctx.ff_encode(x, m["nb"], m["seed"], m["preset_min"], m["preset_max"])
        except PsfError:
            assert m["status"] == "error", m["name"]
            continue
        assert m["status"] == "ok", m["name"]
        assert np.array_equal(codes.cpu().numpy(), arrs[f"codes{i}"]), m["name"]
        assert _bits(mn) == m["min_bits"] and _bits(mx) == m["max_bits"], m["name"]
        dec = ctx.ff_decode(codes, m["nb"], mn, mx, dtype=x.dtype)
        assert dec.cpu().numpy().tobytes() == arrs[f"dec{i}"].tobytes(), m["name"]


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("nb", [1, 2, 3, 4, 6])
def test_ff_random_vs_port(ctx, port, dtype, nb):
    n = (1 << 20) + 3  # ragged tail
    x = np.random.default_rng(nb).standard_normal(n).astype(dtype) * 4
    xt = torch.from_numpy(x).to(DEV)
    for seed in (12345, -99):
        codes, mn, mx = ctx.ff_encode(xt, nb, seed)
        st, pc, pmn, pmx = port.ff_encode(x, nb, seed)
        assert st == 0
        assert _bits(mn) == _bits(pmn) and _bits(mx) == _bits(pmx)
        assert np.array_equal(codes.cpu().numpy(), pc)
        dec = ctx.ff_decode(codes, nb, mn, mx, dtype=xt.dtype)
        st, pd = port.ff_decode(pc, nb, pmn, pmx, dtype)
        assert dec.cpu().numpy().tobytes() == pd.tobytes()


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("nb", [1, 2, 3])
def test_ff_quantisation_boundaries(ctx, port, dtype, nb):
    """Values on and next to the quantisation grid, where floor() of the
    reference's tmp flips: exercises the exact-division fallback of the HIP
    quantiser, with preset and with computed min/max."""
    rng = np.random.default_rng(100 + nb)
    ratio = float(2 ** (8 * nb) - 2)
    for mn, mx in ((-1.0, 1.0), (0.1, 0.7), (-3.5, 12.25)):
        k = rng.integers(0, int(ratio) + 1, 20000)
        g = (np.float64(mn) + k * ((np.float64(mx) - np.float64(mn)) / ratio)).astype(dtype)
        x = np.concatenate([g, np.nextafter(g, dtype(np.inf)), np.nextafter(g, dtype(-np.inf)),
                            np.array([mn, mx, mn - 1, mx + 1], dtype)]).astype(dtype)
        xt = torch.from_numpy(x).to(DEV)
        for preset in (True, False):
            a, b = (mn, mx) if preset else (None, None)
            codes, cmn, cmx = ctx.ff_encode(xt, nb, 4321, a, b)
            st, pc, pmn, pmx = port.ff_encode(x, nb, 4321, a, b)
            assert st == 0
            assert np.array_equal(codes.cpu().numpy(), pc), (mn, mx, preset)


def test_ff_unaligned_and_preset(ctx, port):
    n = 100003
    x = np.random.default_rng(3).standard_normal(n + 1).astype(np.float32)
    xt = torch.from_numpy(x).to(DEV)[1:]  # 4-byte offset: scalar path
    for nb in (1, 2, 3):
        codes, mn, mx = ctx.ff_encode(xt, nb, 777, -1.5, 1.5)
        st, pc, _, _ = port.ff_encode(x[1:], nb, 777, -1.5, 1.5)
        assert np.array_equal(codes.cpu().numpy(), pc)
        # unaligned code buffer on decode
        buf = torch.zeros(codes.numel() + 1, dtype=torch.uint8, device=DEV)
        buf[1:] = codes
        dec = ctx.ff_decode(buf[1:], nb, mn, mx)
        st, pd = port.ff_decode(pc, nb, -1.5, 1.5, np.float32)
        assert dec.cpu().numpy().tobytes() == pd.tobytes()


def test_ff_async_device_range(ctx, port):
    n = 1 << 18
    x = torch.randn(n, device=DEV)
    codes = torch.empty(n, dtype=torch.uint8, device=DEV)
    rng = torch.empty(2, dtype=torch.float32, device=DEV)
    status = torch.full((1,), 7, dtype=torch.int32, device=DEV)
    ctx.ff_encode_async(x, 1, 42, codes, rng, status)
    out = torch.empty(n, device=DEV)
    ctx.ff_decode_async(codes, 1, rng, out)
    ctx.sync()
    assert int(status.item()) == 0
    st, pc, mn, mx = port.ff_encode(x.cpu().numpy(), 1, 42)
    assert np.array_equal(codes.cpu().numpy(), pc)
    assert rng.cpu().numpy().tobytes() == np.array([mn, mx], np.float32).tobytes()
    st, pd = port.ff_decode(pc, 1, mn, mx, np.float32)
    assert out.cpu().numpy().tobytes() == pd.tobytes()


def test_ff_full_size_properties(ctx):
    """BASELINE size (2^28 f32, 1 GiB): round-trip error bound and code
    statistics (the CPU oracle is too slow to compare every byte here; the
    2^20-element comparisons above cover the same kernels)."""
    n = 1 << 28
    x = torch.randn(n, device=DEV)
    codes, mn, mx = ctx.ff_encode(x, 1, 12345)
    assert mn == float(x.min().item())
    assert np.float32(mx) == np.float32(np.float64(x.max().item()) + 1e-6)
    dec = ctx.ff_decode(codes, 1, mn, mx)
    step = (np.float64(mx) - np.float64(mn)) / 254.0
    err = (dec.double() - x.double()).abs().max().item()
    assert err <= step * (1 + 1e-6) + 1e-6  # fixing_float.h: |out - x| <= bin/ratio (+ f32 rounding)
    # code range: floor(tmp) + bit <= ratio + 1 = 255, and the extremes are hit
    # (x == min -> 0 + bit; x == max - 1e-6 -> 253 or 254 + bit)
    c = codes.long()
    hist = torch.bincount(c, minlength=256)
    assert hist.numel() == 256
    assert int(c.min()) <= 1 and int(c.max()) >= 253
    # the stochastic-rounding bit: code - floor(tmp) is the LCG bit of element
    # i, the inverted bit 16 of the MSVC LCG state s_{i+1}; over a full period
    # of the low 17 bits it is exactly balanced, so over 2^28 elements (2^11
    # periods) it is balanced to the element
    # tmp as fixing_float.h:80 forms it, (proj - min_v) / bin * ratio with an
    # IEEE division: the divisor is a device tensor, because torch divides by a
    # host scalar as a multiply by its reciprocal, which moves floor(tmp) by one
    # for values within an ulp of a code boundary
    mn64, mx64 = np.float64(mn), np.float64(mx)
    bin_d = torch.tensor(mx64 - mn64, dtype=torch.float64, device=DEV)
    tmp = torch.floor((x.double().clamp(mn64, mx64) - mn64) / bin_d * 254.0).long()
    bit = c - tmp
    if int(bit.min()) < 0 or int(bit.max()) > 1:  # diagnostics for a failure
        bad = ((bit < 0) | (bit > 1)).nonzero().flatten()[:8]
        recip = torch.floor((x.double().clamp(mn64, mx64) - mn64) / (mx64 - mn64) * 254.0).long()
        print("bad", bad.tolist(), "x", x[bad].tolist(), "code", c[bad].tolist(), "floor", tmp[bad].tolist(),
              "floor via reciprocal", recip[bad].tolist(), "min/max", mn, mx)
    assert int(bit.min()) >= 0 and int(bit.max()) <= 1
    assert int(bit.sum()) == n // 2
    del x, dec, c, tmp, bit


@pytest.mark.parametrize("log2n", [27, 28])
def test_roundtrip_driver_c2_vs_port(ctx, port, log2n):
    """The timed driver (psf_node_roundtrip, what bench.py runs) on the bench
    template at BASELINE configs[1]'s size (2^27 f32) and at the bench default
    (2^28 f32, 1 GiB: the decode's 32768-workgroup grid), chain [FIXING_FLOAT
    nb=1], min/max computed: the encoded message as it went on the wire (codes
    + side-info) and the decoded message, byte for byte against the C
    restatement."""
    from parameter_server_amd import FIXING_FLOAT
    from parameter_server_amd import filter as F
    n = 1 << log2n
    g = torch.Generator(device=DEV)
    g.manual_seed(1)
    xs = [torch.randn(n, device=DEV, generator=g) for _ in range(2)]
    tm = []
    for x in xs:
        m = F.Message(request=True, push=True, key_channel=0)
        m.add_value(x)
        m.add_filter(FIXING_FLOAT, num_bytes=1)
        tm.append(m)
    worker, server = F.RemoteNode(ctx), F.RemoteNode(ctx)
    F.set_clock(12345)
    try:
        enc, dec = worker.roundtrip(server, tm, 5, keep_last=True)  # last = tm[0]
    finally:
        F.set_clock(None)
    (has_mn, mn, has_mx, mx), = enc.fixed_points(0)
    st, pc, pmn, pmx = port.ff_encode(xs[0].cpu().numpy(), 1, 12345)
    assert st == 0 and has_mn and has_mx
    assert _bits(mn) == _bits(pmn) and _bits(mx) == _bits(pmx)
    assert np.array_equal(worker.value(enc, 0).cpu().numpy(), pc)
    st, pd = port.ff_decode(pc, 1, pmn, pmx, np.float32)
    assert server.value(dec, 0).cpu().numpy().tobytes() == pd.tobytes()
    assert dec.fixed_points(0) == enc.fixed_points(0)


@pytest.mark.parametrize("nb", [2, 3])
def test_ff_single_array_2_28_vs_port(ctx, port, nb):
    """The single-array encode and decode at the bench size (2^28 f32: the
    16384-workgroup encode and 32768-workgroup decode grids) with nb = 2 and 3,
    codes, side-info and decoded values byte for byte against the C
    restatement (fixing_float.h:73-101)."""
    n = 1 << 28
    g = torch.Generator(device=DEV)
    g.manual_seed(nb)
    x = torch.randn(n, device=DEV, generator=g)
    codes, mn, mx = ctx.ff_encode(x, nb, 2024)
    xh = x.cpu().numpy()
    st, pc, pmn, pmx = port.ff_encode(xh, nb, 2024)
    assert st == 0
    assert _bits(mn) == _bits(pmn) and _bits(mx) == _bits(pmx)
    assert np.array_equal(codes.cpu().numpy(), pc)
    del xh
    dec = ctx.ff_decode(codes, nb, mn, mx)
    st, pd = port.ff_decode(pc, nb, pmn, pmx, np.float32)
    assert st == 0
    assert dec.cpu().numpy().tobytes() == pd.tobytes()
    del x, codes, dec


def test_crc32c_vectors(ctx):
    d = np.load(os.path.join(GOLDEN, "crc32c.npz"))
    offs, crc = d["offsets"], d["crc"]
    data = torch.from_numpy(d["data"]).to(DEV)
    for j in range(len(crc)):
        seg = data[offs[j]:offs[j + 1]]
        got = ctx.crc32c(seg) if seg.numel() else ctx.crc32c(data, 0)
        assert got == int(crc[j]), j
    big = torch.randint(0, 256, (80_000_017,), dtype=torch.uint8, device=DEV)
    import oracle
    assert ctx.crc32c(big) == oracle.Port().crc32c(big.cpu().numpy())


def test_key_signature_prefix(ctx, port):
    keys = torch.arange(10_000_000, dtype=torch.int64, device=DEV) * 97
    assert ctx.key_signature(keys) == port.key_signature(keys[:256].cpu().numpy())


@pytest.mark.parametrize("which", ["key_caching", "chain_ctr", "ff_message", "compressing"])
def test_scenarios_match_restatement(scenario_golden, which):
    """The message path (RemoteNode + filters, HBM buffers) reproduces the
    committed scenario records of oracle/chain.py (parity unpinned by the
    reference: DESIGN.md §3)."""
    import scenarios
    steps = {"key_caching": scenarios.kc_scenario, "chain_ctr": scenarios.chain_scenario,
             "ff_message": scenarios.ff_message_scenario,
             "compressing": scenarios.compress_scenario}[which]()
    got = scenarios.run(scenarios.PsfImpl(device=0), steps)
    want = scenario_golden[which]
    for g, w in zip(got, want):
        assert g == w, (g["name"], g, w)
    assert len(got) == len(want)


def test_c3_10m_keys_miss_then_hit_vs_port(ctx, port):
    """BASELINE configs[2] (C3) at its stated size: 10M sorted unique uint64
    keys sampled from [0, 1e9) (1 % density) + 10M f32, chain [KEY_CACHING,
    FIXING_FLOAT nb=1].  The first send misses (keys travel, the receiver
    checks the CRC and caches them), the repeat hits (keys elided on the wire,
    restored by the receiver); signatures, codes, side-info and all 10M
    decoded values byte for byte against the restatement
    (key_caching.h:9-60, fixing_float.h:50-101)."""
    from parameter_server_amd import FIXING_FLOAT, KEY_CACHING
    from parameter_server_amd import filter as F
    rng = np.random.default_rng(3)
    keys = np.sort(rng.choice(10**9, 10_000_000, replace=False)).astype(np.uint64)
    kd = torch.from_numpy(keys.view(np.int64)).to(DEV)
    worker, server = F.RemoteNode(ctx), F.RemoteNode(ctx)
    sig_want = port.key_signature(keys)
    F.set_clock(777)
    try:
        for send in range(2):
            x = rng.standard_normal(keys.size).astype(np.float32)
            m = F.Message(request=True, push=True, key_channel=3, key_range=(0, 10**9))
            m.set_key(kd)
            m.add_value(torch.from_numpy(x).to(DEV))
            m.add_filter(KEY_CACHING)
            fi = m.add_filter(FIXING_FLOAT, num_bytes=1)
            worker.encode(m)
            assert m.signature(0) == (True, sig_want), send
            wire_keys = m.key_ptr()[1]
            assert wire_keys == (keys.nbytes if send == 0 else 0), send  # elided on the hit
            st, pc, pmn, pmx = port.ff_encode(x, 1, 777)
            assert st == 0
            (has_mn, mn, has_mx, mx), = m.fixed_points(fi)
            assert _bits(mn) == _bits(pmn) and _bits(mx) == _bits(pmx)
            assert np.array_equal(worker.value(m, 0).cpu().numpy(), pc), send
            w = m.clone()
            server.decode(w)
            got_keys = server.key(w).cpu().numpy().view(np.uint64)
            assert np.array_equal(got_keys, keys), send  # restored from the cache on the hit
            st, pd = port.ff_decode(pc, 1, pmn, pmx, np.float32)
            assert server.value(w, 0).cpu().numpy().tobytes() == pd.tobytes(), send
            del m, w
    finally:
        F.set_clock(None)
