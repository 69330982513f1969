"""CPU: the oracle restatements (oracle/psf_port.c, snappy_port.c,
oracle/chain.py) against the committed golden fixtures (tests/golden/,
tests/golden/make_golden.py), and -- where they are available here -- against
the reference's own crc32c.cc and the snappy 1.1.8 library.  The fixtures of
FIXING_FLOAT, NOISE, KEY_CACHING scenarios and EvenDivide are restatement
outputs: parity with the reference is unpinned for them."""
import os

import numpy as np
import pytest

from conftest import GOLDEN


def _dt(tag):
    return np.float32 if tag == "f32" else np.float64


def test_ff_cases_port_matches_reference_fixtures(port, ff_golden):
    meta, arrs = ff_golden
    assert len(meta) >= 60
    for i, m in enumerate(meta):
        x = arrs[f"x{i}"]
        st, codes, mn, mx = port.ff_encode(x, m["nb"], m["seed"], m["preset_min"], m["preset_max"])
        if m["status"] == "error":
            assert st != 0, m["name"]
            continue
        assert st == 0, m["name"]
        assert np.array_equal(codes, arrs[f"codes{i}"]), m["name"]
        assert int(np.float32(mn).view(np.uint32)) == m["min_bits"], m["name"]
        assert int(np.float32(mx).view(np.uint32)) == m["max_bits"], m["name"]
        st, dec = port.ff_decode(codes, m["nb"], mn, mx, _dt(m["dtype"]))
        assert st == 0
        assert dec.tobytes() == arrs[f"dec{i}"].tobytes(), m["name"]


def test_ff_fixtures_cover_reference_defects(ff_golden):
    meta, _ = ff_golden
    names = {m["name"]: m for m in meta}
    # fixing_float.h:71 CHECK_GT(bin, 0) for a constant array with |c| >= 32
    assert names["f32_const_ge32"]["status"] == "error"
    assert names["f32_const_small"]["status"] == "ok"
    # nb = 4..7 are accepted (int-shift ratio), see SURVEY.md §0.5
    assert all(names[f"f32_gauss_nb{nb}"]["status"] == "ok" for nb in range(1, 8))


def test_crc32c_vectors(port):
    d = np.load(os.path.join(GOLDEN, "crc32c.npz"))
    offs, crc = d["offsets"], d["crc"]
    for j in range(len(crc)):
        assert port.crc32c(d["data"][offs[j]:offs[j + 1]]) == int(crc[j])
    assert port.crc32c(b"123456789") == 0xE3069283


def test_noise_port_matches_reference(port):
    d = np.load(os.path.join(GOLDEN, "noise.npz"))
    for tag in ("f32", "f64"):
        for j in range(3):
            mean, sd = d[f"{tag}_{j}_param"]
            out = port.add_noise(d[f"{tag}_{j}_in"], float(mean), float(sd))
            assert out.tobytes() == d[f"{tag}_{j}_out"].tobytes()


def test_noise_port_matches_libstdcxx(port):
    """NOISE's restatement (psf_port.c) against libstdc++ itself: a default
    std::default_random_engine feeding std::normal_distribution<V>(mean, std),
    fresh per array, as add_noise.h:29-39 calls them (oracle/noise_std.cc,
    built with the reference's flags)."""
    import oracle
    S = oracle.NoiseStd()
    rng = np.random.default_rng(0)
    for dt in (np.float32, np.float64):
        for n in (1, 2, 3, 7, 64, 1001, 4099, 1 << 18):
            for mean, sd in ((0.0, 1.0), (0.25, 2.0), (-3.0, 0.01), (1e3, 1e-3)):
                x = rng.standard_normal(n).astype(dt)
                a = port.add_noise(x, np.float32(mean), np.float32(sd))
                b = S.add_noise(x, np.float32(mean), np.float32(sd))
                assert a.tobytes() == b.tobytes(), (dt, n, mean, sd)


def test_lcg_jump_ahead(port):
    # fixing_float.h:18-21; the HIP encoder jumps the LCG per lane
    s = np.uint32(12345)
    for k in range(1, 200):
        s = np.uint32((214013 * int(s) + 2531011) & 0xFFFFFFFF)
        assert port.lcg_state(12345, k) == int(s)
    s = (-7) & 0xFFFFFFFF
    for _ in range(1 << 12):
        s = (214013 * s + 2531011) & 0xFFFFFFFF
    assert port.lcg_state(-7, 1 << 12) == s


def test_ratio_defect(port):
    # fixing_float.h:55 on x86: 1 << (nb*8) with a masked shift count
    assert port.ratio(1) == 254.0
    assert port.ratio(2) == 65534.0
    assert port.ratio(3) == 16777214.0
    assert port.ratio(4) == -1.0
    assert port.ratio(5) == 254.0
    assert port.ratio(7) == 16777214.0


def test_minmax_tie_rule(port):
    # documented divergence: -0.0 orders below +0.0 in the computed min
    x = np.array([0.0, 1.0, -0.0, 0.5], np.float32)
    st, codes, mn, mx = port.ff_encode(x, 1, 1)
    assert st == 0 and np.signbit(mn) and mn == 0.0


def test_fast_floor_guard_is_sound():
    """The HIP encoder skips the f64 division when d*(ratio/bin) is farther
    than 2^-26 from an integer (ff_codec.hip quant_floor).  Check, in IEEE
    double without FMA (numpy), that the guard never lets a floor differ from
    the reference's floor(d / bin * ratio)."""
    rng = np.random.default_rng(0)
    guard = 2.0 ** -26
    for nb in (1, 2, 3):
        ratio = float(2 ** (8 * nb) - 2)
        for trial in range(20):
            lo = np.float32(rng.standard_normal() * 10.0 ** rng.integers(-3, 4))
            hi = np.float32(lo + abs(rng.standard_normal()) * 10.0 ** rng.integers(-6, 4) + 1e-30)
            if not hi > lo:
                continue
            mn, mx = np.float64(lo), np.float64(hi)
            bin_ = mx - mn
            x = rng.uniform(mn, mx, 200_000)
            # adversarial: exact grid points and their float32 neighbours
            k = rng.integers(0, int(ratio) + 1, 50_000)
            g = (mn + k * (bin_ / ratio)).astype(np.float32).astype(np.float64)
            x = np.concatenate([x, g, np.nextafter(g, np.inf), np.nextafter(g, -np.inf)])
            proj = np.clip(x, mn, mx)
            d = proj - mn
            exact = np.floor(d / bin_ * ratio)
            t = d * (ratio / bin_)
            fr = t - np.floor(t)
            fast_ok = (fr > guard) & (fr < 1 - guard)
            assert np.array_equal(np.floor(t)[fast_ok], exact[fast_ok]), (nb, trial)
            assert fast_ok.mean() > 0.5


def test_fast_floor_f32_guard_is_sound():
    """The f32 / num_bytes=1 encoder (ff_codec.hip encode_tile_f32_nb1)
    computes t = (med3(x, min, max) - min) * float(ratio / bin) in float32 and
    takes floor(t) when frac(t) is farther than 2^-14 from an integer (tested
    on the u32 bit pattern of frac); numpy float32 arithmetic (IEEE, no FMA)
    replays it here against the reference's double floor((proj - min) / bin *
    ratio) on random and adversarial (grid point +- 1 ulp) values."""
    rng = np.random.default_rng(1)
    f = np.float32
    guard_bits = np.array([2.0 ** -14], np.float32).view(np.uint32)[0]
    one_minus = np.array([1 - 2.0 ** -14], np.float32).view(np.uint32)[0]
    ratio = 254.0
    checked = 0
    for trial in range(40):
        lo = f(rng.standard_normal() * 10.0 ** rng.integers(-3, 4))
        hi = f(lo + abs(rng.standard_normal()) * 10.0 ** rng.integers(-5, 4) + 1e-30)
        if not hi > lo:
            continue
        mn, mx = np.float64(lo), np.float64(hi)
        bin_ = mx - mn
        x = rng.uniform(mn, mx, 100_000).astype(np.float32)
        k = rng.integers(0, 255, 50_000)
        g = (mn + k * (bin_ / ratio)).astype(np.float32)
        x = np.concatenate([x, g, np.nextafter(g, f(np.inf)), np.nextafter(g, f(-np.inf)),
                            np.array([lo, hi], np.float32)])
        c = np.clip(x, lo, hi).astype(np.float32)
        scale = f(ratio / bin_)
        t = ((c - lo).astype(np.float32) * scale).astype(np.float32)
        fl = np.floor(t)
        fb = (t - fl).astype(np.float32).view(np.uint32)
        fast_ok = (fb > guard_bits) & (fb < one_minus)
        exact = np.floor((np.clip(x.astype(np.float64), mn, mx) - mn) / bin_ * ratio)
        assert np.array_equal(fl[fast_ok].astype(np.float64), exact[fast_ok]), trial
        checked += int(fast_ok.sum())
    assert checked > 1_000_000


def test_noise_logf_matches_libm():
    """The NOISE kernel's logf (csrc/glibc_logf.h) equals this libm's logf
    (the reference's std::log(float)); exhaustive check: run logf_check
    without arguments."""
    import subprocess

    import oracle
    exe = os.path.join(oracle.HERE, "_port", "logf_check")
    if not os.path.exists(exe):
        oracle.build(ref=False)
    out = subprocess.run([exe, "3000000"], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout


def test_noise_log_matches_libm():
    """The NOISE kernel's double log (csrc/glibc_log.h) equals this libm's log
    (the reference's std::log(double)) bit for bit: 4 x 2M random doubles of
    each kind (bit patterns in (0, 1], near 1, polar r2, above 1) and every
    exponent's extreme mantissas (~3.8e8 doubles with argument 1e8: 0 found)."""
    import subprocess

    import oracle
    exe = os.path.join(oracle.HERE, "_port", "log_check")
    if not os.path.exists(exe):
        oracle.build(ref=False)
    out = subprocess.run([exe, "2000000"], capture_output=True, text=True)
    assert out.returncode == 0 and " 0 mismatches" in out.stdout, out.stdout


def test_crc32c_reference_source(port):
    """CRC32C pinned to the reference itself: src/util/crc32c.cc compiled in
    place (oracle/_ref/libcrc32c_ref.so) agrees with the restatement and the
    committed vectors (all lengths 0..4096 of random bytes, every alignment)."""
    import oracle
    if not os.path.exists(oracle.CRC_REF_SO):
        pytest.skip("oracle/_ref/libcrc32c_ref.so not built (needs /root/reference)")
    R = oracle.RefCrc32c()
    assert R.crc32c(b"123456789") == 0xE3069283
    d = np.load(os.path.join(GOLDEN, "crc32c.npz"))
    offs, crc, data = d["offsets"], d["crc"], d["data"]
    for j in range(len(crc)):
        assert R.crc32c(data[offs[j]:offs[j + 1]]) == int(crc[j]), j
    b = np.random.default_rng(4).integers(0, 256, 8192, dtype=np.uint8)
    for n in range(0, 4097, 13):
        for off in (0, 1, 2, 3):
            assert R.crc32c(b[off:off + n]) == port.crc32c(b[off:off + n]), (n, off)
    keys = np.sort(np.random.default_rng(5).integers(0, 2**63, 100000, dtype=np.uint64))
    assert R.key_signature(keys) == port.key_signature(keys)


@pytest.mark.parametrize("which", ["key_caching", "chain_ctr", "ff_message", "compressing"])
def test_chain_restatement_reproduces_scenarios(scenario_golden, which):
    """oracle/chain.py (RemoteNode + the four filters restated over the C port)
    produces every committed scenario record (tests/golden/scenarios.json)."""
    import scenarios
    from oracle.chain import PortImpl
    steps = {"key_caching": scenarios.kc_scenario, "chain_ctr": scenarios.chain_scenario,
             "ff_message": scenarios.ff_message_scenario, "compressing": scenarios.compress_scenario}[which]()
    assert scenarios.run(PortImpl(), steps) == scenario_golden[which]


# ---- COMPRESSING: snappy 1.1.8 restated (oracle/snappy_port.c) -------------
def _snappy_fixtures():
    a = np.load(os.path.join(GOLDEN, "snappy.npz"), allow_pickle=False)
    names = sorted(k[:-3] for k in a.files if k.endswith("_in"))
    return [(k, a[f"{k}_in"].tobytes(), a[f"{k}_out"].tobytes()) for k in names]


def _snappy_dec_fixtures():
    a = np.load(os.path.join(GOLDEN, "snappy_dec.npz"), allow_pickle=False)
    d, off, st, out, ooff = a["data"], a["offsets"], a["status"], a["out"], a["out_offsets"]
    return [(d[off[i]:off[i + 1]].tobytes(), int(st[i]), out[ooff[i]:ooff[i + 1]].tobytes())
            for i in range(len(st))]


def test_snappy_port_compress_matches_1_1_8(port):
    fx = _snappy_fixtures()
    assert len(fx) >= 20
    for name, x, want in fx:
        assert port.snappy_compress(x) == want, name
        st, back = port.snappy_uncompress(want)
        assert st == 0 and back == x, name


def test_snappy_port_decoder_verdicts(port):
    fx = _snappy_dec_fixtures()
    assert sum(1 for _, s, _ in fx if s != 0) > 100
    for s, st, out in fx:
        assert port.snappy_uncompress(s, cap=1 << 20) == (st, out), s[:16]


def test_snappy_port_vs_libsnappy_random(port):
    """snappy_port.c against snappy 1.1.8 itself (the image's libsnappy, the
    third-party library COMPRESSING links) on random inputs of three kinds."""
    import oracle
    try:
        S = oracle.Snappy118()
    except FileNotFoundError:
        pytest.skip("snappy 1.1.8 library not in this image")
    rng = np.random.default_rng(123)
    for t in range(60):
        n = int(rng.integers(0, 200000))
        kind = t % 3
        if kind == 0:
            b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        elif kind == 1:
            b = np.sort(rng.integers(0, 10**9, n // 8 + 1, dtype=np.uint64)).tobytes()[:n]
        else:
            b = np.repeat(rng.integers(0, 8, n // 5 + 1, dtype=np.uint8), 5).tobytes()[:n]
        assert port.snappy_compress(b) == S.compress(b), (t, n)


@pytest.mark.parametrize("nb", [1, 2, 3])
def test_decode_quotient(port, nb):
    """The device decode forms r / ratio as fma(fma(-q0, ratio, r), inv, q0)
    with q0 = r * inv, inv = RN(1/ratio) (ff_codec.hip dequant_q); it must
    equal the IEEE quotient of fixing_float.h:97 for every possible code."""
    assert port.decode_quotient_mismatches(nb) == 0


def test_golden_fixtures_regenerate():
    """Every committed fixture is reproduced, byte for byte, by its generator
    (tests/golden/make_golden.py --check): the restatements, the reference's
    own crc32c.cc and the snappy 1.1.8 library."""
    import oracle
    if not os.path.exists(oracle.CRC_REF_SO):
        pytest.skip("oracle/_ref not built (needs /root/reference)")
    import sys
    sys.path.insert(0, GOLDEN)
    import make_golden
    assert make_golden.check(snappy=os.path.exists(oracle.SNAPPY_SO)) == []
