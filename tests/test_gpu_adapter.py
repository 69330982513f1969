"""GPU: the reference-side drop-in (include/psf_ps_filter.h), compiled against
a test double of the PS types (oracle/ps_mock, oracle/adapter_harness.cc) and
run on PS::Messages in host memory, as a patched reference would run it:
wire bytes, FilterConfig side-info and decoded arrays against the C
restatement (oracle/psf_port.c, snappy_port.c, oracle/chain.py); each adapter
instance on its own stream, several of them concurrently on their own threads."""
import ctypes as C
import os

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

SO = os.path.join(ROOT, "oracle", "_port", "libpsadapter.so")


@pytest.fixture(scope="module")
def harness():
    assert os.path.exists(SO), "adapter harness not built (make -C oracle adapter)"
    L = C.CDLL(SO)
    vp, sz = C.c_void_p, C.c_size_t
    L.psadapter_ff.argtypes = [vp, sz, C.c_int, C.c_int, C.c_int64, C.c_int, C.c_float, C.c_int, C.c_float,
                               vp, C.POINTER(C.c_float), vp]
    L.psadapter_ff.restype = C.c_int
    L.psadapter_ff_threads.argtypes = [C.c_int, C.c_int, vp, sz, C.c_int, C.c_int, C.c_int64, vp,
                                       C.POINTER(C.c_float), vp]
    L.psadapter_ff_threads.restype = C.c_double
    L.psadapter_compress.argtypes = [vp, sz, vp, sz, C.c_int, vp, C.POINTER(sz), vp, C.POINTER(sz),
                                     C.POINTER(C.c_uint64), C.POINTER(C.c_int), vp, vp]
    L.psadapter_compress.restype = C.c_int
    L.psadapter_noise.argtypes = [vp, sz, C.c_int, C.c_float, C.c_float, vp, vp]
    L.psadapter_noise.restype = C.c_int
    L.psadapter_kc.argtypes = [C.c_int, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]
    L.psadapter_kc.restype = None
    L.psadapter_last_error.restype = C.c_char_p
    return L


def _ff(L, x, nb, seed, mn=None, mx=None):
    codes = np.zeros(x.size * nb, np.uint8)
    dec = np.zeros_like(x)
    rng = (C.c_float * 2)()
    rc = L.psadapter_ff(x.ctypes.data, x.nbytes, 9 if x.dtype == np.float32 else 10, nb, seed,
                        mn is not None, 0.0 if mn is None else mn, mx is not None, 0.0 if mx is None else mx,
                        codes.ctypes.data, rng, dec.ctypes.data)
    return rc, codes, (rng[0], rng[1]), dec


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("nb", [1, 2, 3, 5])
def test_adapter_fixing_float_vs_port(harness, port, dtype, nb):
    x = np.random.default_rng(nb).standard_normal(100_003).astype(dtype)
    for seed, mn, mx in ((12345, None, None), (-77, -1.0, 1.0)):
        rc, codes, (gmn, gmx), dec = _ff(harness, x, nb, seed, mn, mx)
        assert rc == 0, harness.psadapter_last_error()
        st, pc, pmn, pmx = port.ff_encode(x, nb, seed, mn, mx)
        assert st == 0 and np.array_equal(codes, pc)
        assert np.float32(gmn).tobytes() == np.float32(pmn).tobytes()
        assert np.float32(gmx).tobytes() == np.float32(pmx).tobytes()
        st, pd = port.ff_decode(pc, nb, pmn, pmx, dtype)
        assert dec.tobytes() == pd.tobytes()


def test_adapter_rejects_like_reference(harness):
    x = np.full(64, 40.0, np.float32)  # fixing_float.h:71 CHECK_GT(bin, 0)
    assert _ff(harness, x, 1, 1)[0] == -1


def test_adapter_instances_concurrent(harness, port):
    """Four adapter instances on four threads (four Customers' executor
    threads), each with its own libpsf context: every thread's output equals
    the restatement; the wall times of 1 and 4 concurrent threads are
    printed (host-memory messages: PCIe-bound)."""
    x = np.random.default_rng(3).standard_normal(1 << 22).astype(np.float32)
    st, pc, pmn, pmx = port.ff_encode(x, 1, 99)
    st, pd = port.ff_decode(pc, 1, pmn, pmx, np.float32)
    times = {}
    for T in (1, 4):
        codes = np.zeros(T * x.size, np.uint8)
        dec = np.zeros(T * x.size, np.float32)
        rng = (C.c_float * (2 * T))()
        t = harness.psadapter_ff_threads(T, 4, x.ctypes.data, x.nbytes, 9, 1, 99, codes.ctypes.data, rng,
                                         dec.ctypes.data)
        assert t > 0, harness.psadapter_last_error()
        times[T] = t
        for k in range(T):
            assert np.array_equal(codes[k * x.size:(k + 1) * x.size], pc), k
            assert dec[k * x.size:(k + 1) * x.size].tobytes() == pd.tobytes(), k
            assert (rng[2 * k], rng[2 * k + 1]) == (pmn, pmx)
    print(f"adapter: 4 x 16 MiB encode+decode, 1 thread {times[1]:.3f} s, 4 threads x 4 {times[4]:.3f} s")


@pytest.mark.parametrize("nkeys", [0, 5, 3000, 200_000])
def test_adapter_compressing_vs_port(harness, port, nkeys):
    """CompressingFilter (compressing.h:8-37): snappy 1.1.8 bytes for keys
    and values, uncompressed_size side-info, decode restores the input."""
    rng = np.random.default_rng(nkeys)
    keys = np.sort(rng.choice(10**9, size=nkeys, replace=False)).astype(np.uint64)
    for vals in (rng.standard_normal(nkeys + 7).astype(np.float32),
                 np.clip(rng.standard_normal(70_000) * 20 + 128, 0, 255).astype(np.uint8),
                 np.zeros(0, np.float32)):
        kcap, vcap = 64 + keys.nbytes * 2, 64 + vals.nbytes * 2
        ko, vo = np.zeros(kcap, np.uint8), np.zeros(vcap, np.uint8)
        kd, vd = np.zeros(max(keys.nbytes, 1), np.uint8), np.zeros(max(vals.nbytes, 1), np.uint8)
        kl, vl, ns = C.c_size_t(), C.c_size_t(), C.c_int()
        sizes = (C.c_uint64 * 2)()
        rc = harness.psadapter_compress(keys.ctypes.data if nkeys else None, keys.nbytes,
                                        vals.ctypes.data if vals.size else None, vals.nbytes, 9,
                                        ko.ctypes.data, C.byref(kl), vo.ctypes.data, C.byref(vl), sizes,
                                        C.byref(ns), kd.ctypes.data, vd.ctypes.data)
        assert rc == 0, (rc, harness.psadapter_last_error())
        want_k = port.snappy_compress(keys.tobytes()) if nkeys else b""
        want_v = port.snappy_compress(vals.tobytes()) if vals.size else b""
        assert ko[:kl.value].tobytes() == want_k and vo[:vl.value].tobytes() == want_v
        want_sizes = ([keys.nbytes] if nkeys else []) + [vals.nbytes]
        assert [sizes[i] for i in range(ns.value)] == want_sizes
        assert kd[:keys.nbytes].tobytes() == keys.tobytes() and vd[:vals.nbytes].tobytes() == vals.tobytes()


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_adapter_noise_in_place_vs_port(harness, port, dtype):
    """AddNoiseFilter (add_noise.h:11-39): bit-identical noise, written into
    the shared buffer itself (an alias of the array sees it too)."""
    x = np.linspace(-1, 1, 5001).astype(dtype)
    out, alias = np.zeros_like(x), np.zeros_like(x)
    rc = harness.psadapter_noise(x.ctypes.data, x.nbytes, 9 if dtype == np.float32 else 10, 0.5, 2.0,
                                 out.ctypes.data, alias.ctypes.data)
    assert rc == 0, (rc, harness.psadapter_last_error())
    want = port.add_noise(x, 0.5, 2.0)
    assert out.tobytes() == want.tobytes() and alias.tobytes() == want.tobytes()


def test_adapter_key_caching_vs_restatement(harness, port):
    """KeyCachingFilter (key_caching.h:9-60) through libpsf, sender and
    receiver instances over a message sequence: hits clear the key on the wire
    and the receiver restores it, per (channel, key_range); a key changed only
    past its first 2 KiB is a (reference) false hit; clear_cache_if_done on a
    push request or a response drops the entry; a restarted receiver fails
    the decode CHECK.  Every wire length, signature and restored key equals
    the restatement's (oracle/chain.py)."""
    from oracle import chain
    rng = np.random.default_rng(11)
    A = np.sort(rng.choice(10**9, 5000, replace=False)).astype(np.uint64).view(np.uint8)
    B = np.sort(rng.choice(10**9, 7000, replace=False)).astype(np.uint64).view(np.uint8)
    B2 = B.copy()
    B2[3000] ^= 0x5A  # past the signature's 2 KiB
    Cs = rng.integers(0, 256, 100, dtype=np.uint8)
    E = np.zeros(0, np.uint8)
    R0, R1 = (0, 1 << 40), (1 << 40, 1 << 41)
    seq = [(A, 0, R0, 1), (A, 0, R0, 1), (A, 1, R0, 1), (A, 0, R1, 1), (B, 0, R0, 1), (B2, 0, R0, 1),
           (E, 0, R0, 1), (B, 0, R0, 1 | 2 | 4), (B, 0, R0, 1), (B, 0, R0, 1), (A, 1, R0, 4),
           (A, 1, R0, 1), (Cs, 2, R1, 1), (Cs, 2, R1, 1 | 8)]
    n = len(seq)
    kbuf = np.concatenate([k for k, *_ in seq])
    koff = np.concatenate([[0], np.cumsum([k.size for k, *_ in seq])]).astype(np.uint64)
    ch = np.array([c for _, c, _, _ in seq], np.int32)
    rb = np.array([r[0] for _, _, r, _ in seq], np.uint64)
    re_ = np.array([r[1] for _, _, r, _ in seq], np.uint64)
    fl = np.array([f for *_, f in seq], np.int32)
    sent, has, sig = np.zeros(n, np.uint64), np.zeros(n, np.int32), np.zeros(n, np.uint32)
    got, rc = np.zeros(n, np.int32), np.zeros(n, np.int32)
    harness.psadapter_kc(n, kbuf.ctypes.data, koff.ctypes.data, ch.ctypes.data, rb.ctypes.data, re_.ctypes.data,
                         fl.ctypes.data, sent.ctypes.data, has.ctypes.data, sig.ctypes.data, got.ctypes.data,
                         rc.ctypes.data)
    snd, rcv = chain.KeyCaching(port), chain.KeyCaching(port)
    for i, (k, c, r, f) in enumerate(seq):
        if f & 8:
            rcv = chain.KeyCaching(port)
        t = chain.Task(bool(f & 1), bool(f & 2), bool(f & 2), c, r)
        m = chain.Message(t)
        if k.size:
            m.set_key_char(k)
        conf = chain.FilterConfig(chain.KEY_CACHING)
        conf.clear_cache_if_done = bool(f & 4)
        t.filter.append(conf)
        snd.encode(m)
        assert rc[i] != 1, (i, harness.psadapter_last_error())
        assert (int(sent[i]), bool(has[i]), int(sig[i])) == (m.key.size, conf.has_signature, conf.signature), i
        w = m.clone()
        try:
            rcv.decode(w)
        except chain.CheckFailed:
            assert rc[i] == 2, i  # both fail the CHECK here
            assert i == n - 1
            break
        assert rc[i] == 0, (i, harness.psadapter_last_error())
        want = w.key.size == k.size and w.key.tobytes() == k.tobytes()
        assert bool(got[i]) == want, i
    assert rc[-1] == 2 and not got[5] and sent[1] == 0 and sent[5] == 0


def test_adapter_256_instances_one_device_budget(harness):
    """A server with 256 worker peers: 256 per-filter FIXING_FLOAT adapter
    instances on one device, message sizes cycling.  The cached HBM of all of
    them together stays under the ONE device cap (psf_device_memory_stats), and
    their contexts share the device's 4 streams instead of 256 private ones."""
    import torch  # noqa: F401  (HIP runtime up before the harness)

    from parameter_server_amd import filter as F
    L = harness
    L.psadapter_many_instances.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_size_t, C.c_size_t,
                                           C.POINTER(C.c_uint64)]
    L.psadapter_many_instances.restype = C.c_int
    cap = 96 << 20
    F.set_device_cache_limit(0, cap, 32 << 20)
    try:
        x = np.random.default_rng(3).standard_normal(1 << 21).astype(np.float32)
        out = (C.c_uint64 * 6)()
        rc = L.psadapter_many_instances(256, 3, x.ctypes.data, 1 << 16, 1 << 21, out)
        assert rc == 0, L.psadapter_last_error()
        peak_cached, dev_cap, streams, shared, evictions, peak_alloc = list(out)
        assert dev_cap == cap
        assert peak_cached <= cap, (peak_cached, cap)
        assert evictions > 0  # 256 instances x distinct sizes would cache far more than 96 MiB
        assert shared <= 4 and streams <= 16, (streams, shared)
    finally:
        F.set_device_cache_limit(0, *F.DEFAULT_CACHE_LIMIT)


def test_adapter_context_used_from_another_thread(harness, port):
    """An instance created on one thread and run from another (the
    reference's app thread encodes, the executor thread decodes): every
    libpsf entry makes the context's device current and restores the
    thread's own.  With one GPU this runs on device 0 on both threads."""
    import torch
    L = harness
    L.psadapter_ff_cross_thread.argtypes = [C.c_void_p, C.c_size_t, C.c_int, C.c_int64, C.c_int, C.c_void_p,
                                            C.POINTER(C.c_float), C.c_void_p]
    L.psadapter_ff_cross_thread.restype = C.c_int
    other = 1 if torch.cuda.device_count() > 1 else 0
    x = np.random.default_rng(5).standard_normal(300_007).astype(np.float32)
    codes = np.zeros(x.size, np.uint8)
    dec = np.zeros_like(x)
    rng = (C.c_float * 2)()
    rc = L.psadapter_ff_cross_thread(x.ctypes.data, x.nbytes, 1, 99, other, codes.ctypes.data, rng,
                                     dec.ctypes.data)
    assert rc == 0, (rc, L.psadapter_last_error())
    st, pc, mn, mx = port.ff_encode(x, 1, 99)
    assert st == 0 and np.array_equal(codes, pc)
    st, pd = port.ff_decode(pc, 1, mn, mx, np.float32)
    assert dec.tobytes() == pd.tobytes()
