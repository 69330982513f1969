"""GPU: the per-RemoteNode chain adapter (psf_hip::Chain, include/psf_ps_filter.h)
against the reference's RemoteNode loop restated in oracle/chain.py.

The chain runs the whole of task.filter on one libpsf node per peer (one
context, arrays kept in HBM between filters, only the chain's result back in
host SArrays).  Over the canonical ctr chain [KEY_CACHING(clear_cache_if_done),
FIXING_FLOAT nb=1] (example/linear/ctr/online_l1lr.conf:36-53) driven as the
async-SGD triple (pull request, pull response, push request;
src/app/linear_method/async_sgd.h:229-296), and the C5 chain [KEY_CACHING,
FIXING_FLOAT, COMPRESSING] on dim-128 rows: every wire key and value, every
side-info field and every decoded array equals the restatement's, and equals
what the per-filter adapters behind the reference's own RemoteNode loop give.
"""
import ctypes as C
import os

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

SO = os.path.join(ROOT, "oracle", "_port", "libpsadapter.so")
KC, COMP, FF = 1, 2, 3


@pytest.fixture(scope="module")
def harness():
    assert os.path.exists(SO), "adapter harness not built (make -C oracle adapter)"
    L = C.CDLL(SO)
    vp, sz, u64 = C.c_void_p, C.c_size_t, C.c_uint64
    L.psadapter_peer_new.argtypes = [C.c_int]
    L.psadapter_peer_new.restype = vp
    L.psadapter_peer_free.argtypes = [vp]
    L.psadapter_chain_msg.argtypes = [vp, vp, C.c_int, C.c_int, u64, u64, vp, sz, vp, sz, C.c_int, C.c_int, vp, vp,
                                      vp, C.POINTER(sz), vp, C.POINTER(sz), vp, vp, C.POINTER(sz), vp,
                                      C.POINTER(sz)]
    L.psadapter_chain_msg.restype = C.c_int
    L.psadapter_last_error.restype = C.c_char_p
    return L


class Peer:
    def __init__(self, L, chain):
        self.L, self.h = L, L.psadapter_peer_new(int(chain))

    def __del__(self):
        self.L.psadapter_peer_free(self.h)


def run_msg(L, snd, rcv, flags, ch, kr, key, val, filters):
    """one message through the harness: (wire key, wire value, side-info rows,
    decoded key, decoded value) as bytes / int tuples"""
    key = np.zeros(0, np.uint8) if key is None else np.ascontiguousarray(key).view(np.uint8)
    vb = None if val is None else np.ascontiguousarray(val).view(np.uint8)
    nf = len(filters)
    ft = (C.c_int * nf)(*[f[0] for f in filters])
    fp = (C.c_int * nf)(*[f[1] for f in filters])
    kcap = 64 + 2 * key.size
    vcap = 64 + 2 * (0 if vb is None else vb.size)
    wk, wv = np.zeros(kcap, np.uint8), np.zeros(vcap, np.uint8)
    dk, dv = np.zeros(kcap, np.uint8), np.zeros(vcap, np.uint8)
    side = np.zeros(8 * nf, np.int64)
    wkl, wvl, dkl, dvl = C.c_size_t(), C.c_size_t(), C.c_size_t(), C.c_size_t()
    rc = L.psadapter_chain_msg(snd.h, rcv.h, flags, ch, kr[0], kr[1], key.ctypes.data if key.size else None,
                               key.size, None if vb is None else vb.ctypes.data, 0 if vb is None else vb.size, 9,
                               nf, ft, fp, wk.ctypes.data, C.byref(wkl), wv.ctypes.data, C.byref(wvl),
                               side.ctypes.data, dk.ctypes.data, C.byref(dkl), dv.ctypes.data, C.byref(dvl))
    assert rc == 0, (rc, L.psadapter_last_error())
    rows = [tuple(int(v) for v in side[8 * i:8 * i + 8]) for i in range(nf)]
    return (wk[:wkl.value].tobytes(), wv[:wvl.value].tobytes(), rows, dk[:dkl.value].tobytes(),
            dv[:dvl.value].tobytes())


def oracle_msg(port, snd, rcv, flags, ch, kr, key, val, filters):
    from oracle import chain
    t = chain.Task(bool(flags & 1), bool(flags & 2), bool(flags & 2), ch, kr)
    m = chain.Message(t)
    if key is not None and key.size:
        m.set_key_char(np.ascontiguousarray(key).view(np.uint8))
    if val is not None:
        t.value_type.append(chain.DT_FLOAT)
        m.value.append(np.ascontiguousarray(val).view(np.uint8))
    for ty, p in filters:
        f = chain.FilterConfig(ty)
        if ty == FF:
            f.num_bytes = p
        if ty == KC:
            f.clear_cache_if_done = bool(p)
        t.filter.append(f)
    snd.encode(m)
    rows = []
    for f in t.filter:
        mn = mx = np.float32(0)
        if f.fixed_point:
            mn, mx = np.float32(f.fixed_point[0].min_value), np.float32(f.fixed_point[0].max_value)
        u = list(f.uncompressed_size) + [0, 0]
        rows.append((int(f.has_signature), int(f.signature), int(bool(f.fixed_point)),
                     int(mn.view(np.uint32)), int(mx.view(np.uint32)), len(f.uncompressed_size), int(u[0]),
                     int(u[1])))
    wk = m.key.tobytes()
    wv = m.value[0].tobytes() if m.value else b""
    w = m.clone()
    rcv.decode(w)
    return wk, wv, rows, w.key.tobytes(), (w.value[0].tobytes() if w.value else b"")


def _triple(rng, nkeys, steps):
    """the async-SGD message triple per minibatch over one key set"""
    keys = np.sort(rng.choice(10**12, nkeys, replace=False)).astype(np.uint64)
    for s in range(steps):
        w = (rng.standard_normal(nkeys) * 0.1).astype(np.float32)
        g = rng.standard_normal(nkeys).astype(np.float32)
        yield "w2s", 1, keys, None      # pull request: keys only
        yield "s2w", 0, keys, w         # pull response: keys + weights
        yield "w2s", 3, keys, g         # push request: keys + gradients


@pytest.mark.parametrize("chain_on", [True, False])
def test_ctr_chain_triple_vs_restatement(harness, port, chain_on):
    from oracle import chain
    rng = np.random.default_rng(2)
    seed = 4242
    from parameter_server_amd import filter as F
    F.set_clock(seed)
    try:
        W, S = Peer(harness, chain_on), Peer(harness, chain_on)  # the worker's node for the server, and back
        oW, oS = chain.Node(port, lambda: seed), chain.Node(port, lambda: seed)
        filters = [(KC, 1), (FF, 1)]
        kr = (0, (1 << 64) - 1)
        for i, (d, flags, keys, val) in enumerate(_triple(rng, 100_000, 3)):
            snd, rcv = (W, S) if d == "w2s" else (S, W)
            osnd, orcv = (oW, oS) if d == "w2s" else (oS, oW)
            got = run_msg(harness, snd, rcv, flags, 7, kr, keys, val, filters)
            want = oracle_msg(port, osnd, orcv, flags, 7, kr, keys, val, filters)
            for part, g, w in zip(("wire key", "wire value", "side-info", "decoded key", "decoded value"), got,
                                  want):
                assert g == w, (i, d, flags, part)
    finally:
        F.set_clock(None)


@pytest.mark.parametrize("chain_on", [True, False])
def test_c5_full_chain_vs_restatement(harness, port, chain_on):
    """[KEY_CACHING, FIXING_FLOAT nb=1, COMPRESSING] on m keys x 128 f32 rows:
    the first send compresses the keys (a miss), the repeats elide them."""
    from oracle import chain
    from parameter_server_amd import filter as F
    rng = np.random.default_rng(5)
    m = 1 << 13
    keys = np.sort(rng.choice(1 << 62, m, replace=False)).astype(np.uint64)
    seed = 99
    F.set_clock(seed)
    try:
        W, S = Peer(harness, chain_on), Peer(harness, chain_on)
        oW, oS = chain.Node(port, lambda: seed), chain.Node(port, lambda: seed)
        filters = [(KC, 0), (FF, 1), (COMP, 0)]
        kr = (0, (1 << 64) - 1)
        for step in range(3):
            v = rng.standard_normal(m * 128).astype(np.float32)
            got = run_msg(harness, W, S, 3, 11, kr, keys, v, filters)
            want = oracle_msg(port, oW, oS, 3, 11, kr, keys, v, filters)
            for part, g, w in zip(("wire key", "wire value", "side-info", "decoded key", "decoded value"), got,
                                  want):
                assert g == w, (step, part)
            assert (len(got[0]) > 0) == (step == 0)  # keys travel (compressed) on the miss only
    finally:
        F.set_clock(None)

