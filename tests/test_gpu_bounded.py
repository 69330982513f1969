"""GPU: every device-side wait of the snappy kernels is bounded.

* The uncompress's window scan / link / index steps (K1, K2, K3) are three
  ordinary launches, so two contexts decoding tag-dense streams at once (each
  holding part of the machine) cannot deadlock; both decode byte for byte as
  snappy 1.1.8's RawUncompress does (oracle/snappy_port.c restates it).
* The compressor's look-back gives up after a capped number of polls: with a
  fragment that never publishes (the psf_debug_snappy_stall knob), the call
  returns PSF_ERR_TIMEOUT instead of hanging, and the context still works.

Reference: src/filter/compressing.h:8-37, src/util/shared_array_inl.h:232-255.
"""
import threading

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _sorted_keys(seed, nbytes):
    rng = np.random.default_rng(seed)
    return np.sort(rng.integers(0, 10**9, nbytes // 8, dtype=np.uint64)).tobytes()


def _run_threads(fns):
    errs = [None] * len(fns)

    def wrap(i):
        try:
            fns[i]()
        except BaseException as e:  # noqa: BLE001 - reported below
            errs[i] = e

    ts = [threading.Thread(target=wrap, args=(i,)) for i in range(len(fns))]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=90)
        assert not t.is_alive(), "a decoding thread did not finish"
    for e in errs:
        if e is not None:
            raise e


def test_two_contexts_uncompress_tag_dense_concurrently(port):
    from parameter_server_amd import filter as F
    inputs = [_sorted_keys(1, 12 << 20), bytes(24 << 20), _sorted_keys(2, 6 << 20) + bytes(6 << 20)]
    streams = [port.snappy_compress(x) for x in inputs]
    for x, s in zip(inputs, streams):
        st, back = port.snappy_uncompress(s, cap=len(x))
        assert st == 0 and back == x
    devs = [torch.from_numpy(np.frombuffer(s, dtype=np.uint8).copy()).cuda() for s in streams]
    torch.cuda.synchronize()
    ctxs = [F.Context(0, stream=torch.cuda.Stream()) for _ in range(2)]
    results = [[], []]

    def worker(k):
        def go():
            for rep in range(3):
                for i in range(len(devs)):
                    j = (i + k) % len(devs)  # the two threads decode different streams at once
                    out = ctxs[k].snappy_uncompress(devs[j])
                    ctxs[k].sync()
                    results[k].append((j, out.cpu().numpy().tobytes()))
        return go

    _run_threads([worker(0), worker(1)])
    for k in range(2):
        assert len(results[k]) == 3 * len(devs)
        for j, got in results[k]:
            assert got == inputs[j], (k, j)


def test_two_contexts_compressing_filter_decode_concurrently(port):
    """The same through the COMPRESSING filter's batched decode (the message
    path): one node per context, sorted keys and zeros as the values."""
    from parameter_server_amd import COMPRESSING
    from parameter_server_amd import filter as F
    vals = [np.frombuffer(_sorted_keys(3, 8 << 20), dtype=np.uint8), np.zeros(16 << 20, dtype=np.uint8)]
    ctxs = [F.Context(0, stream=torch.cuda.Stream()) for _ in range(2)]
    encoded = []
    for v in vals:
        m = F.Message(request=True, push=True)
        m.add_value(torch.from_numpy(v.copy()).cuda())
        m.add_filter(COMPRESSING)
        F.RemoteNode(ctxs[0]).encode(m)
        ctxs[0].sync()
        p, n, loc = m.value_ptr(0)
        got = F.copy_out(p, n, loc, "cuda:0").cpu().numpy().tobytes()
        assert got == port.snappy_compress(v.tobytes())
        encoded.append(m)
    out = [[], []]

    def worker(k):
        def go():
            node = F.RemoteNode(ctxs[k])
            for rep in range(3):
                for i in range(len(encoded)):
                    j = (i + k) % len(encoded)
                    w = encoded[j].clone()
                    node.decode(w)
                    ctxs[k].sync()
                    p, n, loc = w.value_ptr(0)
                    out[k].append((j, F.copy_out(p, n, loc, "cuda:0").cpu().numpy().tobytes()))
        return go

    _run_threads([worker(0), worker(1)])
    for k in range(2):
        for j, got in out[k]:
            assert got == vals[j].tobytes(), (k, j)


def test_compress_lookback_cap_returns_timeout(ctx, port):
    from parameter_server_amd import COMPRESSING, lib
    from parameter_server_amd import filter as F
    from parameter_server_amd._lib import PSF_ERR_TIMEOUT, PsfError
    rng = np.random.default_rng(11)
    x = rng.integers(0, 4, 40 * 65536 + 777, dtype=np.uint8)  # 41 fragments, some matches
    xd = torch.from_numpy(x).cuda()
    want = port.snappy_compress(x.tobytes())
    try:
        for frag in (0, 17):
            lib().psf_debug_snappy_stall(frag, 1 << 12)
            with pytest.raises(PsfError) as e:
                ctx.snappy_compress(xd)
            assert e.value.code == PSF_ERR_TIMEOUT, frag
        # the message path (COMPRESSING encode, batched launch with the
        # context's pre-zeroed look-back region) reports it as well
        m = F.Message(request=True, push=True)
        m.add_value(xd)
        m.add_filter(COMPRESSING)
        with pytest.raises(PsfError) as e:
            F.RemoteNode(ctx).encode(m)
        assert e.value.code == PSF_ERR_TIMEOUT
    finally:
        lib().psf_debug_snappy_stall(-1, 0)
    # the context keeps working: both paths byte-identical again
    assert ctx.snappy_compress(xd).cpu().numpy().tobytes() == want
    for _ in range(2):  # both halves of the pre-zeroed region pair
        m = F.Message(request=True, push=True)
        m.add_value(xd)
        m.add_filter(COMPRESSING)
        F.RemoteNode(ctx).encode(m)
        ctx.sync()
        p, n, loc = m.value_ptr(0)
        assert F.copy_out(p, n, loc, "cuda:0").cpu().numpy().tobytes() == want
