"""GPU: ordering and failure paths of the batched drivers.

* The KEY_CACHING signatures the round-trip drivers compute ahead on the
  context's side stream (presign) read key buffers that work already queued on
  the context's stream may still be writing: they are ordered after it, so the
  signature is that of the keys the caller wrote (key_caching.h:18).
* ff_fused_batch's in-launch min/max hand-off, when its bound runs out, makes
  the encode report an error (never silently wrong codes), and leaves the
  context's counter lines clean: the next fused batch is exact.
"""
import ctypes as C

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def test_presign_waits_for_keys_written_on_the_stream(ctx, port):
    """Keys written on the context's stream behind a long kernel, then the
    round trip at once: the presigned CRC must see the written keys."""
    from parameter_server_amd import FIXING_FLOAT, KEY_CACHING
    from parameter_server_amd import filter as F
    m = 50_000
    src = np.sort(np.random.default_rng(3).choice(10**9, m, replace=False)).astype(np.int64)
    src_d = torch.from_numpy(src).to(DEV)
    vals = torch.randn(m, device=DEV)
    torch.cuda.synchronize()
    keys = torch.zeros(m, dtype=torch.int64, device=DEV)
    torch.cuda.synchronize()
    torch.cuda._sleep(100_000_000)  # the keys are written well after the driver starts
    keys.copy_(src_d)
    t = F.Message(request=True, push=True, key_channel=5, key_range=(0, 10**9))
    t.set_key(keys)
    t.add_value(vals)
    t.add_filter(KEY_CACHING)
    t.add_filter(FIXING_FLOAT, num_bytes=1)
    snd, rcv = F.RemoteNode(ctx), F.RemoteNode(ctx)
    F.set_clock(11)
    try:
        (enc, dec), = F.RemoteNode.roundtrip_many([snd], [rcv], [t], 1, keep_last=True)
    finally:
        F.set_clock(None)
    torch.cuda.synchronize()
    assert enc.signature(0) == (True, port.key_signature(src.view(np.uint64)))
    assert snd.key(dec).cpu().numpy().tobytes() == src.tobytes()


def _ff_batch(F, n_arrays, m, seed):
    from parameter_server_amd import FIXING_FLOAT
    g = torch.Generator(device=DEV)
    g.manual_seed(seed)
    msgs, xs = [], []
    for i in range(n_arrays):
        x = torch.randn(m + 17 * i, device=DEV, generator=g)
        t = F.Message(request=True, push=True, key_channel=i)
        t.add_value(x)
        t.add_filter(FIXING_FLOAT, num_bytes=1)
        msgs.append(t)
        xs.append(x.cpu().numpy())
    return msgs, xs


def test_fused_handoff_late_path_reports_error(ctx, port):
    from parameter_server_amd import PsfError, lib
    from parameter_server_amd import filter as F
    from parameter_server_amd._lib import PSF_ERR_HIP
    L = lib()
    L.psf_debug_set_handoff_ticks.argtypes = [C.c_uint64]
    L.psf_debug_set_handoff_ticks.restype = C.c_int
    F.set_clock(77)
    try:
        msgs, _ = _ff_batch(F, 32, 100_000, 1)
        nodes = [F.RemoteNode(ctx) for _ in msgs]
        assert L.psf_debug_set_handoff_ticks(1) == 0
        errors = []
        try:
            try:
                F.RemoteNode.encode_many(nodes, msgs)
                ctx.sync()
            except PsfError as e:
                errors.append(e)
            for m in msgs:
                try:
                    m.fixed_points(0)
                except PsfError as e:
                    errors.append(e)
        finally:
            assert L.psf_debug_set_handoff_ticks(0) == 0
        assert errors, "a hand-off bound of one tick must give up somewhere"
        assert all(e.code == PSF_ERR_HIP and "hand-off" in str(e) for e in errors), errors
        # the counters are clean again: a fresh fused batch is exact
        msgs2, xs2 = _ff_batch(F, 32, 100_000, 2)
        nodes2 = [F.RemoteNode(ctx) for _ in msgs2]
        F.RemoteNode.encode_many(nodes2, msgs2)
        ctx.sync()
        for nd, m, x in zip(nodes2, msgs2, xs2):
            st, codes, mn, mx = port.ff_encode(x, 1, 77)
            (hm, gmn, hx, gmx), = m.fixed_points(0)
            assert (gmn, gmx) == (mn, mx)
            assert nd.value(m, 0).cpu().numpy().tobytes() == codes.tobytes()
    finally:
        F.set_clock(None)
