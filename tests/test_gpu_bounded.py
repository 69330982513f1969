"""GPU: every device-side wait of the snappy kernels is bounded.

* The uncompress's window scan / link / index steps (K1, K2, K3) are three
  ordinary launches, so two contexts decoding tag-dense streams at once (each
  holding part of the machine) cannot deadlock; both decode byte for byte as
  snappy 1.1.8's RawUncompress does (oracle/snappy_port.c restates it).
* The compressor has no device-side wait at all (probe, parse, scan and place
  are four launches; every dependency is a kernel boundary): two contexts
  compressing tag-dense and incompressible streams at once give 1.1.8's bytes.

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


def test_two_contexts_compress_concurrently(port):
    from parameter_server_amd import filter as F
    inputs = [_sorted_keys(4, 4 << 20), np.random.default_rng(5).integers(0, 256, 24 << 20, dtype=np.uint8).tobytes(),
              bytes(8 << 20)]
    want = [port.snappy_compress(x) for x in inputs]
    devs = [torch.from_numpy(np.frombuffer(x, dtype=np.uint8).copy()).cuda() for x in inputs]
    torch.cuda.synchronize()
    ctxs = [F.Context(0, stream=torch.cuda.Stream()) for _ in range(2)]
    results = [[], []]

    def worker(k):
        def go():
            for rep in range(2):
                for i in range(len(devs)):
                    j = (i + k) % len(devs)
                    out = ctxs[k].snappy_compress(devs[j])
                    results[k].append((j, out.cpu().numpy().tobytes()))
        return go

    _run_threads([worker(0), worker(1)])
    for k in range(2):
        for j, got in results[k]:
            assert got == want[j], (k, j)
