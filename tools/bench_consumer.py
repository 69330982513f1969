#!/usr/bin/env python3
"""Server-side consumers after decode, MI355X.

Two consumers of a received push message [KEY_CACHING, FIXING_FLOAT nb=1]
whose m keys are sorted unique uint64:

  kvmap   the async-SGD server: KVMap<Key,float,FTRLEntry>::SetValue
          (kv_map.h:80-91, async_sgd.h:137-151) into a table already holding
          the keys (steady state: every key found)
  match   the BCD server: KVVector::SetValue's ParallelOrderedMatch PLUS
          (kv_vector.h:182-183) of the message into a sorted key/value store
          of D keys

each timed two ways, with HIP events on the context stream:
  unfused FIXING_FLOAT decode materialises the f32 array, the consumer reads it
  fused   the decode is deferred and the consumer dequantises in-register

plus the C restatement (oracle/psf_port.c) of the same consumer on one host
core for scale.  Prints one JSON line.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=10_000_000, help="keys per push message")
    ap.add_argument("--dst", type=int, default=100_000_000, help="keys in the KVVector store")
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    from parameter_server_amd import FIXING_FLOAT, KEY_CACHING
    from parameter_server_amd import filter as F

    dev = "cuda:0"
    ctx = F.Context(0)
    F.set_clock(12345)
    g = torch.Generator(device=dev).manual_seed(3)
    # D sorted unique keys (store), the message's m keys a random subset
    dst = torch.unique(torch.randint(0, 1 << 62, (a.dst + a.dst // 50,), device=dev, generator=g))[:a.dst]
    pick = torch.randperm(dst.numel(), device=dev, generator=g)[:a.m]
    keys = torch.sort(dst[pick])[0].contiguous()
    x = torch.randn(a.m, device=dev, generator=g)
    worker = F.RemoteNode(ctx)
    m = F.Message(request=True, push=True, key_channel=1)
    m.set_key(keys)
    m.add_value(x)
    m.add_filter(KEY_CACHING)
    m.add_filter(FIXING_FLOAT, num_bytes=1)
    worker.encode(m)
    plain, deferred = F.RemoteNode(ctx), F.RemoteNode(ctx)
    deferred.set_defer_dequant(True)
    payload = 12 * a.m  # 8 key + 4 value bytes per key
    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
    res = {"what": "server-side consumer of a [KEY_CACHING, FIXING_FLOAT nb=1] push", "m": a.m,
           "dst_keys": a.dst, "iters": a.iters}

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        e0, e1 = ev(), ev()
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.iters  # ms

    # -- KVMap FTRL -------------------------------------------------------------
    kv = F.KVMap(ctx, capacity=a.m, lr_type=2, alpha=0.01, beta=10.0, lambda1=10.0, lambda2=1.0)
    w0 = m.clone()
    plain.decode(w0)
    kv.set_value(w0)  # insert every key once (steady state afterwards)

    def kv_unfused():
        w = m.clone()
        plain.decode(w)
        kv.set_value(w)

    def kv_fused():
        w = m.clone()
        deferred.decode(w)
        kv.set_value(w)

    t_u, t_f = timed(kv_unfused), timed(kv_fused)
    res["kvmap"] = {"unfused_ms": round(t_u, 3), "fused_ms": round(t_f, 3),
                    "fused_GiBps_payload": round(payload / (t_f * 1e-3) / 2**30, 1),
                    "unfused_GiBps_payload": round(payload / (t_u * 1e-3) / 2**30, 1)}
    del kv

    # -- KVVector ordered match (PLUS) ------------------------------------------
    dval = torch.zeros(a.dst, device=dev)

    def mt_unfused():
        w = m.clone()
        plain.decode(w)
        w.ordered_match(ctx, 0, dst, dval, 1, 1)

    def mt_fused():
        w = m.clone()
        deferred.decode(w)
        w.ordered_match(ctx, 0, dst, dval, 1, 1)

    t_u, t_f = timed(mt_unfused), timed(mt_fused)
    res["match"] = {"unfused_ms": round(t_u, 3), "fused_ms": round(t_f, 3),
                    "fused_GiBps_payload": round(payload / (t_f * 1e-3) / 2**30, 1),
                    "unfused_GiBps_payload": round(payload / (t_u * 1e-3) / 2**30, 1)}

    # per-kernel HIP-event breakdown of the fused paths
    ctx.profile(True)
    ctx.profile_reset()
    kv2 = F.KVMap(ctx, capacity=a.m, lr_type=2, alpha=0.01, beta=10.0, lambda1=10.0, lambda2=1.0)
    for _ in range(3):
        mt_fused()
        w = m.clone()
        deferred.decode(w)
        kv2.set_value(w)
    torch.cuda.synchronize()
    res["kernels"] = {k: {"launches": v[0], "avg_us": round(v[1] / v[0] * 1e3, 1),
                          "alg_GBps": round(v[2] / v[0] / (v[1] / v[0] * 1e-3) / 1e9, 1)}
                      for k, v in ctx.profile_read().items()}
    ctx.profile(False)

    # -- CPU restatement, one core, on a bounded sample --------------------------
    import oracle
    P = oracle.Port()
    ms = min(a.m, 1 << 21)
    sk = keys[:ms].cpu().numpy().view(np.uint64)
    xs = x[:ms].cpu().numpy()
    st, codes, mn, mx = P.ff_encode(xs, 1, 12345)
    idx = np.arange(ms, dtype=np.int64)
    wz = [np.zeros(ms, np.float32) for _ in range(3)]
    nnz, ws, ds = C.c_int64(), C.c_float(), C.c_float()
    t0 = time.perf_counter()
    st, dec = P.ff_decode(codes, 1, mn, mx, np.float32)
    P.lib.port_ftrl_update(idx.ctypes.data_as(C.c_void_p), ms, dec.ctypes.data_as(C.c_void_p),
                           *[w.ctypes.data_as(C.c_void_p) for w in wz], 1, 0.01, 10.0, 10.0, 1.0,
                           C.byref(nnz), C.byref(ws), C.byref(ds))
    t_cpu = time.perf_counter() - t0
    res["cpu_port_kvmap"] = {"GiBps_payload": round(12 * ms / t_cpu / 2**30, 3), "cores": 1,
                             "sample": f"{ms} keys: decode + FTRL update, entries pre-indexed (no hash map)"}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
