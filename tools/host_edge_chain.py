"""The host edge through the reference-side adapter (include/psf_ps_filter.h):
messages built in host memory (PS::Message test double, oracle/ps_mock) run
through the patched RemoteNode (psf_hip::Chain: one libpsf context per peer,
arrays in HBM between filters) and, for comparison, through the reference's
own RemoteNode loop over the per-filter adapters (Filter::create hook only).
Rates are GiB/s of key-value payload (key + value bytes before encode, as the
bench's metric) through encode + decode, H2D and D2H included.

  python tools/host_edge_chain.py [--out gpurun_out/host_edge_chain.jsonl]

Each config runs warm twice first, then: "chain" (encode then decode, one
thread), "chain_two_threads" (the encodes on one thread and the decodes on
another, as the reference's application and executor threads run them;
single-direction configs), "per_filter".  PSAD_FRESH=1: new arrays every
round (an application allocating a new gradient array per minibatch).

Configs: the ctr triple (C1: 10^5 keys, [KEY_CACHING(clear_cache_if_done),
FIXING_FLOAT nb=1], pull request / pull response / push request), C2 on the
host (2^27 f32, [FIXING_FLOAT nb=1]), C5 + COMPRESSING (2^20 keys x 128 f32
rows, [KEY_CACHING, FIXING_FLOAT nb=1, COMPRESSING]) with keys elided (hits)
and with every send a miss (clear_cache_if_done on a push).
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SO = os.path.join(ROOT, "oracle", "_port", "libpsadapter.so")
KC, COMP, FF = 1, 2, 3


def harness():
    L = C.CDLL(SO)
    vp = C.c_void_p
    L.psadapter_peer_new.argtypes = [C.c_int]
    L.psadapter_peer_new.restype = vp
    L.psadapter_peer_free.argtypes = [vp]
    L.psadapter_chain_bench.argtypes = [vp, vp, C.c_int, C.c_int, vp, vp, vp, vp, vp, vp, C.c_int, C.c_int,
                                        C.c_int, vp, vp, C.POINTER(C.c_double), C.POINTER(C.c_double)]
    L.psadapter_chain_bench.restype = C.c_double
    L.psadapter_chain_bench_pipelined.argtypes = [vp, vp, C.c_int, C.c_int, vp, vp, vp, vp, vp, C.c_int, C.c_int,
                                                  C.c_int, vp, vp]
    L.psadapter_chain_bench_pipelined.restype = C.c_double
    L.psadapter_last_error.restype = C.c_char_p
    return L


def run(L, name, msgs, filters, iters, warm=2):
    """msgs: [(flags, dir, keys u8 array, values u8 array)]"""
    keys = [m[2] for m in msgs]
    vals = [m[3] for m in msgs]
    kbuf = np.concatenate(keys) if keys else np.zeros(0, np.uint8)
    vbuf = np.concatenate(vals) if vals else np.zeros(0, np.uint8)
    koff = np.concatenate([[0], np.cumsum([k.size for k in keys])]).astype(np.uint64)
    voff = np.concatenate([[0], np.cumsum([v.size for v in vals])]).astype(np.uint64)
    fl = np.array([m[0] for m in msgs], np.int32)
    dr = np.array([m[1] for m in msgs], np.int32)
    ft = np.array([f[0] for f in filters], np.int32)
    fp = np.array([f[1] for f in filters], np.int32)
    payload = int(koff[-1] + voff[-1])
    out = {"config": name, "payload_bytes_per_round": payload}
    for mode in ("chain", "per_filter"):
        W, S = L.psadapter_peer_new(int(mode == "chain")), L.psadapter_peer_new(int(mode == "chain"))
        e, d = C.c_double(), C.c_double()
        args = (W, S, 0, len(msgs), kbuf.ctypes.data, koff.ctypes.data, vbuf.ctypes.data, voff.ctypes.data,
                fl.ctypes.data, dr.ctypes.data, 1, 9, len(filters), ft.ctypes.data, fp.ctypes.data, C.byref(e),
                C.byref(d))
        a = list(args)
        a[2] = warm
        assert L.psadapter_chain_bench(*a) > 0, L.psadapter_last_error()
        a[2] = iters
        t = L.psadapter_chain_bench(*a)
        assert t > 0, L.psadapter_last_error()
        out[mode] = {"gib_s": payload / t / 2**30, "s_per_round": t, "encode_s": e.value, "decode_s": d.value}
        if mode == "chain" and not any(m[1] for m in msgs):
            # the encodes and decodes on two threads (app thread / executor thread)
            tp = L.psadapter_chain_bench_pipelined(W, S, iters, len(msgs), kbuf.ctypes.data, koff.ctypes.data,
                                                   vbuf.ctypes.data, voff.ctypes.data, fl.ctypes.data, 1, 9,
                                                   len(filters), ft.ctypes.data, fp.ctypes.data)
            assert tp > 0, L.psadapter_last_error()
            out["chain_two_threads"] = {"gib_s": payload / tp / 2**30, "s_per_round": tp}
        L.psadapter_peer_free(W)
        L.psadapter_peer_free(S)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "host_edge_chain.jsonl"))
    ap.add_argument("--quick", action="store_true")
    a = ap.parse_args()
    from parameter_server_amd import filter as F
    F.set_clock(12345)
    L = harness()
    rng = np.random.default_rng(2)
    res = []
    # C1: the ctr triple
    keys = np.sort(rng.choice(10**12, 100_000, replace=False)).astype(np.uint64).view(np.uint8)
    w = (rng.standard_normal(100_000) * 0.1).astype(np.float32).view(np.uint8)
    g = rng.standard_normal(100_000).astype(np.float32).view(np.uint8)
    e = np.zeros(0, np.uint8)
    res.append(run(L, "c1_ctr_triple_1e5_keys", [(1, 0, keys, e), (0, 1, keys, w), (3, 0, keys, g)],
                   [(KC, 1), (FF, 1)], 20 if not a.quick else 3))
    # C2 from host memory
    n = 1 << (27 if not a.quick else 24)
    x = rng.standard_normal(n).astype(np.float32).view(np.uint8)
    res.append(run(L, f"c2_host_2^{n.bit_length() - 1}_f32", [(3, 0, e, x)], [(FF, 1)], 5 if not a.quick else 2))
    del x
    # C5 + COMPRESSING from host memory
    m = 1 << (20 if not a.quick else 16)
    k5 = np.sort(rng.choice(1 << 62, m, replace=False)).astype(np.uint64).view(np.uint8)
    v5 = rng.standard_normal(m * 128).astype(np.float32).view(np.uint8)
    res.append(run(L, "c5_compress_hits", [(3, 0, k5, v5)], [(KC, 0), (FF, 1), (COMP, 0)], 3 if not a.quick else 2))
    res.append(run(L, "c5_compress_miss", [(3, 0, k5, v5)], [(KC, 1), (FF, 1), (COMP, 0)], 3 if not a.quick else 2))
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        for r in res:
            line = json.dumps(r)
            print(line, flush=True)
            f.write(line + "\n")


if __name__ == "__main__":
    t0 = time.time()
    main()
    print(f"host_edge_chain: {time.time() - t0:.1f} s", flush=True)
