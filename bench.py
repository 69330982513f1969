#!/usr/bin/env python3
"""bench.py -- BASELINE.json metric: GiB/s of key-value payload through the
filter encode+decode chain, device-resident, on MI355X.

Default workload (BASELINE.json configs[1]): one message
per step carrying n = 2^27 dense float32 values (512 MiB, N(0,1), seed 1) and
the chain [FIXING_FLOAT num_bytes=1] with min/max computed; a step encodes it on
the worker's RemoteNode, delivers it and decodes it on the server's
(libpsf psf_node_roundtrip: no Python per message).  Payload = 4n bytes/step.

N GPUs (torchrun, one rank per GPU): rank g is server g of EvenDivide(N, g)
and codes its own pre-placed shard (no data-path collective; weak scaling).
Timed region: barrier + synchronize, K steps, barrier + synchronize; the max
elapsed over ranks is the job time.  value = N * K * payload / time.

roofline: per-kernel durations from HIP events recorded on the launch stream
around every kernel inside the timed region (libpsf profiler); the dominant
kernel's algorithmic bytes / average duration vs 8 TB/s.  traffic: PMC-derived
HBM bytes per launch from profiles/pmc_traffic.json when it matches (see
tools/pmc_traffic.py), else null.
cpu_baseline: the reference's own filter code (oracle/_ref, unmodified
headers) -- or the C restatement if that is absent -- on one host core, rank 0
at N=1 only, over a bounded sample (2^24 values, repeated ~10 s).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

GIB = float(1 << 30)
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, MI355X_MICROARCH.md


WORKLOADS = {
    "c2": "C2 (BASELINE configs[1]): dense f32 values, chain [FIXING_FLOAT num_bytes={nb}], "
          "min/max computed, encode+decode round trip per step",
    "c3": "C3 (BASELINE configs[2]): 10M uint64 keys @1% of [0,1e9) + f32 values, chain "
          "[KEY_CACHING, FIXING_FLOAT num_bytes={nb}], repeat send (key cache hit: keys elided)",
    "c3miss": "C3 (BASELINE configs[2]) first-send path: 10M uint64 keys @1% of [0,1e9) + f32 "
              "values, chain [KEY_CACHING(clear_cache_if_done), FIXING_FLOAT num_bytes={nb}], "
              "every send a key cache miss",
    "c4": "C4 (BASELINE configs[3]): {streams} push streams in total (stream s on rank s % N), each "
          "{m} sorted unique uint64 keys spread over 2^64 (splitmix64) + f32 values, sliced at the "
          "EvenDivide(N) server ranges, per-(stream, server) [KEY_CACHING, FIXING_FLOAT num_bytes={nb}], "
          "cross-range slices spilled in one all-to-all-v per step (RCCL), repeat sends (key cache hit)",
    "c1": "C1 (BASELINE configs[0]) on the device: the ctr example's push stream "
          "(example/linear/ctr/online_l1lr.conf: [KEY_CACHING(clear_cache_if_done), FIXING_FLOAT "
          "num_bytes={nb}]), {streams} concurrent minibatch streams of {m} sorted unique keys + f32 "
          "gradients, all streams' messages of a step encoded / decoded in one batched call (repeat sends)",
    "c5": "C5 (BASELINE configs[4]) per GPU: 2^20 uint64 keys spread over 2^64 (splitmix64) + "
          "embedding rows dim=128 f32 (512 MiB, one min/max per array), chain [KEY_CACHING, "
          "FIXING_FLOAT num_bytes={nb}{cmp}], repeat send (key cache hit)",
}


def splitmix64_keys(m: int, seed: int):
    """m sorted unique uint64 keys splitmix64(seed + i)."""
    import numpy as np
    with np.errstate(over="ignore"):
        z = (np.arange(m, dtype=np.uint64) + np.uint64(seed)) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return np.unique(z)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--n", type=int, default=1 << 27, help="values per message (per GPU)")
    ap.add_argument("--nb", type=int, default=1, help="FIXING_FLOAT num_bytes")
    ap.add_argument("--bufs", type=int, default=3, help="distinct messages cycled through")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--streams", type=int, default=64, help="c4: push streams in total")
    ap.add_argument("--config", default="c2", choices=["c1", "c2", "c3", "c3miss", "c4", "c5"],
                    help="c2: dense f32 values (default, the headline); c3: 10M sorted uint64 "
                         "keys from [0,1e9) + f32 values, [KEY_CACHING, FIXING_FLOAT] repeat "
                         "sends (cache hits); c3miss: same with clear_cache_if_done (every send "
                         "a miss)")
    ap.add_argument("--m", type=int, default=None, help="keys per message (c3: 10M, c5: 2^20)")
    ap.add_argument("--compress", action="store_true", help="append COMPRESSING to the chain (c5)")
    return ap.parse_args()


def cpu_baseline(n_sample: int, nb: int, seconds: float, config: str = "c2"):
    import ctypes as C

    import numpy as np

    import oracle
    x = np.random.default_rng(1).standard_normal(n_sample).astype(np.float32)
    keys = None
    if config != "c2":  # C3 sample: sorted unique keys from [0, 1e9), KEY_CACHING first
        keys = np.unique(np.random.default_rng(3).integers(0, 10**9, n_sample + n_sample // 8,
                                                            dtype=np.uint64))[:n_sample]
        keys = np.ascontiguousarray(keys[:x.size])
        x = x[:keys.size]
    kind = "port"
    try:
        R = oracle.Ref()
        kind = "reference"
    except Exception:
        R = None
    reps, t = 0, 0.0
    if R is not None:
        L = R.lib
        R.set_time(12345)
        snd, rcv = L.psref_node_new(), L.psref_node_new()
        while t < seconds or reps == 0:
            m = R.msg_new(request=True, push=True, key_range=(0, 10**9))
            if keys is not None:
                L.psref_msg_set_key(m, keys.ctypes.data_as(C.c_void_p), keys.nbytes, 8)
                kf = L.psref_msg_add_filter(m, 1)
                L.psref_fc_set_clear_cache(m, kf, int(config == "c3miss"))
            L.psref_msg_add_value(m, x.ctypes.data_as(C.c_void_p), x.nbytes, 9)
            fi = L.psref_msg_add_filter(m, 3)
            L.psref_fc_set_num_bytes(m, fi, nb)
            t0 = time.perf_counter()
            assert L.psref_node_encode(snd, m) == 0
            w = L.psref_msg_clone(m)
            assert L.psref_node_decode(rcv, w) == 0
            t += time.perf_counter() - t0
            L.psref_msg_free(w)
            L.psref_msg_free(m)
            reps += 1
    else:
        P = oracle.Port()
        while t < seconds or reps == 0:
            t0 = time.perf_counter()
            st, codes, mn, mx = P.ff_encode(x, nb, 12345)
            P.ff_decode(codes, nb, mn, mx)
            t += time.perf_counter() - t0
            reps += 1
    payload = x.nbytes + (keys.nbytes if keys is not None else 0)
    chain = "FIXING_FLOAT" if keys is None else "KEY_CACHING+FIXING_FLOAT"
    return {
        "value": round(reps * payload / t / GIB, 4),
        "unit": "GiB/s",
        "cores": 1,
        "kind": kind,
        "sample": f"{reps} x {chain}(nb={nb}) encode+decode of 2^{n_sample.bit_length() - 1} f32 "
                  f"({payload >> 20} MiB payload), single-threaded as the reference's filters run, "
                  f"{t:.1f} s CPU",
        "cpu_model": _cpu_model(),
        "nproc": os.cpu_count(),
    }


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def pmc_traffic(kernel: str, n: int, nb: int, config: str):
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        d = json.load(open(path))
    except (OSError, ValueError):
        return None
    e = d.get(kernel)
    # profiles/pmc_traffic.json holds the C2 passes (tools/gpu_profile.sh)
    if config != "c2" or not e or e.get("n") != n or e.get("nb") != nb:
        return None
    return e.get("hbm_bytes_per_launch")


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    import torch.distributed as dist

    # rehearsal knobs (never set by the driver): PSF_DIST_BACKEND=gloo and
    # PSF_SAME_GPU=1 run N ranks on one GPU with a host-staged exchange
    backend = os.environ.get("PSF_DIST_BACKEND", "nccl")
    if os.environ.get("PSF_SAME_GPU") == "1":
        local = 0
    torch.cuda.set_device(local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        else:
            dist.init_process_group(backend)

    from parameter_server_amd import COMPRESSING, FIXING_FLOAT, KEY_CACHING
    from parameter_server_amd import filter as F

    n, nb = args.n, args.nb
    dev = f"cuda:{local}"
    g = torch.Generator(device=dev)
    g.manual_seed(1 + rank)
    ctx = F.Context(local)
    worker, server = F.RemoteNode(ctx), F.RemoteNode(ctx)
    F.set_clock(12345)  # FIXING_FLOAT seed (time(NULL) in the reference)
    tmpls = []
    router = None
    streams_batch = None
    if args.config == "c1":
        # async SGD pushes (async_sgd.h:264-296): every minibatch stream pushes
        # its ~10^5 keys with gradients, [KEY_CACHING, FIXING_FLOAT nb=1]
        m = args.m or 100_000
        nstreams = args.streams
        for sid in range(nstreams):
            keys = torch.unique(torch.randint(0, 10**9, (m + m // 8,), device=dev, generator=g))[:m]
            t = F.Message(request=True, push=True, key_channel=sid, key_range=(0, 10**9))
            t.set_key(torch.sort(keys)[0])
            t.add_value(torch.randn(m, device=dev, generator=g, dtype=torch.float32))
            t.add_filter(KEY_CACHING)
            t.add_filter(FIXING_FLOAT, num_bytes=nb)
            tmpls.append(t)
        streams_batch = ([F.RemoteNode(ctx) for _ in tmpls], [F.RemoteNode(ctx) for _ in tmpls])
        n = m * nstreams
        payload = 12 * n
    elif args.config == "c4":
        # stream s lives on rank s % N; every step slices,
        # encodes per destination server, spills and decodes (shard.PushRouter)
        from parameter_server_amd import shard
        m = args.m or (1 << 21)
        ex = shard.SpillExchange(device=dev) if world > 1 else None
        router = shard.PushRouter(ctx, shard.server_ranges(world), rank, world, ex)
        streams = {}
        nloc = 0
        for sid in range(rank, args.streams, world):
            keys = torch.from_numpy(splitmix64_keys(m, 4 + sid).view("int64")).to(dev)
            t = F.Message(request=True, push=True, key_channel=sid, key_range=shard.KEY_ALL)
            t.set_key(keys)
            t.add_value(torch.randn(keys.numel(), device=dev, generator=g, dtype=torch.float32))
            t.add_filter(KEY_CACHING)
            t.add_filter(FIXING_FLOAT, num_bytes=nb)
            streams[sid] = t
            nloc += keys.numel()
        n = nloc
        payload = 12 * nloc  # this rank's streams: 8 key + 4 value bytes per key
    elif args.config == "c2":
        # this rank's shard of the key range (range.h:100-107 EvenDivide),
        # pre-placed.  Consecutive steps use different messages (args.bufs
        # distinct arrays whose total exceeds the 256 MiB Infinity Cache), so no
        # step reads data a previous step left on chip.
        xs = [torch.randn(n, device=dev, generator=g, dtype=torch.float32) for _ in range(args.bufs)]
        for x in xs:
            t = F.Message(request=True, push=True, key_channel=0)
            t.add_value(x)
            t.add_filter(FIXING_FLOAT, num_bytes=nb)
            tmpls.append(t)
        payload = 4 * n  # key bytes 0 (dense values), value bytes 4n
    elif args.config == "c5":
        m = args.m or (1 << 20)
        keys = torch.from_numpy(splitmix64_keys(m, 4 + rank).view("int64")).to(dev)
        m = keys.numel()
        n = m * 128
        xs = [torch.randn(n, device=dev, generator=g, dtype=torch.float32) for _ in range(args.bufs)]
        for x in xs:
            t = F.Message(request=True, push=True, key_channel=0)
            t.set_key(keys)
            t.add_value(x)
            t.add_filter(KEY_CACHING)
            t.add_filter(FIXING_FLOAT, num_bytes=nb)
            if args.compress:
                t.add_filter(COMPRESSING)
            tmpls.append(t)
        payload = 8 * m + 4 * n
    else:
        # C3: m sorted unique keys sampled without replacement from [0, 1e9)
        # (SURVEY.md §8(d)), one f32 value per key; the worker's push stream
        # repeats the key set (KEY_CACHING hit) or clears it after every
        # send (c3miss: clear_cache_if_done on push, key_caching.h:30-33)
        m = args.m or 10_000_000
        keys = torch.unique(torch.randint(0, 10**9, (m + m // 8,), device=dev, generator=g))
        keys = torch.sort(keys[torch.randperm(keys.numel(), device=dev, generator=g)[:m]])[0]
        assert keys.numel() == m
        n = m
        xs = [torch.randn(m, device=dev, generator=g, dtype=torch.float32) for _ in range(args.bufs)]
        for x in xs:
            t = F.Message(request=True, push=True, key_channel=0, key_range=(0, 10**9))
            t.set_key(keys)
            t.add_value(x)
            t.add_filter(KEY_CACHING, clear_cache_if_done=(args.config == "c3miss"))
            t.add_filter(FIXING_FLOAT, num_bytes=nb)
            tmpls.append(t)
        payload = 12 * m  # 8m key bytes + 4m value bytes
    tmpl = tmpls

    def run(k):
        if router is not None:
            for _ in range(k):
                router.step(streams)
        elif streams_batch is not None:
            F.RemoteNode.roundtrip_many(streams_batch[0], streams_batch[1], tmpl, k)
        else:
            worker.roundtrip(server, tmpl, k)

    run(args.warmup)
    torch.cuda.synchronize()

    # diagnostic pass (not timed): every kernel bracketed by HIP events, to
    # find the dominant kernel and report the per-kernel breakdown
    diag = {}
    if not args.no_profile:
        ctx.profile(True)
        ctx.profile_reset()
        run(min(args.steps, 20))
        torch.cuda.synchronize()
        diag = ctx.profile_read()
        ctx.profile(False)
    dom = max(diag, key=lambda k: diag[k][1]) if diag else None

    # timed region: events only around the dominant kernel (live roofline);
    # in the many-small-message configs only every 8th launch of it, so the
    # event pairs do not dominate a step of short kernels
    stride = 8 if args.config in ("c1", "c4") else 1
    if dom:
        ctx.profile(True, kernels=[dom], stride=stride)
    ctx.profile_reset()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(args.steps)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    prof = ctx.profile_read()
    ctx.profile(False)

    if world > 1:
        t = torch.tensor([elapsed], device=f"cuda:{local}" if backend == "nccl" else "cpu", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    value = world * args.steps * payload / elapsed / GIB

    roofline = None
    if dom and dom in prof:
        launches, ms, alg = prof[dom]
        per_launch_bytes = alg / launches
        avg_s = ms / launches / 1e3
        achieved = per_launch_bytes / avg_s / 1e9
        traffic = pmc_traffic(dom, n, nb, args.config)
        roofline = {
            "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "kernel": dom,
            "avg_us": round(avg_s * 1e6, 2),
            "alg_bytes_per_launch": int(per_launch_bytes),
            "launches_timed": launches,
            "launch_sample_stride": stride,
            # breakdown from the separate diagnostic pass (all kernels evented)
            "kernels": {k: {"launches": v[0], "avg_us": round(v[1] / v[0] * 1e3, 2),
                            "alg_bytes_per_launch": int(v[2] / v[0]),
                            "GBps": round(v[2] / v[0] / (v[1] / v[0] / 1e3) / 1e9, 1)}
                        for k, v in diag.items()},
        }

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.config not in ("c1", "c4", "c5"):
        cpu = cpu_baseline(1 << 24 if args.config == "c2" else 1 << 22, nb, args.cpu_seconds, args.config)

    if rank == 0:
        line = {
            "metric": "GiB/s key-value payload through filter encode+decode, device-resident",
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong" if args.config == "c4" else "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic: f32 N(0,1) values, seed 1+rank, FIXING_FLOAT LCG seed 12345"
                    + {"c2": "", "c5": "; sorted unique uint64 keys splitmix64(4+rank+i)",
                       "c4": "; sorted unique uint64 keys splitmix64(4+stream+i)",
                       "c1": "; sorted unique uint64 keys from [0,1e9) per stream"}.get(
                        args.config, "; sorted unique uint64 keys from [0,1e9)"),
            "config": {
                "workload": WORKLOADS[args.config].format(nb=nb, cmp=", COMPRESSING" if args.compress else "",
                                                          streams=args.streams,
                                                          m=args.m or (100_000 if args.config == "c1" else 1 << 21)),
                "n_values_per_gpu": n,
                "payload_bytes_per_step_per_gpu": payload,
                "value_type": "float32",
                "num_bytes": nb,
                "parallelism": f"server key-range shards x{world} (EvenDivide), " + (
                    "cross-range spill: one all-to-all-v per step" if args.config == "c4" and world > 1
                    else "no data-path collective"),
            },
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)

    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
