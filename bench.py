#!/usr/bin/env python3
"""bench.py -- BASELINE.json metric: GiB/s of key-value payload through the
filter encode+decode chain, device-resident, on MI355X.

Default workload (BASELINE.json north_star target; SURVEY.md §8(d) C2 at the
north-star size): one message per step carrying n = 2^28 dense float32 values
(1 GiB, N(0,1), seed 1) and the chain [FIXING_FLOAT num_bytes=1] with min/max
computed; a step encodes it on the worker's RemoteNode, delivers it and
decodes it on the server's (libpsf psf_node_roundtrip: no Python per message).
Payload = 4n bytes/step.  The same run also measures BASELINE configs[1]'s
128M values (2^27) and reports it under "config_128M".

N GPUs: rank g is server g of EvenDivide(N, g) and codes its own pre-placed
shard (no data-path collective; weak scaling).  `python bench.py --gpus N`
starts the N rank processes itself (from a parent that makes no GPU call)
unless WORLD_SIZE is already set (torchrun).  Timed region: barrier +
synchronize, K steps, barrier + synchronize; the max elapsed over ranks is the
job time.  value = N * K * payload / time.

Other configs (--config): c1 (ctr push streams, batched), c3 / c3miss (10M
keys @1% + values, KEY_CACHING hit / miss), c4 (64 push streams over 8 server
key ranges, cross-range spill in one all-to-all-v per step), c5 (embedding
rows dim 128 sliced over 8 servers, [KEY_CACHING, FIXING_FLOAT(, COMPRESSING)]).

roofline: per-kernel durations from HIP events recorded on the launch stream
around the dominant kernel inside the timed region (libpsf profiler); its
algorithmic bytes / average duration vs 8 TB/s.  traffic: PMC-derived HBM bytes
per launch from profiles/pmc_traffic.json when it matches this kernel and
size (tools/pmc_traffic.py), else null.
cpu_baseline: the C restatement of the reference's filter code (oracle/,
"port") on the host cores of the same box, rank 0 at N=1 only, over a bounded
sample of the same workload: one core where the reference's filters run
serialised (C1-C3), one thread per stream / slice up to 16 for C4 / C5
(SURVEY.md §8(d)).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

GIB = float(1 << 30)
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, MI355X_MICROARCH.md
CPU_THREADS_MAX = 16   # the GPU box's CPU share per GPU


WORKLOADS = {
    "c2": "C2 (BASELINE configs[1] chain at the north-star size): dense f32 values, chain "
          "[FIXING_FLOAT num_bytes={nb}], min/max computed, encode+decode round trip per step",
    "c3": "C3 (BASELINE configs[2]): 10M uint64 keys @1% of [0,1e9) + f32 values, chain "
          "[KEY_CACHING, FIXING_FLOAT num_bytes={nb}], repeat send (key cache hit: keys elided)",
    "c3miss": "C3 (BASELINE configs[2]) first-send path: 10M uint64 keys @1% of [0,1e9) + f32 "
              "values, chain [KEY_CACHING(clear_cache_if_done), FIXING_FLOAT num_bytes={nb}], "
              "every send a key cache miss",
    "c4": "C4 (BASELINE configs[3]): {streams} push streams in total (stream s on rank s % N), each "
          "{m} sorted unique uint64 keys spread over 2^64 (splitmix64) + f32 values, sliced at the "
          "EvenDivide({servers}) server ranges (servers in contiguous blocks per rank), "
          "per-(stream, server) [KEY_CACHING, FIXING_FLOAT num_bytes={nb}], cross-range slices spilled in "
          "one all-to-all-v per step (RCCL), {sends}",
    "c1": "C1 (BASELINE configs[0]) on the device: the ctr example's minibatch "
          "(example/linear/ctr/online_l1lr.conf:36-53) for {streams} concurrent streams of {m} sorted unique "
          "keys: pull request (keys, [KEY_CACHING, FIXING_FLOAT num_bytes={nb}]), pull response (keys elided "
          "+ f32 weights), push (keys elided + f32 gradients, [KEY_CACHING(clear_cache_if_done), "
          "FIXING_FLOAT num_bytes={nb}]), each batched over the streams",
    "c4pull": "C4's partition on the pull side (SURVEY.md CS-2, §8(e)): {streams} pull request streams in total "
              "(stream s on rank s % N), each {m} sorted unique uint64 keys spread over 2^64 (splitmix64), sliced "
              "at the EvenDivide({servers}) server ranges, per-(stream, server) [KEY_CACHING, FIXING_FLOAT "
              "num_bytes={nb}]; each server answers its slices from its KVMap (GetValue), encodes the response "
              "(keys elided on the cache hit, min/max per slice), the requester decodes it into the stream's "
              "key-ordered array; repeat pulls (key cache hit)",
    "c5": "C5 (BASELINE configs[4]) per GPU: one stream of {m} uint64 keys spread over 2^64 "
          "(splitmix64) + embedding rows dim=128 f32, sliced at the EvenDivide({servers}) server ranges "
          "(k = 128 values per key), per-(stream, server) [KEY_CACHING, FIXING_FLOAT num_bytes={nb}{cmp}], "
          "cross-range slices spilled in one all-to-all-v per step, {sends}",
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


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--no-host-floor", action="store_true",
                    help="c4 / c5: skip the host-cost run (the same step with 4096 keys per stream)")
    ap.add_argument("--steps", type=int, default=None,
                    help="timed steps (default 20; 200 for c1 / c3, whose step is 0.04-0.07 ms: 20 of them "
                         "time only about 1 ms)")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--n", type=int, default=1 << 28, help="c2: values per message (per GPU)")
    ap.add_argument("--nb", type=int, default=1, help="FIXING_FLOAT num_bytes")
    ap.add_argument("--bufs", type=int, default=3, help="distinct messages cycled through")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--prof-stride", type=int, default=0,
                    help="time every k-th launch of the dominant kernel in the timed region (0: the config's default)")
    ap.add_argument("--no-128m", action="store_true", help="c2: skip the configs[1] 2^27 measurement")
    ap.add_argument("--no-c4", action="store_true",
                    help="c2: skip the companion C4 measurement (cross-range spill) reported as config_c4")
    ap.add_argument("--c4-m", type=int, default=1 << 21, help="c2's companion C4 line: keys per stream")
    ap.add_argument("--streams", type=int, default=64, help="c1/c4: push streams in total")
    ap.add_argument("--servers", type=int, default=8, help="c4/c5: server key ranges (>= N)")
    ap.add_argument("--config", default="c2", choices=["c1", "c2", "c3", "c3miss", "c4", "c4pull", "c5"])
    ap.add_argument("--m", type=int, default=None, help="keys per message (c1 1e5, c3 10M, c4 2^21, c5 2^20)")
    ap.add_argument("--compress", action="store_true", help="append COMPRESSING to the chain (c5)")
    ap.add_argument("--miss", action="store_true",
                    help="c4/c5: KEY_CACHING(clear_cache_if_done): every send a key cache miss (keys travel, "
                         "and are compressed with --compress)")
    ap.add_argument("--launch-check", action="store_true",
                    help="start the ranks and the process group only (no GPU work); for CPU tests")
    a = ap.parse_args(argv)
    if a.steps is None:
        a.steps = 200 if a.config in ("c1", "c3", "c3miss") else 20
    return a


# --------------------------------------------------------------- launcher --
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch(args) -> int:
    """Start args.gpus rank processes (one per GPU), the way torchrun would;
    this parent never touches the GPU.  Returns the worst exit code."""
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rcs = [p.wait() for p in procs]
    bad = [rc for rc in rcs if rc != 0]
    return bad[0] if bad else 0


# ----------------------------------------------------------- CPU baseline --
def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _run_tasks(tasks, threads: int, seconds: float):
    """Run the list of task callables (one step of the sample) repeatedly on
    `threads` host threads until `seconds` of wall time; returns (reps, t)."""
    from concurrent.futures import ThreadPoolExecutor
    reps, t = 0, 0.0
    with ThreadPoolExecutor(max_workers=threads) as ex:
        while t < seconds or reps == 0:
            t0 = time.perf_counter()
            list(ex.map(lambda f: f(), tasks))
            t += time.perf_counter() - t0
            reps += 1
    return reps, t


def cpu_baseline(args, nb: int):
    """The C restatement of the reference's filters (oracle/psf_port.c) on
    host cores, over a bounded sample of the configured workload."""
    import numpy as np

    import oracle
    P = oracle.Port()
    rng = np.random.default_rng(1)
    cfg, seed = args.config, 12345
    tasks, payload, threads, what = [], 0, 1, ""

    def ff_rt(x):
        def f():
            st, codes, mn, mx = P.ff_encode(x, nb, seed)
            if args.compress:
                c = P.snappy_compress(codes)
                P.snappy_uncompress(c, cap=codes.size + 64)
            P.ff_decode(codes, nb, mn, mx)
        return f

    def kc_ff(keys, x, decode_crc):
        rt = ff_rt(x)

        def f():
            P.key_signature(keys)   # KEY_CACHING encode: CRC of the first <= 2 KiB
            if decode_crc:
                P.key_signature(keys)  # decode checks the CRC when keys travel
                if args.compress:  # a miss: the keys travel, snappy-compressed
                    c = P.snappy_compress(keys.view(np.uint8))
                    P.snappy_uncompress(c, cap=keys.nbytes + 64)
            rt()
        return f

    if cfg == "c2":
        # the line's own size: one message of args.n f32 values (2^28 = 1 GiB)
        x = rng.standard_normal(args.n, dtype=np.float32)
        tasks, payload = [ff_rt(x)], x.nbytes
        what = f"FIXING_FLOAT(nb={nb}) encode+decode of {args.n} f32 ({x.nbytes >> 20} MiB, the line's size)"
    elif cfg in ("c3", "c3miss"):
        m = 1 << 22
        keys = np.unique(np.random.default_rng(3).integers(0, 10**9, m + m // 8, dtype=np.uint64))[:m]
        x = rng.standard_normal(keys.size).astype(np.float32)
        tasks, payload = [kc_ff(keys, x, cfg == "c3miss")], keys.nbytes + x.nbytes
        what = f"KEY_CACHING+FIXING_FLOAT(nb={nb}) of 2^22 keys from [0,1e9) + f32"
    elif cfg == "c1":
        m = args.m or 100_000
        ns = args.streams
        for s in range(ns):
            keys = np.unique(np.random.default_rng(100 + s).integers(0, 10**9, m + m // 8, dtype=np.uint64))[:m]
            w = rng.standard_normal(keys.size).astype(np.float32)
            x = rng.standard_normal(keys.size).astype(np.float32)
            sig = lambda k=keys: P.key_signature(k)  # noqa: E731
            # pull request: CRC on encode and on decode (keys travel); pull
            # response and push: CRC on encode (hit, keys elided) + FF round trip
            tasks += [sig, sig, kc_ff(keys, w, False), kc_ff(keys, x, False)]
            payload += 8 * keys.size + 2 * (keys.nbytes + x.nbytes)
        what = (f"{ns} ctr minibatches (pull request, pull response, push; [KEY_CACHING, "
                f"FIXING_FLOAT(nb={nb})]) of {m} keys + f32, one core (the reference's filters run "
                f"serialised per Customer)")
    elif cfg == "c4pull":
        # per slice: the request's CRC, the server's GetValue (a lookup per key
        # in a sorted key table, numpy), the response's CRC and FIXING_FLOAT
        # round trip (keys elided: a cache hit on both sides)
        from parameter_server_amd import shard
        ranges = shard.server_ranges(args.servers)
        bounds = np.array([r[0] for r in ranges] + [ranges[-1][1]], dtype=np.uint64)
        m = args.m or (1 << 21)
        nstreams = min(args.streams, CPU_THREADS_MAX)
        tk = np.unique(np.concatenate([splitmix64_keys(m, 4 + s) for s in range(nstreams)]))
        tw = rng.standard_normal(tk.size).astype(np.float32)

        def pull_slice(keys):
            def f():
                P.key_signature(keys)  # request encode (hit)
                w = tw[np.searchsorted(tk, keys)]  # KVMap::GetValue
                P.key_signature(keys)  # response encode (hit)
                ff_rt(w)()
            return f
        for s in range(nstreams):
            keys = splitmix64_keys(m, 4 + s)
            pos = np.searchsorted(keys, bounds)
            for d in range(args.servers):
                lo, hi = int(pos[d]), int(pos[d + 1])
                if hi > lo:
                    tasks.append(pull_slice(keys[lo:hi]))
            payload += 20 * keys.size
        what = (f"{nstreams} pull stream(s) of {m} keys sliced over {args.servers} servers: request CRC, "
                f"GetValue (sorted-table lookup), response CRC + FIXING_FLOAT(nb={nb}) round trip per slice")
    else:  # c4 / c5: the per-(stream, server) slices, one thread per slice up to 16
        from parameter_server_amd import shard
        ranges = shard.server_ranges(args.servers)
        bounds = np.array([r[0] for r in ranges] + [ranges[-1][1]], dtype=np.uint64)
        if cfg == "c4":
            m, dim = args.m or (1 << 21), 1
            nstreams = min(args.streams, CPU_THREADS_MAX)
        else:
            m, dim = min(args.m or (1 << 20), 1 << 18), 128
            nstreams = 1
        for s in range(nstreams):
            keys = splitmix64_keys(m, 4 + s)
            x = rng.standard_normal(keys.size * dim).astype(np.float32)
            pos = np.searchsorted(keys, bounds)
            for d in range(args.servers):
                lo, hi = int(pos[d]), int(pos[d + 1])
                if hi > lo:
                    tasks.append(kc_ff(keys[lo:hi], x[lo * dim:hi * dim], args.miss))
            payload += keys.nbytes + x.nbytes
        what = (f"{nstreams} stream(s) of {m} keys (dim {dim}) sliced over {args.servers} servers, "
                f"[KEY_CACHING, FIXING_FLOAT(nb={nb}){', COMPRESSING' if args.compress else ''}] per slice")
    if cfg in ("c4", "c4pull", "c5"):
        try:
            avail = len(os.sched_getaffinity(0))
        except AttributeError:
            avail = os.cpu_count() or 1
        threads = max(1, min(len(tasks), CPU_THREADS_MAX, avail))
    reps, t = _run_tasks(tasks, threads, args.cpu_seconds)
    return {
        "value": round(reps * payload / t / GIB, 4),
        "unit": "GiB/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{reps} x {what}, {threads} thread(s), {t:.1f} s",
        "cpu_model": _cpu_model(),
        "nproc": os.cpu_count(),
    }


def line_key(args):
    """The name tools/pmc_traffic.py gives this run's line, when it runs at the
    line's default sizes (the PMC passes' shape), else None."""
    if args.nb != 1 or args.miss:
        return None
    c = args.config
    if c == "c2":
        return "c2" if args.n == 1 << 28 else None
    if c == "c1":
        return "c1" if args.m in (None, 100_000) and args.streams == 64 else None
    if c == "c3":
        return "c3" if args.m in (None, 10_000_000) else None
    if c in ("c4", "c4pull"):
        return c if args.m in (None, 1 << 21) and args.streams == 64 and args.servers == 8 else None
    if c == "c5":
        return ("c5z" if args.compress else "c5") if args.m in (None, 1 << 20) and args.servers == 8 else None
    return None


def pmc_traffic(kernel: str, args):
    """HBM bytes per launch of `kernel` on this line, from the PMC passes in
    profiles/pmc_traffic.json (tools/pmc_traffic.py), or None."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    key = line_key(args)
    try:
        d = json.load(open(path))
    except (OSError, ValueError):
        return None
    e = d.get("lines", {}).get(key or "", {}).get("kernels", {}).get(kernel)
    return e.get("hbm_bytes_per_launch") if e else None


# ------------------------------------------------------------- workloads --
def c4_args(args):
    """the C4 companion measurement of a c2 run: 64 streams, EvenDivide(8)
    (the default --streams / --servers), repeat sends"""
    a4 = argparse.Namespace(**vars(args))
    a4.config, a4.m, a4.compress, a4.miss = "c4", args.c4_m, False, False
    return a4


def c4_config(args, world_pg: int, backend_pg: str) -> dict:
    a4 = c4_args(args)
    return {"workload": WORKLOADS["c4"].format(nb=args.nb, streams=a4.streams, servers=a4.servers, m=a4.m,
                                               sends="repeat sends (key cache hit)", cmp=""),
            "scaling": "strong" if world_pg > 1 else "weak",
            "world_size": world_pg, "backend": backend_pg,
            "parallelism": f"{a4.servers} servers in blocks over {world_pg} rank(s); "
                           + ("cross-range slices in one all-to-all-v per step" if world_pg > 1
                              else "every slice local (no exchange at world 1)"),
            "measured": False}


def build_workload(args, F, ctx, rank, world, dev, g, n):
    """Returns (run(k), payload bytes per step on this rank, n values, extra)."""
    import torch

    from parameter_server_amd import COMPRESSING, FIXING_FLOAT, KEY_CACHING
    nb = args.nb
    if args.config == "c1":
        # the ctr example's async SGD minibatch (async_sgd.h:229-296, CS-1/CS-2
        # of SURVEY.md): per stream and step a pull request (keys,
        # pull_filter [KEY_CACHING, FIXING_FLOAT nb=1]), the server's pull
        # response (keys elided on the cache hit + weights) and the push
        # (keys elided + gradients, push_filter [KEY_CACHING(clear_cache_if_done),
        # FIXING_FLOAT nb=1]); each of the three runs batched over all streams
        m = args.m or 100_000
        S = args.streams
        wk = [F.RemoteNode(ctx) for _ in range(S)]  # worker's node for its server
        sv = [F.RemoteNode(ctx) for _ in range(S)]  # server's node for the worker
        req, resp, push = [], [], []
        for sid in range(S):
            keys = torch.sort(torch.unique(torch.randint(0, 10**9, (m + m // 8,), device=dev, generator=g))[:m])[0]
            for lst, request, is_push, vals, clear in ((req, True, False, False, None),
                                                       (resp, False, False, True, None),
                                                       (push, True, True, True, True)):
                t = F.Message(request=request, push=is_push, key_channel=sid, key_range=(0, 10**9))
                t.set_key(keys)
                if vals:
                    t.add_value(torch.randn(m, device=dev, generator=g, dtype=torch.float32))
                t.add_filter(KEY_CACHING, clear_cache_if_done=clear)
                t.add_filter(FIXING_FLOAT, num_bytes=nb)
                lst.append(t)
        tmpls, snd, rcv = req + resp + push, wk + sv + wk, sv + wk + sv

        def run(k, wire=False):
            F.RemoteNode.roundtrip_many(snd, rcv, tmpls, k, phase_end=[S, 2 * S, 3 * S], wire=wire)
        # keys travel with the pull request only; the response and the push hit
        return run, 32 * m * S, 2 * m * S, {"key_bytes_elided": 16 * m * S, "wire": True}
    if args.config == "c4pull":
        # the pull leg over C4's partition: requests out, per-range responses
        # answered from each rank's KVMap, merged back in key order
        import numpy as np

        from parameter_server_amd import shard
        if args.servers < world:
            raise SystemExit(f"--servers {args.servers} < {world} ranks")
        ex = None
        if world > 1:
            same = os.environ.get("PSF_SAME_GPU") == "1" or not str(dev).startswith("cuda")
            ex = shard.NativeExchange.create(ctx, transport="host" if same else "rccl")
        ranges = shard.server_ranges(args.servers)
        router = shard.PushRouter(ctx, ranges, rank, world, ex)
        m = args.m or (1 << 21)
        sids = list(range(rank, args.streams, world))
        allk = np.unique(np.concatenate([splitmix64_keys(m, 4 + s) for s in range(args.streams)]))
        mine = [d for d in range(args.servers) if router.owner(d) == rank]
        lo, hi = ranges[mine[0]][0], ranges[mine[-1]][1]
        own = allk[(allk >= np.uint64(lo)) & ((allk < np.uint64(hi)) | (np.uint64(hi) == np.uint64(0)))]
        kv = F.KVMap(ctx, capacity=max(1024, 2 * own.size))
        if own.size:
            kt = torch.from_numpy(own.view("int64")).to(dev)
            kv.push(kt, torch.randn(own.size, device=dev, generator=g, dtype=torch.float32))
        router.set_store(kv)
        reqs, payload = {}, 0
        for sid in sids:
            keys = torch.from_numpy(splitmix64_keys(m, 4 + sid).view("int64")).to(dev)
            t = F.Message(request=True, push=False, key_channel=sid, key_range=shard.KEY_ALL)
            t.set_key(keys)
            t.add_filter(KEY_CACHING)
            t.add_filter(FIXING_FLOAT, num_bytes=nb)
            reqs[sid] = t
            payload += 20 * keys.numel()  # request keys 8 B + response keys 8 B and value 4 B per key
        nloc = payload // 20

        def run(k):
            router.pull(reqs, k)
        # keys travel with the first pull only; later requests and every response hit
        return run, payload, nloc, {"router": router, "key_bytes_elided": 16 * nloc, "store": kv}
    if args.config in ("c4", "c5"):
        # streams sliced at the server ranges, encoded
        # per destination server, spilled (one all-to-all-v) and decoded
        from parameter_server_amd import shard
        if args.servers < world:
            raise SystemExit(f"--servers {args.servers} < {world} ranks")
        ex = None
        if world > 1:
            # libpsf's exchange (one native call per timed region, no device
            # read-back per step): RCCL over xGMI under the driver's nccl
            # backend, the host mailbox when ranks share a GPU (rehearsals);
            # PSF_EXCHANGE=python: torch's all-to-all-v, one Python step each
            mode = os.environ.get("PSF_EXCHANGE", "native")
            if mode == "python":
                ex = shard.SpillExchange(ctx, device=dev)
            else:
                same = os.environ.get("PSF_SAME_GPU") == "1" or not str(dev).startswith("cuda")
                ex = shard.NativeExchange.create(ctx, transport="host" if same else "rccl")
        router = shard.PushRouter(ctx, shard.server_ranges(args.servers), rank, world, ex)
        streams, nloc, payload, elided = {}, 0, 0, 0
        if args.config == "c4":
            m, dim, sids = args.m or (1 << 21), 1, range(rank, args.streams, world)
        else:
            m, dim, sids = args.m or (1 << 20), 128, [rank]
        for sid in sids:
            keys = torch.from_numpy(splitmix64_keys(m, 4 + sid).view("int64")).to(dev)
            t = F.Message(request=True, push=True, key_channel=sid, key_range=shard.KEY_ALL)
            t.set_key(keys)
            t.add_value(torch.randn(keys.numel() * dim, device=dev, generator=g, dtype=torch.float32))
            t.add_filter(KEY_CACHING, clear_cache_if_done=True if args.miss else None)
            t.add_filter(FIXING_FLOAT, num_bytes=nb)
            if args.compress:
                t.add_filter(COMPRESSING)
            streams[sid] = t
            nloc += keys.numel() * dim
            payload += keys.numel() * (8 + 4 * dim)
            elided += 0 if args.miss else 8 * keys.numel()

        def run(k):
            router.run(streams, k)
        return run, payload, nloc, {"router": router, "key_bytes_elided": elided}
    worker, server = F.RemoteNode(ctx), F.RemoteNode(ctx)
    tmpls = []
    if args.config == "c2":
        # this rank's shard of the key range (range.h:100-107 EvenDivide),
        # pre-placed.  Consecutive steps use different messages (args.bufs
        # distinct arrays whose total exceeds the 256 MiB Infinity Cache), so no
        # step reads data a previous step left on chip.
        for _ in range(args.bufs):
            t = F.Message(request=True, push=True, key_channel=0)
            t.add_value(torch.randn(n, device=dev, generator=g, dtype=torch.float32))
            t.add_filter(FIXING_FLOAT, num_bytes=nb)
            tmpls.append(t)
        payload = 4 * n  # key bytes 0 (dense values), value bytes 4n
    else:
        # C3: m sorted unique keys sampled without replacement from [0, 1e9)
        # (SURVEY.md §8(d)), one f32 value per key; the worker's push stream
        # repeats the key set (KEY_CACHING hit) or clears it after every
        # send (c3miss: clear_cache_if_done on push, key_caching.h:30-33)
        m = args.m or 10_000_000
        keys = torch.unique(torch.randint(0, 10**9, (m + m // 8,), device=dev, generator=g))
        keys = torch.sort(keys[torch.randperm(keys.numel(), device=dev, generator=g)[:m]])[0]
        n = m
        for _ in range(args.bufs):
            t = F.Message(request=True, push=True, key_channel=0, key_range=(0, 10**9))
            t.set_key(keys)
            t.add_value(torch.randn(m, device=dev, generator=g, dtype=torch.float32))
            t.add_filter(KEY_CACHING, clear_cache_if_done=(args.config == "c3miss"))
            t.add_filter(FIXING_FLOAT, num_bytes=nb)
            tmpls.append(t)
        payload = 12 * m

    def run(k):
        worker.roundtrip(server, tmpls, k)
    return run, payload, n, {"key_bytes_elided": 8 * m if args.config == "c3" else 0}


def timed(run, steps, world, dist, ctx, prof_kernel=None, stride=1):
    import torch
    if prof_kernel:
        ctx.profile(True, kernels=[prof_kernel], stride=stride)
    ctx.profile_reset()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ctx.host_waits(reset=True)
    t0 = time.perf_counter()
    run(steps)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    prof = ctx.profile_read()
    ctx.profile(False)
    return elapsed, prof


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch(args))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")

    import torch
    import torch.distributed as dist

    # rehearsal knobs (never set by the driver): PSF_DIST_BACKEND=gloo and
    # PSF_SAME_GPU=1 run N ranks on one GPU with a host-staged exchange
    backend = os.environ.get("PSF_DIST_BACKEND", "nccl")
    if os.environ.get("PSF_SAME_GPU") == "1":
        local = 0
    if not args.launch_check:
        torch.cuda.set_device(local)
    if world > 1:
        # bounded collectives: a rank that fails mid-run is an error on the
        # others, not a hang
        import datetime
        tmo = datetime.timedelta(seconds=300)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"), timeout=tmo)
        else:
            dist.init_process_group(backend, timeout=tmo)
        if dist.get_world_size() != args.gpus:
            raise SystemExit(f"bench.py: process group has {dist.get_world_size()} ranks, --gpus {args.gpus}")
    world_pg = dist.get_world_size() if world > 1 else 1
    backend_pg = dist.get_backend() if world > 1 else "none"

    if args.launch_check:  # plumbing only: process group, barrier, max-reduce, one JSON line
        if world > 1:
            t = torch.tensor([float(rank)], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dist.barrier()
        if rank == 0:
            line = {"launch_check": True, "n_gpus": world_pg, "world_size": world_pg,
                    "backend": backend_pg, "config": {"workload": args.config}}
            if args.config == "c2" and not args.no_c4:  # the companion line a real run adds (not measured here)
                line["config_c4"] = c4_config(args, world_pg, backend_pg)
            print(json.dumps(line), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return

    from parameter_server_amd import filter as F

    n, nb = args.n, args.nb
    dev = f"cuda:{local}"
    g = torch.Generator(device=dev)
    g.manual_seed(1 + rank)
    ctx = F.Context(local)
    F.set_clock(12345)  # FIXING_FLOAT seed (time(NULL) in the reference)
    run, payload, n, extra = build_workload(args, F, ctx, rank, world, dev, g, n)

    run(args.warmup)
    torch.cuda.synchronize()

    # diagnostic pass (not timed): every kernel bracketed by HIP events, to
    # find the dominant kernel and report the per-kernel breakdown
    diag = {}
    if not args.no_profile:
        ctx.profile(True)
        ctx.profile_reset()
        run(min(args.steps, 10))
        torch.cuda.synchronize()
        diag = ctx.profile_read()
        ctx.profile(False)
    dom = max(diag, key=lambda k: diag[k][1]) if diag else None

    # timed region: events only around the dominant kernel (live roofline),
    # on every 4th launch of it (every 8th in the many-small-message configs):
    # a launch with start / stop events costs the stream a few us around the
    # kernel (stride 1 against 4, tools/ab_stride.sh r05o: C3 3272 -> 3324,
    # C5 1684 -> 1701, C5 + COMPRESSING 1383 -> 1391 GiB/s; C2 equal)
    stride = args.prof_stride or (8 if args.config in ("c1", "c4", "c4pull") else 4)
    router = extra.get("router")
    if router is not None and router.exchange is not None:
        router.exchange.bytes_sent = 0
    if router is not None:
        router.host_stats(reset=True)
    elapsed, prof = timed(run, args.steps, world, dist, ctx, dom, stride)
    waits = ctx.host_waits()
    spill = router.exchange.bytes_sent if router is not None and router.exchange is not None else 0
    # host accounting of the timed steps (this rank): wall time, the part the
    # host spent blocked on the device, the rest (host work), and the kernel
    # time per step from the diagnostic pass
    host = None
    if diag:
        blocked = sum(v[0] for v in waits.values())
        kern_ms = sum(v[1] for v in diag.values()) / min(args.steps, 10)
        host = {"wall_ms_per_step": round(elapsed / args.steps * 1e3, 4),
                "blocked_ms_per_step": round(blocked / args.steps * 1e3, 4),
                "active_ms_per_step": round((elapsed - blocked) / args.steps * 1e3, 4),
                "kernel_ms_per_step": round(kern_ms, 4),
                "waits": {k: {"ms_per_step": round(v[0] / args.steps * 1e3, 4), "per_step": v[1] / args.steps}
                          for k, v in waits.items()}}
        if router is not None:
            rs = router.host_stats()
            host["router_encode_ms_per_step"] = round(rs["encode_s"] / args.steps * 1e3, 4)
            host["router_decode_ms_per_step"] = round(rs["decode_s"] / args.steps * 1e3, 4)
            # wall - blocked counts the time the host spends inside launch
            # calls while the device is behind (the launch queue is full) as
            # "active"; the host's own cost per step is measured apart: the
            # same streams and servers with 4096 keys each (every kernel a
            # few us), where the step is the host's
            if args.config in ("c4", "c4pull", "c5") and not args.no_host_floor:
                a_f = argparse.Namespace(**vars(args))
                a_f.m = 64 if args.config == "c5" else 4096
                run_f, _, _, extra_f = build_workload(a_f, F, ctx, rank, world, dev, g, 0)
                run_f(args.warmup)
                el_f, _ = timed(run_f, args.steps, world, dist, ctx)
                host["floor_ms_per_step"] = round(el_f / args.steps * 1e3, 4)
                host["floor_what"] = (f"the same {1 if args.config == 'c5' else args.streams} stream(s) x "
                                      f"{args.servers} servers with {a_f.m} keys per stream: the host's own "
                                      "cost of a step (slicing, per-slice Task / filter work, launches)")
                host["floor_over_kernel"] = round(host["floor_ms_per_step"] / kern_ms, 3) if kern_ms else None
                del run_f, extra_f

    def max_over_ranks(v):
        if world == 1:
            return v
        t = torch.tensor([v], device=dev if backend == "nccl" else "cpu", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    elapsed = max_over_ranks(elapsed)
    total_payload = payload
    if world > 1:
        t = torch.tensor([float(payload)], device=dev if backend == "nccl" else "cpu", dtype=torch.float64)
        dist.all_reduce(t)
        total_payload = float(t.item())
    value = args.steps * total_payload / elapsed / GIB

    roofline = None
    if dom and dom in prof:
        launches, ms, alg = prof[dom]
        per_launch_bytes = alg / launches
        avg_s = ms / launches / 1e3
        achieved = per_launch_bytes / avg_s / 1e9
        roofline = {
            "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": pmc_traffic(dom, args),
            "traffic_source": "profiles/pmc_traffic.json (rocprofv3 FETCH_SIZE / WRITE_SIZE passes of this line)"
                              if pmc_traffic(dom, args) else None,
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

    # BASELINE configs[1] (128M values) measured in the same run
    also = None
    if args.config == "c2" and not args.no_128m and n != (1 << 27):
        a2 = argparse.Namespace(**vars(args))
        a2.n = 1 << 27
        del run
        run2, payload2, _, _ = build_workload(a2, F, ctx, rank, world, dev, g, 1 << 27)
        run2(args.warmup)
        el2, _ = timed(run2, args.steps, world, dist, ctx)
        el2 = max_over_ranks(el2)
        also = {"n_values_per_gpu": 1 << 27, "value": round(world * args.steps * payload2 / el2 / GIB, 2),
                "ms_per_step": round(el2 / args.steps * 1e3, 4)}
        del run2

    # the C4 push path (BASELINE configs[3]) in the same process: at N > 1 its
    # cross-range slices travel by RCCL all-to-all-v, so a multi-GPU run of
    # the default command measures the spill too (executor.cc:134-146 over
    # assigner.h:17-28's partition); at N = 1 every slice is local
    c4 = None
    c4_failed = False
    if args.config == "c2" and not args.no_c4:
        if "run" in locals():
            del run
        try:
            a4 = c4_args(args)
            run4, payload4, _, extra4 = build_workload(a4, F, ctx, rank, world, dev, g, 0)
            run4(args.warmup)
            torch.cuda.synchronize()
            r4 = extra4["router"]
            if r4.exchange is not None:
                r4.exchange.bytes_sent = 0
            el4, _ = timed(run4, args.steps, world, dist, ctx)
            spill4 = r4.exchange.bytes_sent if r4.exchange is not None else 0
            el4 = max_over_ranks(el4)
            tot4 = float(payload4)
            if world > 1:
                t = torch.tensor([tot4], device=dev if backend == "nccl" else "cpu", dtype=torch.float64)
                dist.all_reduce(t)
                tot4 = float(t.item())
            c4 = c4_config(args, world_pg, backend_pg)
            c4.update({"measured": True, "value": round(args.steps * tot4 / el4 / GIB, 2),
                       "ms_per_step": round(el4 / args.steps * 1e3, 4),
                       "payload_bytes_per_step_per_gpu_rank0": payload4,
                       "key_bytes_elided_per_step_rank0": extra4["key_bytes_elided"],
                       "spill_bytes_per_step_rank0": spill4 // max(args.steps, 1)})
            del run4, r4, extra4
        except Exception as e:  # noqa: BLE001 -- the companion must not take the C2 line down with it
            c4_failed = True
            c4 = c4_config(args, world_pg, backend_pg)
            c4.update({"measured": False, "error": f"{type(e).__name__}: {e}"[:400]})
            print(f"bench.py: rank {rank}: config_c4 failed: {e!r}", file=sys.stderr, flush=True)
        if world > 1:
            # every rank learns whether any rank's companion failed (the
            # exchange's waits are bounded, so a failed rank's peers fail too
            # instead of hanging in it); the line then reports no C4 number
            flag = torch.tensor([1.0 if c4_failed else 0.0], device=dev if backend == "nccl" else "cpu",
                                dtype=torch.float64)
            dist.all_reduce(flag, op=dist.ReduceOp.MAX)
            if flag.item() > 0 and not c4_failed:
                c4_failed = True
                c4 = c4_config(args, world_pg, backend_pg)
                c4.update({"measured": False, "error": "config_c4 failed on another rank"})

    # C1 with the wire step in the timed region: every encoded Task serialised
    # (its computed min/max settled to the host) and parsed by the receiver,
    # as Van::Send / Recv do after EncodeMessage (van.cc:122-191, 244-269)
    wire_line = None
    if extra.get("wire"):
        run(args.warmup, wire=True)
        elw, _ = timed(lambda k: run(k, wire=True), args.steps, world, dist, ctx)
        elw = max_over_ranks(elw)
        wire_line = {"what": "each encoded Task serialised (min/max settled) and parsed by the receiver",
                     "value": round(world * args.steps * payload / elw / GIB, 2),
                     "ms_per_step": round(elw / args.steps * 1e3, 4)}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args, nb)

    if rank == 0:
        m_default = {"c1": 100_000, "c4": 1 << 21, "c4pull": 1 << 21, "c5": 1 << 20}.get(args.config, 1 << 21)
        line = {
            "metric": "GiB/s key-value payload through filter encode+decode, device-resident",
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world_pg,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            # C4's 64 streams are split over the ranks (total work fixed): strong
            # scaling once there is more than one rank
            "scaling": "strong" if args.config in ("c4", "c4pull") and world_pg > 1 else "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic: f32 N(0,1) values, seed 1+rank, FIXING_FLOAT LCG seed 12345"
                    + {"c2": "", "c5": "; sorted unique uint64 keys splitmix64(4+rank+i)",
                       "c4": "; sorted unique uint64 keys splitmix64(4+stream+i)",
                       "c4pull": "; sorted unique uint64 keys splitmix64(4+stream+i), KVMap weights one FTRL "
                                 "update of N(0,1) gradients",
                       "c1": "; sorted unique uint64 keys from [0,1e9) per stream"}.get(
                        args.config, "; sorted unique uint64 keys from [0,1e9)"),
            "config": {
                "workload": WORKLOADS[args.config].format(
                    nb=nb, cmp=", COMPRESSING" if args.compress else "", streams=args.streams,
                    servers=args.servers, m=args.m or m_default,
                    sends=("every send a key cache miss (KEY_CACHING clear_cache_if_done; keys travel"
                           + (", snappy-compressed)" if args.compress else ")")) if args.miss
                    else "repeat sends (key cache hit)"),
                "n_values_per_gpu": n,
                "payload_bytes_per_step_per_gpu": payload,
                "value_type": "float32",
                "num_bytes": nb,
                "world_size": world_pg,
                "backend": backend_pg,
                "parallelism": f"server key-range shards x{world} (EvenDivide), " + (
                    f"{args.servers} servers, cross-range spill: one all-to-all-v per step"
                    if args.config in ("c4", "c4pull", "c5") and world > 1 else "no data-path collective"),
            },
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        if host:
            line["host"] = host
        if "key_bytes_elided" in extra:
            # payload counts key bytes before encode; on a
            # KEY_CACHING hit they are elided, so these bytes move nowhere
            line["config"]["key_bytes_elided_per_step_per_gpu"] = extra["key_bytes_elided"]
        if spill:
            line["config"]["spill_bytes_per_step_rank0"] = spill // max(args.steps, 1)
        if also:
            line["config_128M"] = also
        if c4:
            line["config_c4"] = c4
        if wire_line:
            line["config_wire"] = wire_line
        print(json.dumps(line), flush=True)

    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
