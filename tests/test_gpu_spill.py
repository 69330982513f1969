"""GPU: the C4 push path across ranks rehearsed
with world_size 2 on one GPU: both ranks run on cuda:0, the cross-range spill
goes through gloo (host-staged) instead of RCCL.  Every stream's message is
sliced at EvenDivide(2) server ranges, each slice encoded by the origin's
per-(stream, server) node [KEY_CACHING, FIXING_FLOAT nb=1], slices for the
other rank travel as wire frames, and each rank checks what it decoded against
the C restatement of the same slice -- on the first step (key cache miss,
keys travel) and the second (hit, keys elided and restored)."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

STREAMS, M, SEED = 4, 1 << 14, 1700000000


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _stream_data(sid):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import splitmix64_keys
    keys = splitmix64_keys(M, 4 + sid)
    vals = np.random.default_rng(100 + sid).standard_normal(keys.size).astype(np.float32)
    return keys, vals


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist

    import oracle
    from parameter_server_amd import FIXING_FLOAT, KEY_CACHING
    from parameter_server_amd import filter as F
    from parameter_server_amd import shard
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        F.set_clock(SEED)
        ctx = F.Context(0)
        ranges = shard.server_ranges(world)
        router = shard.PushRouter(ctx, ranges, rank, world, shard.SpillExchange(device="cuda:0"))
        streams = {}
        for sid in range(STREAMS):
            if sid % world != rank:
                continue
            keys, vals = _stream_data(sid)
            m = F.Message(request=True, push=True, key_channel=sid, key_range=shard.KEY_ALL)
            m.set_key(torch.from_numpy(keys.view(np.int64)).cuda())
            m.add_value(torch.from_numpy(vals).cuda())
            m.add_filter(KEY_CACHING)
            m.add_filter(FIXING_FLOAT, num_bytes=1)
            streams[sid] = m
        port_ = oracle.Port()
        lo, hi = ranges[rank]
        ok, seen = True, 0
        for step in range(2):
            got = router.step(streams)
            torch.cuda.synchronize()
            chans = set()
            for w in got:
                sid = shard.w_channel(w)
                chans.add(sid)
                keys, vals = _stream_data(sid)
                sel = (keys >= np.uint64(lo)) & (keys < np.uint64(hi))
                st, codes, mn, mx = port_.ff_encode(vals[sel], 1, SEED)
                st, dec = port_.ff_decode(codes, 1, mn, mx, np.float32)
                p, n, loc = w.key_ptr()
                kgot = F.copy_out(p, n, loc, "cuda:0").cpu().numpy().view(np.uint64)
                vp, vn, vl = w.value_ptr(0)
                vgot = F.copy_out(vp, vn, vl, "cuda:0").cpu().numpy().view(np.float32)
                ok &= kgot.tobytes() == keys[sel].tobytes()
                ok &= vgot.tobytes() == dec.tobytes()
                seen += 1
            ok &= chans == set(range(STREAMS))
        q.put((rank, bool(ok), seen))
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, repr(e), 0))
    finally:
        dist.destroy_process_group()


def test_push_router_world2_same_gpu():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        r, ok, seen = q.get(timeout=110)
        res[r] = (ok, seen)
    for p in procs:
        p.join(timeout=30)
    assert res == {0: (True, 2 * STREAMS), 1: (True, 2 * STREAMS)}, res
