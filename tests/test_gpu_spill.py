"""GPU: the C4 / C5 multi-server push path.

Every stream's message is sliced at EvenDivide(S) server ranges
(SliceKOFVMessage, message.h:107-147), each slice encoded by the origin's
per-(stream, server) RemoteNode, slices for servers on other ranks packed into
one buffer and moved by one all-to-all-v, and decoded by the server's
per-(server, stream) node.  Each case checks every decoded slice against the C
restatement of the same slice -- on the first step (key cache miss, keys
travel) and the second (hit, keys elided and restored):

* 64 streams x 8 servers in one process (C4's shape at N=1, all local)
* the RCCL path at world 1: `nccl` process group, loopback spill of every
  slice through psf_spill_pack -> all_to_all_single -> psf_spill_unpack
* world 2 on one GPU over gloo (host-staged exchange)
* C5's shape: 2^14 keys x 128-wide f32 rows sliced at EvenDivide(8) (k = 128
  values per key), [KEY_CACHING, FIXING_FLOAT nb=1, COMPRESSING]; the encoded
  slices are also checked byte for byte (codes -> snappy 1.1.8 restatement)
"""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 1700000000


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _stream_data(sid, m, dim):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import splitmix64_keys
    keys = splitmix64_keys(m, 4 + sid)
    vals = np.random.default_rng(100 + sid).standard_normal(keys.size * dim).astype(np.float32)
    return keys, vals


def _make_streams(F, sids, m, dim, compress):
    import torch

    from parameter_server_amd import COMPRESSING, FIXING_FLOAT, KEY_CACHING
    from parameter_server_amd import shard
    streams = {}
    for sid in sids:
        keys, vals = _stream_data(sid, m, dim)
        msg = F.Message(request=True, push=True, key_channel=sid, key_range=shard.KEY_ALL)
        msg.set_key(torch.from_numpy(keys.view(np.int64)).cuda())
        msg.add_value(torch.from_numpy(vals).cuda())
        msg.add_filter(KEY_CACHING)
        msg.add_filter(FIXING_FLOAT, num_bytes=1)
        if compress:
            msg.add_filter(COMPRESSING)
        streams[sid] = msg
    return streams


def _check_step(F, got, ranges, m, dim, port, expect):
    """every (server, decoded slice) equals the restatement; returns the
    (server, stream) pairs seen"""
    from parameter_server_amd import shard
    seen = set()
    for d, w in got:
        sid = shard.w_channel(w)
        seen.add((d, sid))
        keys, vals = _stream_data(sid, m, dim)
        lo, hi = ranges[d]
        sel = (keys >= np.uint64(lo)) & (keys < np.uint64(hi))
        v = vals.reshape(-1, dim)[sel].reshape(-1)
        st, codes, mn, mx = port.ff_encode(v, 1, SEED)
        st, dec = port.ff_decode(codes, 1, mn, mx, np.float32)
        p, n, loc = w.key_ptr()
        kgot = F.copy_out(p, n, loc, "cuda:0").cpu().numpy().view(np.uint64)
        vp, vn, vl = w.value_ptr(0)
        vgot = F.copy_out(vp, vn, vl, "cuda:0").cpu().numpy().view(np.float32)
        assert kgot.tobytes() == keys[sel].tobytes(), (d, sid)
        assert vgot.tobytes() == dec.tobytes(), (d, sid)
    assert seen == expect
    assert len(got) == len(expect), "a step's results hold each (server, stream) once"
    return seen


def test_push_router_64_streams_8_servers():
    """C4's shape at N=1: 64 streams x 8 servers, all slices local."""
    import torch

    import oracle
    from parameter_server_amd import filter as F
    from parameter_server_amd import shard
    STREAMS, M, S = 64, 1 << 13, 8
    F.set_clock(SEED)
    ctx = F.Context(0)
    ranges = shard.server_ranges(S)
    router = shard.PushRouter(ctx, ranges, 0, 1)
    streams = _make_streams(F, range(STREAMS), M, 1, False)
    port = oracle.Port()
    expect = {(d, s) for d in range(S) for s in range(STREAMS)}
    for step in range(2):
        router.step(streams)
        torch.cuda.synchronize()
        _check_step(F, router.results(), ranges, M, 1, port, expect)


@pytest.mark.parametrize("M", [1 << 14, (1 << 16) + 4099])
def test_c5_rows_dim128_full_chain_8_servers(M):
    """C5's shape: M keys x 128 f32, EvenDivide(8) slices (k = 128),
    [KEY_CACHING, FIXING_FLOAT nb=1, COMPRESSING]; the larger M gives slices of
    several fragments with a ragged last one."""
    import torch

    import oracle
    from parameter_server_amd import filter as F
    from parameter_server_amd import shard
    DIM, S = 128, 8
    F.set_clock(SEED)
    ctx = F.Context(0)
    ranges = shard.server_ranges(S)
    router = shard.PushRouter(ctx, ranges, 0, 1)
    streams = _make_streams(F, [0], M, DIM, True)
    port = oracle.Port()
    keys, vals = _stream_data(0, M, DIM)
    for step in range(2):
        router.step(streams, keep_encoded=True)
        torch.cuda.synchronize()
        _check_step(F, router.results(), ranges, M, DIM, port, {(d, 0) for d in range(S)})
        encoded = router.encoded()
        assert sorted(k for k, _ in encoded) == [(0, d) for d in range(S)]
        for (sid, d), enc in encoded:
            lo, hi = ranges[d]
            sel = (keys >= np.uint64(lo)) & (keys < np.uint64(hi))
            st, codes, mn, mx = port.ff_encode(vals.reshape(-1, DIM)[sel].reshape(-1), 1, SEED)
            vp, vn, vl = enc.value_ptr(0)
            cgot = F.copy_out(vp, vn, vl, "cuda:0").cpu().numpy().tobytes()
            assert cgot == port.snappy_compress(codes.tobytes()), (step, d)
            has_key, _ = enc.key_info()
            kp, kn, kl = enc.key_ptr()
            if step == 0:  # miss: snappy'd keys travel
                kgot = F.copy_out(kp, kn, kl, "cuda:0").cpu().numpy().tobytes()
                assert has_key and kgot == port.snappy_compress(keys[sel].tobytes())
            else:  # hit: KEY_CACHING elided them before COMPRESSING ran
                assert not has_key and kn == 0


@pytest.mark.parametrize("dim,compress,m", [(1, False, 1 << 12), (128, True, 1 << 12), (128, True, (1 << 16) + 77)])
def test_router_multi_step_driver(dim, compress, m):
    """psf_router_step over several steps in one call (what bench.py times):
    each step's slicing pass is queued ahead of the previous step's decodes
    and the COMPRESSING lengths are waited for after it; the last step's
    decoded slices equal the restatement's, and a second call continues the
    key cache (hits)."""
    import torch

    import oracle
    from parameter_server_amd import filter as F
    from parameter_server_amd import shard
    STREAMS, M, S = (16, m, 8) if dim == 1 else (1, m, 8)
    F.set_clock(SEED)
    ctx = F.Context(0)
    ranges = shard.server_ranges(S)
    router = shard.PushRouter(ctx, ranges, 0, 1)
    streams = _make_streams(F, range(STREAMS), M, dim, compress)
    port = oracle.Port()
    expect = {(d, s) for d in range(S) for s in range(STREAMS)}
    for _ in range(2):
        router.run(streams, 3)
        torch.cuda.synchronize()
        _check_step(F, router.results(), ranges, M, dim, port, expect)
    hs = router.host_stats()
    assert hs["steps"] == 6


def _spill_worker(rank, world, port, backend, loopback, q, native=None):
    import ctypes as C

    import torch
    import torch.distributed as dist

    import oracle
    from parameter_server_amd import filter as F
    from parameter_server_amd import shard
    from parameter_server_amd._lib import lib
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    self_p2p = native == "rccl_p2p"
    if self_p2p:
        native = "rccl"
        L = lib()
        L.psf_debug_exchange_self_p2p.argtypes = [C.c_int]
        L.psf_debug_exchange_self_p2p.restype = C.c_int
        assert L.psf_debug_exchange_self_p2p(1) == 0
    try:
        torch.cuda.set_device(0)
        if backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda:0"))
        else:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        STREAMS, M, S = 4, 1 << 14, 2 * world
        F.set_clock(SEED)
        ctx = F.Context(0)
        ranges = shard.server_ranges(S)
        if native:
            ex = shard.NativeExchange.create(ctx, transport=native)
        else:
            ex = shard.SpillExchange(ctx, device="cuda:0")
        router = shard.PushRouter(ctx, ranges, rank, world, ex, loopback=loopback)
        streams = _make_streams(F, [s for s in range(STREAMS) if s % world == rank], M, 1, False)
        port_ = oracle.Port()
        mine = [d for d in range(S) if router.owner(d) == rank]
        expect = {(d, s) for d in mine for s in range(STREAMS)}
        sent = []
        for step in range(2):
            router.step(streams)
            torch.cuda.synchronize()
            _check_step(F, router.results(), ranges, M, 1, port_, expect)
            sent.append(ex.bytes_sent)
        if native:
            sent.append(ex.data_stats())
        q.put((rank, True, sent))
    except Exception as e:  # report instead of hanging the parent
        import traceback
        q.put((rank, repr(e) + traceback.format_exc()[-1500:], None))
    finally:
        if self_p2p:
            L.psf_debug_exchange_self_p2p(0)
        if dist.is_initialized():
            dist.destroy_process_group()


def _run_ranks(world, backend, loopback, native=None):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_spill_worker, args=(r, world, port, backend, loopback, q, native))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        r, ok, sent = q.get(timeout=110)
        res[r] = (ok, sent)
    for p in procs:
        p.join(timeout=30)
    return res


@pytest.mark.parametrize("native", [None, "rccl", "rccl_p2p"])
def test_spill_nccl_world1_loopback(native):
    """The RCCL spill path on the device at world 1, every slice through the
    exchange: torch's all_to_all_single (the Python step), or libpsf's own
    exchange (native: the records through the mailbox, the data on the
    exchange's stream, psf_router_step).  rccl_p2p: the self slice goes
    through ncclSend / ncclRecv to self inside the step's group
    (psf_debug_exchange_self_p2p) -- the grouped point-to-point code the
    node's other ranks run (executor.cc:134-146's per-server sends) -- and
    every decoded slice still equals the port's."""
    res = _run_ranks(1, "nccl", True, native)
    ok, sent = res[0]
    assert ok is True, ok
    if native:
        ds = sent[-1]
        assert not ds["failed"]
        if native == "rccl_p2p":
            # every data byte of both steps went through ncclSend, none copied
            assert ds["rccl_sends"] == 2 and ds["rccl_bytes"] > 0 and ds["copied_bytes"] == 0, ds
        else:
            assert ds["rccl_sends"] == 0 and ds["copied_bytes"] > 0, ds


@pytest.mark.parametrize("native", [None, "host"])
def test_push_router_world2_same_gpu(native):
    """Two ranks on cuda:0 over gloo (host-staged), 2 servers per rank; native:
    libpsf's exchange through the host mailbox."""
    res = _run_ranks(2, "gloo", False, native)
    for r in range(2):
        ok, sent = res[r]
        assert ok is True, ok
        # the key-cache hit step sends no keys: fewer spill bytes than the miss step
        assert 0 < sent[1] - sent[0] < sent[0]


@pytest.mark.parametrize("gpus", [1, 2])
def test_bench_default_reports_c4_spill(gpus):
    """bench.py's default command (c2) with its companion C4 line, small sizes:
    at --gpus 2 (two ranks sharing cuda:0 over gloo, the rehearsal knobs) the
    C4 slices for the other rank's servers travel in the all-to-all-v and
    config_c4 reports the spilled bytes; at --gpus 1 nothing spills."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PSF_DIST_BACKEND="gloo", PSF_SAME_GPU="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", str(gpus), "--n", str(1 << 20),
                          "--c4-m", str(1 << 14), "--steps", "3", "--warmup", "1", "--no-cpu-baseline",
                          "--no-profile", "--no-128m"], env=env, capture_output=True, text=True, timeout=110)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [json.loads(x) for x in out.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, out.stdout
    ln = lines[0]
    assert ln["n_gpus"] == gpus and ln["value"] > 0
    c4 = ln["config_c4"]
    assert c4["measured"] and c4["value"] > 0 and c4["world_size"] == gpus
    if gpus == 2:
        assert c4["backend"] == "gloo" and c4["scaling"] == "strong"
        assert c4["spill_bytes_per_step_rank0"] > 0
    else:
        assert c4["spill_bytes_per_step_rank0"] == 0
