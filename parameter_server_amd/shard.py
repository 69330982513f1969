"""The multi-GPU split of the filter path.

Server s owns Range<Key>(key_start, key_end).EvenDivide(S, s)
(src/system/assigner.h:17-28, src/util/range.h:100-107); servers live on ranks
in contiguous blocks (rank r hosts servers [r*S/W, (r+1)*S/W), one server per
GPU when S == W).  A push/pull message is sliced at the server ranges
(SliceKOFVMessage, src/system/message.h:107-147), each slice is encoded by the
sender's per-(stream, server) RemoteNode (executor.cc:131-146) and delivered to
its server, whose per-(server, stream) RemoteNode decodes it.

The only data-path collective is the cross-range spill: slices whose server
lives on another rank travel in one all-to-all-v per step (RCCL over xGMI with
the "nccl" backend; gloo for the CPU tests).  What travels is the ENCODED
slice -- the reference's wire frames [Task][key][value...] (van.cc:122-191),
laid out by libpsf (psf_spill_pack / psf_spill_fill, one gather launch) and
rebuilt zero-copy on the receiver (psf_spill_unpack) -- so KEY_CACHING hits
and FIXING_FLOAT's 4x shrink cut the xGMI bytes too.  Per step the host does
one small all-to-all of segment sizes (one device->host read) and one
all-to-all-v of bytes; no per-frame or per-peer host work.
"""
from __future__ import annotations

import ctypes as C
from typing import List, Optional, Sequence

import torch

from ._lib import check, lib

KEY_ALL = (0, (1 << 64) - 1)  # Range<Key>::All(), range.h:92-95


def even_divide(key_range, n: int, i: int):
    """Range<Key>(key_range).EvenDivide(n, i), exactly (long double)."""
    b, e = C.c_uint64(), C.c_uint64()
    check(lib().psf_range_even_divide(key_range[0], key_range[1], n, i, C.byref(b), C.byref(e)))
    return b.value, e.value


def server_ranges(nservers: int, key_range=KEY_ALL):
    """The key ranges of servers 0..nservers-1 (manager.cc:36-37 + assigner.h:21)."""
    return [even_divide(key_range, nservers, g) for g in range(nservers)]


def server_rank(server: int, nservers: int, world: int) -> int:
    """The rank hosting `server`: contiguous blocks of servers per rank."""
    return server * world // nservers


def slice_message(ctx, msg, ranges: Sequence, key_bytes: int = 8):
    """SliceKOFVMessage: returns one Message per range, or None where the range
    misses the message's key range (the reference marks those invalid and
    does not send them)."""
    return slice_messages(ctx, [msg], ranges, key_bytes)[0]


def slice_messages(ctx, msgs, ranges: Sequence, key_bytes: int = 8):
    """slice_message for many messages with one device synchronisation;
    returns one list per message."""
    from .filter import Message
    n, M = len(ranges), len(msgs)
    for i in range(1, n):
        if ranges[i - 1][1] != ranges[i][0]:
            raise ValueError("ranges must be contiguous (message.h:120)")
    bounds = (C.c_uint64 * (n + 1))(*([r[0] for r in ranges[:1]] + [r[1] for r in ranges]))
    outs = (C.c_void_p * (n * M))()
    valid = (C.c_int * (n * M))()
    hs = (C.c_void_p * M)(*[m.h.value for m in msgs])
    check(lib().psf_msgs_slice(ctx.h, hs, M, bounds, n, key_bytes, outs, valid))
    res = []
    for j, msg in enumerate(msgs):
        row = []
        for i in range(n):
            m = Message(_handle=C.c_void_p(outs[j * n + i]), _refs=msg._refs)
            row.append(m if valid[j * n + i] else None)
        res.append(row)
    return res


def w_channel(m) -> int:
    ch = C.c_int32()
    check(lib().psf_msg_key_channel(m.h, C.byref(ch)))
    return ch.value


class SpillExchange:
    """The cross-range spill of one step: encoded messages -> their ranks, in
    one all-to-all-v (plus one all-to-all of the 2 x world segment sizes).

    `device` is where the buffers live ("cuda:k" with RCCL; with gloo, device
    buffers are staged through host memory, which is what the CPU tests and
    the single-GPU gloo rehearsals use)."""

    def __init__(self, ctx, group=None, device=None):
        import torch.distributed as dist
        self.dist = dist
        self.ctx = ctx
        self.group = group
        self.world = dist.get_world_size(group)
        self.device = device if device is not None else (
            f"cuda:{ctx.device}" if ctx.device >= 0 else "cpu")
        self.staged = dist.get_backend(group) == "gloo" and str(self.device).startswith("cuda")
        self.bytes_sent = 0

    def exchange(self, msgs, dest: List[int], server: List[int]):
        """Send msgs[i] to rank dest[i] (addressed to server server[i]);
        returns (received messages, their servers)."""
        from .filter import Message
        dist, W, L = self.dist, self.world, lib()
        n = len(msgs)
        sizes = (C.c_int64 * (2 * W))()
        plan = C.c_void_p()
        check(L.psf_spill_pack(self.ctx.h, (C.c_void_p * n)(*[m.h.value for m in msgs]),
                               (C.c_int * n)(*dest), (C.c_int * n)(*server), n, W, sizes, C.byref(plan)))
        try:
            wire_dev = "cpu" if self.staged else self.device
            size_t = torch.tensor(list(sizes), dtype=torch.int64)
            size_in = torch.empty_like(size_t)
            if wire_dev != "cpu":
                size_t, size_in = size_t.to(wire_dev, non_blocking=True), size_in.to(wire_dev)
            dist.all_to_all_single(size_in, size_t, group=self.group)
            sizes_in = size_in.cpu().tolist()  # the one device->host read of the step
            in_splits = [sizes[2 * r] + sizes[2 * r + 1] for r in range(W)]
            out_splits = [sizes_in[2 * s] + sizes_in[2 * s + 1] for s in range(W)]
            sendbuf = torch.empty(max(sum(in_splits), 1), dtype=torch.uint8, device=self.device)
            check(L.psf_spill_fill(plan, C.c_void_p(sendbuf.data_ptr())))
        finally:
            L.psf_spill_destroy(plan)
        self.bytes_sent += sum(in_splits) - in_splits[dist.get_rank(self.group)]
        recvbuf = torch.empty(max(sum(out_splits), 1), dtype=torch.uint8, device=wire_dev)
        if self.staged:
            self.ctx.sync()
            sendbuf = sendbuf.cpu()
        dist.all_to_all_single(recvbuf[:sum(out_splits)], sendbuf[:sum(in_splits)], out_splits, in_splits,
                               group=self.group)
        if self.staged:
            recvbuf = recvbuf.to(self.device)
        cap = max(1, sum(sizes_in[0::2]) // 24)  # a record is >= 24 bytes
        outs = (C.c_void_p * cap)()
        servers = (C.c_int * cap)()
        got = C.c_int()
        sin = (C.c_int64 * (2 * W))(*sizes_in)
        check(L.psf_spill_unpack(self.ctx.h, C.c_void_p(recvbuf.data_ptr()), W, sin, outs, servers, cap,
                                 C.byref(got)))
        res = [Message(_handle=C.c_void_p(outs[i]), _refs=[recvbuf]) for i in range(got.value)]
        return res, [servers[i] for i in range(got.value)]


class PushRouter:
    """The multi-server push path of one rank: every
    local stream's message is sliced at the `ranges` of S servers
    (SliceKOFVMessage), each slice is encoded by the sender's per-(stream,
    server) RemoteNode (executor.cc:131-146); slices whose server lives on
    this rank are decoded here, the others travel in ONE all-to-all-v per step
    (the cross-range spill) and are decoded by their server's per-stream node.
    The stream id travels as the Task's key_channel.  `loopback` sends the
    local slices through the exchange too (a world-1 run of the RCCL path)."""

    def __init__(self, ctx, ranges, rank: int, world: int, exchange: Optional[SpillExchange] = None,
                 loopback: bool = False):
        from .filter import RemoteNode
        self.ctx, self.ranges, self.rank, self.world = ctx, ranges, rank, world
        self.nservers = len(ranges)
        if self.nservers < world:
            raise ValueError("need at least one server per rank")
        self.exchange = exchange
        if (world > 1 or loopback) and exchange is None:
            raise ValueError("a spill exchange is needed")
        self.loopback = loopback
        self._RemoteNode = RemoteNode
        self.senders, self.receivers = {}, {}
        self.last_encoded = []  # (stream, server, encoded slice) of the last step

    def owner(self, server: int) -> int:
        return server_rank(server, self.nservers, self.world)

    def _sender(self, s, d):
        if (s, d) not in self.senders:
            self.senders[(s, d)] = self._RemoteNode(self.ctx)
        return self.senders[(s, d)]

    def _receiver(self, d, s):
        if (d, s) not in self.receivers:
            self.receivers[(d, s)] = self._RemoteNode(self.ctx)
        return self.receivers[(d, s)]

    def step(self, streams, keep_encoded: bool = False) -> list:
        """streams: {stream id: template Message (key_channel = stream id)} of
        this rank.  Returns [(server, decoded message)] of what this rank's
        servers received.  All slices of the step are encoded in one batched
        call (psf_nodes_encode) and all received ones decoded in one
        (psf_nodes_decode)."""
        from .filter import RemoteNode
        enc_nodes, enc_msgs, dest = [], [], []
        sids = list(streams)
        clones = [streams[sid].clone() for sid in sids]
        for sid, parts in zip(sids, slice_messages(self.ctx, clones, self.ranges)):
            for d, part in enumerate(parts):
                if part is None:
                    continue
                enc_nodes.append(self._sender(sid, d))
                enc_msgs.append(part)
                dest.append((sid, d))
        if enc_msgs:
            RemoteNode.encode_many(enc_nodes, enc_msgs)
        self.last_encoded = list(zip(dest, enc_msgs)) if keep_encoded else []
        dec_nodes, dec_msgs, got = [], [], []
        out_m, out_r, out_s = [], [], []
        for (sid, d), part in zip(dest, enc_msgs):
            r = self.owner(d)
            if r == self.rank and not self.loopback:
                w = part.clone()  # delivered copy (Task + zero-copy buffers)
                dec_nodes.append(self._receiver(d, sid))
                dec_msgs.append(w)
                got.append((d, w))
            else:
                out_m.append(part)
                out_r.append(r)
                out_s.append(d)
        if self.world > 1 or self.loopback:
            recv, servers = self.exchange.exchange(out_m, out_r, out_s)
            for w, d in zip(recv, servers):
                dec_nodes.append(self._receiver(d, w_channel(w)))
                dec_msgs.append(w)
                got.append((d, w))
        if dec_msgs:
            RemoteNode.decode_many(dec_nodes, dec_msgs)
        return got
