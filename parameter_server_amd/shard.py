"""The multi-GPU split of the filter path.

GPU g is server g and owns Range<Key>(key_start, key_end).EvenDivide(N, g)
(src/system/assigner.h:17-28, src/util/range.h:100-107).  A push/pull message
is sliced at those ranges (SliceKOFVMessage, src/system/message.h:107-147),
each slice is encoded by the sender's per-peer RemoteNode (executor.cc:131-146)
and delivered to its owner, where the owner's RemoteNode decodes it.

The only data-path collective is the cross-range spill: slices whose owner is
another GPU travel in one all-to-all-v per step (RCCL over xGMI with the
"nccl" backend; gloo for the CPU tests).  What travels is the ENCODED slice --
the reference's wire frames [Task][key][value...] (van.cc:122-191) -- so
KEY_CACHING hits and FIXING_FLOAT's 4x shrink cut the xGMI bytes too.
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


def slice_message(ctx, msg, ranges: Sequence, key_bytes: int = 8):
    """SliceKOFVMessage: returns one Message per range, or None where the range
    misses the message's key range (the reference marks those invalid and
    does not send them)."""
    from .filter import Message
    n = len(ranges)
    for i in range(1, n):
        if ranges[i - 1][1] != ranges[i][0]:
            raise ValueError("ranges must be contiguous (message.h:120)")
    bounds = (C.c_uint64 * (n + 1))(*([r[0] for r in ranges[:1]] + [r[1] for r in ranges]))
    outs = (C.c_void_p * n)()
    valid = (C.c_int * n)()
    check(lib().psf_msg_slice(ctx.h, msg.h, bounds, n, key_bytes, outs, valid))
    res: List[Optional[Message]] = []
    for i in range(n):
        m = Message(_handle=C.c_void_p(outs[i]), _refs=msg._refs)
        res.append(m if valid[i] else None)
    return res


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


def parse_frames(frames: List[torch.Tensor]):
    """Split a flat list of received frames into messages: each is a Task frame
    followed by its key frame (when the Task has has_key) and one frame per
    value_type entry (van.cc:193-255)."""
    from .filter import Message
    out, i = [], 0
    while i < len(frames):
        m = Message.from_task_bytes(frames[i].cpu().numpy().tobytes())
        i += 1
        has_key, _ = m.key_info()
        nval = task_value_count(m)
        for _ in range(int(has_key) + nval):
            m.recv_frame(frames[i])
            i += 1
        out.append(m)
    return out


def task_value_count(m) -> int:
    """number of value_type entries of a parsed Task (its value frames)."""
    n = C.c_int()
    check(lib().psf_task_value_count(m.h, C.byref(n)))
    return n.value


class PushRouter:
    """The multi-server push path of one rank: every
    local stream's message is sliced at the server key ranges
    (SliceKOFVMessage), each slice is encoded by the sender's per-(stream,
    server) RemoteNode (executor.cc:131-146); slices owned by this rank are
    decoded here, the others travel as wire frames in ONE all-to-all-v per step
    (the cross-range spill) and are decoded by their owner's per-stream node.
    The stream id travels as the Task's key_channel."""

    def __init__(self, ctx, ranges, rank: int, world: int, exchange=None):
        from .filter import RemoteNode
        self.ctx, self.ranges, self.rank, self.world = ctx, ranges, rank, world
        self.exchange = exchange
        self._RemoteNode = RemoteNode
        self.senders, self.receivers = {}, {}
        self.device = f"cuda:{ctx.device}" if ctx.device >= 0 else "cpu"

    def _sender(self, s, d):
        if (s, d) not in self.senders:
            self.senders[(s, d)] = self._RemoteNode(self.ctx)
        return self.senders[(s, d)]

    def _receiver(self, s):
        if s not in self.receivers:
            self.receivers[s] = self._RemoteNode(self.ctx)
        return self.receivers[s]

    def step(self, streams) -> list:
        """streams: {stream id: template Message (key_channel = stream id)} of
        this rank.  Returns the decoded messages this rank received.  All
        slices of the step are encoded in one batched call (psf_nodes_encode)
        and all received ones decoded in one (psf_nodes_decode)."""
        from .filter import RemoteNode
        send = [[] for _ in range(self.world)]
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
        dec_nodes, dec_msgs = [], []
        for (sid, d), part in zip(dest, enc_msgs):
            if d == self.rank:
                dec_nodes.append(self._receiver(sid))
                dec_msgs.append(part.clone())
            else:
                send[d].extend(part.device_frames(self.device))
        if self.world > 1:
            recv = self.exchange.exchange(send)
            for src in range(self.world):
                for w in parse_frames(recv[src]):
                    dec_nodes.append(self._receiver(w_channel(w)))
                    dec_msgs.append(w)
        if dec_msgs:
            RemoteNode.decode_many(dec_nodes, dec_msgs)
        return dec_msgs


def w_channel(m) -> int:
    ch = C.c_int32()
    check(lib().psf_msg_key_channel(m.h, C.byref(ch)))
    return ch.value


class SpillExchange:
    """All-to-all-v of byte frames between ranks (one collective per step).

    send[dst] is a list of uint8 tensors (frames) for rank dst; the result
    recv[src] is the list of frames rank src sent here, in order.  Frame
    lengths travel first (one small all-to-all), then all bytes in one
    all_to_all_single with per-peer split sizes."""

    def __init__(self, group=None, device=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.device = device

    def exchange(self, send: List[List[torch.Tensor]]) -> List[List[torch.Tensor]]:
        dist, W = self.dist, self.world
        dev = self.device if self.device is not None else "cpu"
        if dist.get_backend(self.group) == "gloo" and str(dev).startswith("cuda"):
            # gloo moves host memory only: stage through the host (CPU tests /
            # single-GPU rehearsals; RCCL moves HBM directly)
            self.device = "cpu"
            try:
                recv = self.exchange([[f.cpu() for f in frames] for frames in send])
            finally:
                self.device = dev
            return [[f.to(dev) for f in frames] for frames in recv]
        counts = torch.tensor([len(f) for f in send], dtype=torch.int64, device=dev)
        counts_in = torch.empty_like(counts)
        dist.all_to_all_single(counts_in, counts, group=self.group)
        # every rank must use the same row width for the lens all-to-all
        maxf_t = torch.tensor([max(1, int(counts.max()))], dtype=torch.int64, device=dev)
        dist.all_reduce(maxf_t, op=dist.ReduceOp.MAX, group=self.group)
        maxf = int(maxf_t.item())
        lens = torch.zeros(W, maxf, dtype=torch.int64, device=dev)
        for d, frames in enumerate(send):
            for j, f in enumerate(frames):
                lens[d, j] = f.numel()
        lens_in = torch.empty_like(lens)
        dist.all_to_all_single(lens_in.view(-1), lens.view(-1), group=self.group)
        in_splits = [int(lens[d].sum()) for d in range(W)]
        out_splits = [int(lens_in[s].sum()) for s in range(W)]
        flat = [f.reshape(-1) for frames in send for f in frames]
        sendbuf = torch.cat(flat) if flat else torch.empty(0, dtype=torch.uint8, device=dev)
        recvbuf = torch.empty(sum(out_splits), dtype=torch.uint8, device=dev)
        dist.all_to_all_single(recvbuf, sendbuf, out_splits, in_splits, group=self.group)
        recv, off = [], 0
        counts_l = counts_in.tolist()
        lens_l = lens_in.tolist()
        for s in range(W):
            frames = []
            for j in range(counts_l[s]):
                ln = lens_l[s][j]
                frames.append(recvbuf[off:off + ln])
                off += ln
            recv.append(frames)
        return recv
