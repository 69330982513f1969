"""ORACLE TEST INFRASTRUCTURE -- a CPU restatement of the reference's message
path for the filter chain, the checker for libpsf's RemoteNode / Filter
classes.  Only tests/ and tests/golden/make_golden.py use it.

Restates, on numpy byte buffers:

* ``Message`` / ``Task`` / ``FilterConfig`` fields the filters read and write
  (src/system/message.h:10-76, task.proto:28-39, filter.proto:3-35): has_key
  = key non-empty, clear_key, set_key<char> (key_type CHAR), proto2 has-bits
* ``Node`` = RemoteNode (remote_node.cc:7-29): one filter instance per type,
  encode in task.filter order, decode in reverse; ``Filter::find``
  (filter.cc:26-31) = the first config of a type
* KEY_CACHING (key_caching.h:9-75): CRC32C signature of the first 2 KiB, cache
  per (key_channel, key_range), hit = same signature and byte length,
  clear_cache_if_done when !request || param.push, fatal receiver miss
* FIXING_FLOAT (fixing_float.h:24-101): the message rules of convert() --
  num_bytes 0 no-op, value/value_type count CHECK, empty arrays skipped, a
  fixed_point entry added per non-empty array while k runs past the list,
  k advanced only for FLOAT/DOUBLE -- with the element arithmetic of
  oracle/psf_port.c (Port.ff_encode / ff_decode)
* COMPRESSING (compressing.h:8-37, shared_array_inl.h:232-255): snappy 1.1.8
  restated in oracle/snappy_port.c; empty arrays stay empty
* NOISE (add_noise.h:11-39): Port.add_noise, in place

Any CHECK failure of the reference is a status of -1 (the reference aborts).
``PortImpl`` puts this behind tests/scenarios.py's runner interface.
"""
from __future__ import annotations

import copy

import numpy as np

KEY_CACHING, COMPRESSING, FIXING_FLOAT, NOISE = 1, 2, 3, 4
DT_UINT64, DT_FLOAT, DT_DOUBLE, DT_CHAR = 8, 9, 10, 11
_EMPTY = np.zeros(0, np.uint8)


class CheckFailed(Exception):
    """a glog CHECK of the reference fired"""


def _check(cond, what):
    if not cond:
        raise CheckFailed(what)


class FixedPoint:
    def __init__(self):
        self.has_min = self.has_max = False
        self.min_value, self.max_value = np.float32(-1), np.float32(1)  # filter.proto:22-25 defaults


class FilterConfig:
    def __init__(self, ftype):
        self.type = ftype
        self.has_signature, self.signature = False, 0
        self.uncompressed_size = []
        self.fixed_point = []
        self.num_bytes = 3  # filter.proto:21 default
        self.clear_cache_if_done = False
        self.mean = self.std = 0.0


class Task:
    def __init__(self, request, push, has_param, channel, kr):
        self.request, self.push, self.has_param = request, push, has_param
        self.key_channel = channel
        self.has_key_range = kr is not None
        self.key_range = tuple(kr) if kr is not None else (0, 0)
        self.has_key, self.key_type = False, 0
        self.value_type = []
        self.filter = []


class Message:
    def __init__(self, task):
        self.task = task
        self.key = _EMPTY
        self.value = []

    def has_key(self):
        return self.key.size > 0

    def clear_key(self):  # message.h:22
        self.task.has_key = False
        self.key = _EMPTY

    def set_key_char(self, k):  # message.h:69-76 with T = char
        self.task.key_type = DT_CHAR
        if self.has_key():
            self.clear_key()
        self.task.has_key = True
        self.key = k
        if not self.task.has_key_range:
            self.task.has_key_range, self.task.key_range = True, (0, (1 << 64) - 1)

    def clone(self):
        """the receiver's copy: the Task by value, the buffers shared"""
        m = Message(copy.deepcopy(self.task))
        m.key = self.key
        m.value = list(self.value)
        return m


def find(ftype, msg):  # filter.cc:26-31
    for f in msg.task.filter:
        if f.type == ftype:
            return f
    return None


class KeyCaching:
    def __init__(self, port):
        self.port = port
        self.cache = {}

    def _sig(self, key):
        return self.port.key_signature(key)  # crc32c of the first min(size, 2048) bytes

    @staticmethod
    def _done(t):  # key_caching.h:63-67
        return (not t.request) or (t.has_param and t.push)

    def encode(self, msg):  # key_caching.h:9-34
        conf = find(KEY_CACHING, msg)
        if conf is None:
            return
        if not msg.has_key():
            conf.has_signature, conf.signature = False, 0
            return
        sig = self._sig(msg.key)
        conf.has_signature, conf.signature = True, sig
        ck = (msg.task.key_channel, msg.task.key_range)
        c = self.cache.setdefault(ck, [0, _EMPTY])
        if c[0] == sig and c[1].size == msg.key.size:
            msg.clear_key()
        else:
            c[0], c[1] = sig, msg.key
        if conf.clear_cache_if_done and self._done(msg.task):
            del self.cache[ck]

    def decode(self, msg):  # key_caching.h:36-60
        conf = find(KEY_CACHING, msg)
        if conf is None or not conf.has_signature:
            return
        sig = conf.signature
        if msg.has_key():
            _check(self._sig(msg.key) == sig, "CHECK_EQ(crc32c, sig)")
        ck = (msg.task.key_channel, msg.task.key_range)
        c = self.cache.setdefault(ck, [0, _EMPTY])
        if msg.has_key():
            c[0], c[1] = sig, msg.key
        else:
            _check(sig == c[0], "CHECK_EQ(sig, cache.first)")
            msg.set_key_char(c[1])
        if conf.clear_cache_if_done and self._done(msg.task):
            del self.cache[ck]


class FixingFloat:
    def __init__(self, port, clock):
        self.port, self.clock = port, clock

    def encode(self, msg):
        self._convert(msg, True)

    def decode(self, msg):
        self._convert(msg, False)

    def _convert(self, msg, encode):  # fixing_float.h:24-47
        conf = find(FIXING_FLOAT, msg)
        _check(conf is not None, "CHECK_NOTNULL(find(FIXING_FLOAT))")
        if conf.num_bytes == 0:
            return
        _check(len(msg.value) == len(msg.task.value_type), "CHECK_EQ(n, value_type_size())")
        k = 0
        for i, v in enumerate(msg.value):
            if v.size == 0:
                continue
            t = msg.task.value_type[i]
            if len(conf.fixed_point) <= k:
                conf.fixed_point.append(FixedPoint())
            if t in (DT_FLOAT, DT_DOUBLE):
                msg.value[i] = self._array(v, t, encode, conf.num_bytes, conf.fixed_point[k])
                k += 1

    def _array(self, v, t, encode, nb, fp):  # fixing_float.h:50-101
        _check(0 < nb < 8, "CHECK_GT(nbytes, 0) / CHECK_LT(nbytes, 8)")
        dt = np.float32 if t == DT_FLOAT else np.float64
        if encode:
            x = v.view(dt)
            st, codes, mn, mx = self.port.ff_encode(x, nb, self.clock(),
                                                    fp.min_value if fp.has_min else None,
                                                    fp.max_value if fp.has_max else None)
            # the side-info is written before CHECK_GT(bin, 0) fires (fixing_float.h:58-71)
            if not fp.has_min:
                fp.has_min, fp.min_value = True, np.float32(mn)
            if not fp.has_max:
                fp.has_max, fp.max_value = True, np.float32(mx)
            _check(st == 0, "CHECK_GT(bin, 0)")
            return codes
        _check(fp.has_min and fp.has_max, "CHECK(conf->has_min_value() / has_max_value())")
        _check(float(fp.max_value) - float(fp.min_value) > 0, "CHECK_GT(bin, 0)")
        st, out = self.port.ff_decode(v, nb, float(fp.min_value), float(fp.max_value), dt)
        _check(st == 0, "ff_decode")
        return out.view(np.uint8)


class Compressing:
    def __init__(self, port):
        self.port = port

    def _compress(self, b):  # SArray::CompressTo: empty stays empty
        return _EMPTY if b.size == 0 else np.frombuffer(self.port.snappy_compress(b.tobytes()), np.uint8)

    def _uncompress(self, b):  # SArray::UncompressFrom
        if b.size == 0:
            return _EMPTY
        st, out = self.port.snappy_uncompress(b.tobytes(), cap=1 << 31)
        _check(st == 0, "CHECK(snappy::RawUncompress)")
        return np.frombuffer(out, np.uint8)

    def encode(self, msg):  # compressing.h:8-19
        conf = find(COMPRESSING, msg)
        if conf is None:
            return
        conf.uncompressed_size = []
        if msg.has_key():
            conf.uncompressed_size.append(int(msg.key.size))
            msg.key = self._compress(msg.key)
        for i, v in enumerate(msg.value):
            conf.uncompressed_size.append(int(v.size))
            msg.value[i] = self._compress(v)

    def decode(self, msg):  # compressing.h:20-37
        conf = find(COMPRESSING, msg)
        if conf is None:
            return
        has_key = 1 if msg.has_key() else 0
        _check(len(conf.uncompressed_size) == len(msg.value) + has_key, "CHECK_EQ(uncompressed_size_size())")
        if has_key:
            msg.key = self._uncompress(msg.key)
        for i, v in enumerate(msg.value):
            msg.value[i] = self._uncompress(v)


class AddNoise:
    def __init__(self, port):
        self.port = port

    def encode(self, msg):  # add_noise.h:11-25
        conf = find(NOISE, msg)
        _check(conf is not None, "CHECK_NOTNULL(find(NOISE))")
        _check(len(msg.value) == len(msg.task.value_type), "CHECK_EQ(n, value_type_size())")
        for i, v in enumerate(msg.value):
            t = msg.task.value_type[i]
            if v.size == 0 or t not in (DT_FLOAT, DT_DOUBLE):
                continue
            dt = np.float32 if t == DT_FLOAT else np.float64
            msg.value[i] = self.port.add_noise(v.view(dt), conf.mean, conf.std).view(np.uint8)

    def decode(self, msg):
        pass


class Node:
    """RemoteNode (remote_node.cc:7-29, remote_node.h:61-63)."""

    def __init__(self, port, clock):
        self.port, self.clock = port, clock
        self.filters = {}

    def _filter(self, conf):  # FindFilterOrCreate + Filter::create (filter.cc:9-23)
        f = self.filters.get(conf.type)
        if f is None:
            f = {KEY_CACHING: lambda: KeyCaching(self.port),
                 COMPRESSING: lambda: Compressing(self.port),
                 FIXING_FLOAT: lambda: FixingFloat(self.port, self.clock),
                 NOISE: lambda: AddNoise(self.port)}[conf.type]()
            self.filters[conf.type] = f
        return f

    def encode(self, msg):
        for conf in list(msg.task.filter):
            self._filter(conf).encode(msg)

    def decode(self, msg):
        for conf in reversed(list(msg.task.filter)):
            self._filter(conf).decode(msg)


class PortImpl:
    """This restatement behind tests/scenarios.py's runner interface."""

    def __init__(self, port=None):
        if port is None:
            import oracle
            port = oracle.Port()
        self.port = port
        self.t = 0

    def set_clock(self, t):
        self.t = t

    def new_node(self):
        return Node(self.port, lambda: self.t)

    def free_node(self, n):
        pass

    def new_msg(self, request, push, channel, kr):
        return Message(Task(request, push, True, channel, kr))

    def free_msg(self, m):
        pass

    def clone(self, m):
        return m.clone()

    def set_key(self, m, keys):
        k = np.ascontiguousarray(keys).view(np.uint8).copy()
        m.key = k
        m.task.has_key = k.size > 0
        m.task.key_type = DT_UINT64
        if not m.task.has_key_range:
            m.task.has_key_range, m.task.key_range = True, (0, (1 << 64) - 1)

    def add_value(self, m, v):
        dt = {np.dtype(np.float32): DT_FLOAT, np.dtype(np.float64): DT_DOUBLE,
              np.dtype(np.uint64): DT_UINT64}[v.dtype]
        m.task.value_type.append(dt)
        m.value.append(np.ascontiguousarray(v).view(np.uint8).copy())

    def add_filter(self, m, ftype, num_bytes=None, clear_cache_if_done=None, fixed_point=None, noise=None):
        f = FilterConfig(ftype)
        if num_bytes is not None:
            f.num_bytes = num_bytes
        if clear_cache_if_done is not None:
            f.clear_cache_if_done = bool(clear_cache_if_done)
        if noise is not None:
            f.mean, f.std = noise
        for mn, mx in fixed_point or []:
            fp = FixedPoint()
            if mn is not None:
                fp.has_min, fp.min_value = True, np.float32(mn)
            if mx is not None:
                fp.has_max, fp.max_value = True, np.float32(mx)
            f.fixed_point.append(fp)
        m.task.filter.append(f)
        return len(m.task.filter) - 1

    def encode(self, n, m):
        try:
            n.encode(m)
            return 0
        except CheckFailed:
            return -1

    def decode(self, n, m):
        try:
            n.decode(m)
            return 0
        except CheckFailed:
            return -1

    def key(self, m):
        return m.key

    def key_info(self, m):
        return bool(m.task.has_key), int(m.task.key_type)

    def values(self, m):
        return list(m.value)

    def signature(self, m, i):
        f = m.task.filter[i]
        return bool(f.has_signature), int(f.signature)

    def fixed_points(self, m, i):
        return [(fp.has_min, float(fp.min_value), fp.has_max, float(fp.max_value))
                for fp in m.task.filter[i].fixed_point]

    def uncompressed(self, m, i):
        return [int(s) for s in m.task.filter[i].uncompressed_size]
