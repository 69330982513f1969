"""ORACLE TEST INFRASTRUCTURE -- numpy restatements of the key-range split.

even_divide   <- Range<T>::EvenDivide, src/util/range.h:100-107 (x87 long
                 double == numpy.longdouble on x86-64 Linux)
slice_kofv    <- SliceKOFVMessage<K>, src/system/message.h:107-147
The reference's own range.h is also compiled here (oracle/_ref/libpsrange.so)
and pins even_divide (tests/golden/even_divide.json).
"""
from __future__ import annotations

import numpy as np


def _x86_ld_to_u64(v) -> int:
    """static_cast<uint64_t>(long double) as g++/x86-64 lowers it: values
    >= 2^63 go through (v - 2^63) -> fistp -> xor 2^63, so a value that rounded
    up to 2^64 comes out as 0 (e.g. EvenDivide(7, 6) over Range::All())."""
    iv = int(v)
    if iv >= (1 << 64):
        return 0
    return iv


def even_divide(begin: int, end: int, n: int, i: int):
    assert end >= begin and n > 0 and i < n
    itv = np.longdouble(end - begin) / np.longdouble(n)
    b = np.longdouble(begin) + itv * np.longdouble(i)
    e = np.longdouble(begin) + itv * np.longdouble(i + 1)
    return _x86_ld_to_u64(b), _x86_ld_to_u64(e)


def project(mr, v):
    return max(mr[0], min(mr[1], v))


def slice_kofv(keys: np.ndarray, values, msg_range, krs):
    """Returns per range: None (invalid) or (key segment, [value segments])."""
    n = len(krs)
    for i in range(1, n):
        assert krs[i - 1][1] == krs[i][0]
    mask = (1 << (8 * keys.dtype.itemsize)) - 1
    pos = [0] * (n + 1)
    if n:
        pos[0] = int(np.searchsorted(keys, keys.dtype.type(project(msg_range, krs[0][0]) & mask), "left"))
    for i in range(n):
        pos[i + 1] = int(np.searchsorted(keys, keys.dtype.type(project(msg_range, krs[i][1]) & mask), "left"))
    out = []
    for i in range(n):
        if max(krs[i][0], msg_range[0]) >= min(krs[i][1], msg_range[1]):
            out.append(None)
            continue
        if keys.size == 0:
            out.append((keys[:0], []))
            continue
        lo, hi = pos[i], pos[i + 1]
        vs = []
        for v in values:
            b = v.view(np.uint8)
            k = b.size // keys.size
            assert k * keys.size == b.size
            vs.append(b[lo * k:hi * k])
        out.append((keys[lo:hi], vs))
    return out
