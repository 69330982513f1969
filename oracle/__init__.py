"""ORACLE TEST INFRASTRUCTURE -- the parity checker, never the product.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package.  Two CPU implementations live here:

* ``Port`` -- ``oracle/psf_port.c``: a plain-C restatement of the reference's
  codec arithmetic (FIXING_FLOAT fixing_float.h:18-101, CRC32C crc32c.cc:292-335,
  NOISE add_noise.h:29-39).  Builds from this repo alone; travels to the GPU box.
* ``Ref`` -- ``oracle/_ref/libpsref.so``: the reference's UNMODIFIED filter
  headers + filter.cc + crc32c.cc compiled from /root/reference against
  ``oracle/ref_stub``.  Used to generate and re-check the
  golden fixtures in tests/golden/ and to pin ``Port``.

``keycache.KeyCacheModel`` restates the KEY_CACHING state machine
(key_caching.h:9-75) in Python for small message sequences.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
PORT_SO = os.path.join(HERE, "_port", "libpsf_port.so")
REF_SO = os.path.join(HERE, "_ref", "libpsref.so")

DT_FLOAT, DT_DOUBLE = 9, 10
KEY_CACHING, COMPRESSING, FIXING_FLOAT, NOISE = 1, 2, 3, 4

PORT_OK, PORT_ERR_ARG, PORT_ERR_NBYTES, PORT_ERR_BIN = 0, -1, -2, -3


def build(ref: bool | None = None) -> None:
    """Compile the C restatement (always) and the reference harness (when
    /root/reference is present)."""
    subprocess.check_call(["make", "-s", "-C", HERE, "port"])
    if ref is None:
        ref = os.path.isdir("/root/reference/src/filter")
    if ref:
        subprocess.check_call(["make", "-s", "-C", HERE, "ref"])
        if os.path.exists(os.path.join(os.path.dirname(HERE), "parameter_server_amd", "libpsf.so")):
            subprocess.check_call(["make", "-s", "-C", HERE, "adapter"])


def _np_dtype(dt: int):
    return np.float32 if dt == DT_FLOAT else np.float64


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


def _uncompress(fn, b, cap):
    a = np.frombuffer(bytes(b) + b"\0", dtype=np.uint8)  # never hand out a NULL pointer
    n = C.c_size_t(0)
    hdr = np.empty(0, np.uint8)
    st = fn(_ptr(a), a.size - 1, _ptr(hdr), 0, C.byref(n))
    if st != -2:
        return st, b""
    if n.value > cap:
        return -2, b""
    out = np.empty(max(n.value, 1), dtype=np.uint8)
    st = fn(_ptr(a), a.size - 1, _ptr(out), n.value, C.byref(n))
    return st, (out[:n.value].tobytes() if st == 0 else b"")


class Port:
    """ctypes view of oracle/psf_port.c."""

    def __init__(self, path: str = PORT_SO):
        if not os.path.exists(path):
            build(ref=False)
        L = self.lib = C.CDLL(path)
        L.port_ff_encode.argtypes = [C.c_void_p, C.c_size_t, C.c_int, C.c_int, C.c_int,
                                     C.POINTER(C.c_float), C.c_int, C.POINTER(C.c_float),
                                     C.c_int32, C.c_void_p]
        L.port_ff_encode.restype = C.c_int
        L.port_ff_decode.argtypes = [C.c_void_p, C.c_size_t, C.c_int, C.c_int, C.c_float,
                                     C.c_float, C.c_void_p]
        L.port_ff_decode.restype = C.c_int
        L.port_ff_ratio.argtypes = [C.c_int]
        L.port_ff_ratio.restype = C.c_double
        L.port_crc32c.argtypes = [C.c_void_p, C.c_size_t]
        L.port_crc32c.restype = C.c_uint32
        L.port_key_signature.argtypes = [C.c_void_p, C.c_size_t]
        L.port_key_signature.restype = C.c_uint32
        L.port_lcg_state.argtypes = [C.c_int32, C.c_uint64]
        L.port_lcg_state.restype = C.c_uint32
        L.port_add_noise.argtypes = [C.c_void_p, C.c_size_t, C.c_int, C.c_float, C.c_float]
        L.port_add_noise.restype = C.c_int
        L.port_snappy_compress.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p]
        L.port_snappy_compress.restype = C.c_size_t
        L.port_snappy_uncompress.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t,
                                             C.POINTER(C.c_size_t)]
        L.port_snappy_uncompress.restype = C.c_int
        L.port_ordered_match.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p, C.c_size_t,
                                         C.c_void_p, C.c_int, C.c_int, C.c_int]
        L.port_ordered_match.restype = C.c_size_t
        L.port_ftrl_update.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p, C.c_void_p,
                                       C.c_void_p, C.c_int, C.c_float, C.c_float, C.c_float, C.c_float,
                                       C.POINTER(C.c_int64), C.POINTER(C.c_float), C.POINTER(C.c_float)]
        L.port_ftrl_update.restype = C.c_int
        L.port_decode_quotient_mismatches.argtypes = [C.c_int]
        L.port_decode_quotient_mismatches.restype = C.c_long

    def ff_encode(self, x: np.ndarray, nb: int, seed: int, mn=None, mx=None):
        """Returns (status, codes:uint8[n*nb], min, max)."""
        x = np.ascontiguousarray(x)
        dt = DT_FLOAT if x.dtype == np.float32 else DT_DOUBLE
        cmn = C.c_float(0.0 if mn is None else mn)
        cmx = C.c_float(0.0 if mx is None else mx)
        out = np.empty(x.size * max(nb, 0), dtype=np.uint8)
        st = self.lib.port_ff_encode(_ptr(x), x.size, dt, nb, mn is not None, C.byref(cmn),
                                     mx is not None, C.byref(cmx), C.c_int32(seed), _ptr(out))
        return st, out, cmn.value, cmx.value

    def ff_decode(self, code: np.ndarray, nb: int, mn: float, mx: float, dtype=np.float32):
        code = np.ascontiguousarray(code, dtype=np.uint8)
        dt = DT_FLOAT if np.dtype(dtype) == np.float32 else DT_DOUBLE
        out = np.empty(code.size // nb if nb > 0 else 0, dtype=dtype)
        st = self.lib.port_ff_decode(_ptr(code), code.size, dt, nb, mn, mx, _ptr(out))
        return st, out

    def crc32c(self, b) -> int:
        b = np.frombuffer(bytes(b), dtype=np.uint8) if not isinstance(b, np.ndarray) else b
        b = np.ascontiguousarray(b).view(np.uint8)
        return int(self.lib.port_crc32c(_ptr(b), b.size))

    def key_signature(self, keys: np.ndarray) -> int:
        b = np.ascontiguousarray(keys).view(np.uint8)
        return int(self.lib.port_key_signature(_ptr(b), b.size))

    def lcg_state(self, seed: int, k: int) -> int:
        return int(self.lib.port_lcg_state(C.c_int32(seed), k))

    def ratio(self, nb: int) -> float:
        return float(self.lib.port_ff_ratio(nb))

    def decode_quotient_mismatches(self, nb: int) -> int:
        """Codes of num_bytes nb where the device decode's fma-corrected
        quotient differs from r / ratio (exhaustive over all 2^(8nb) codes)."""
        return int(self.lib.port_decode_quotient_mismatches(nb))

    def add_noise(self, x: np.ndarray, mean: float, sd: float) -> np.ndarray:
        y = np.array(x, copy=True)
        dt = DT_FLOAT if y.dtype == np.float32 else DT_DOUBLE
        st = self.lib.port_add_noise(_ptr(y), y.size, dt, mean, sd)
        assert st == 0
        return y

    def snappy_compress(self, b) -> bytes:
        """snappy 1.1.8 RawCompress restated (oracle/snappy_port.c)."""
        a = np.frombuffer(bytes(b), dtype=np.uint8)
        out = np.empty(32 + a.size + a.size // 6, dtype=np.uint8)
        n = self.lib.port_snappy_compress(_ptr(a) if a.size else None, a.size, _ptr(out))
        return out[:n].tobytes()

    def snappy_uncompress(self, b, cap: int = 1 << 26):
        """(status, bytes): 0 ok, -1 bad header, -2 declared length > cap, -3 bad body."""
        return _uncompress(self.lib.port_snappy_uncompress, b, cap)

    def ordered_match(self, src_key, src_val, dst_key, dst_val, k=1, op=0) -> int:
        """ParallelOrderedMatch; dst_val is updated in place; returns *n."""
        sk = np.ascontiguousarray(src_key, np.uint64)
        dk = np.ascontiguousarray(dst_key, np.uint64)
        sv = np.ascontiguousarray(src_val)
        assert dst_val.flags.c_contiguous and dst_val.dtype == sv.dtype
        dt = DT_FLOAT if sv.dtype == np.float32 else DT_DOUBLE
        return int(self.lib.port_ordered_match(_ptr(sk), sk.size, _ptr(sv), _ptr(dk), dk.size,
                                               _ptr(dst_val), k, dt, op))


class FtrlModel:
    """KVMap<Key, float, FTRLEntry, SGDState> restated for tests: a key ->
    entry map (the reference's unordered_map, kv_map.h:65) in numpy arrays,
    updated by oracle/psf_port.c's port_ftrl_update (async_sgd.h:137-151)."""

    def __init__(self, port: "Port", lr_type=2, alpha=0.01, beta=10.0, lambda1=0.0, lambda2=0.0):
        self.port = port
        self.decay = 0 if lr_type == 1 else 1
        self.alpha, self.beta = np.float32(alpha), np.float32(beta)
        self.l1, self.l2 = np.float32(lambda1), np.float32(lambda2)
        self.index = {}
        cap = 1 << 10
        self.w = np.zeros(cap, np.float32)
        self.z = np.zeros(cap, np.float32)
        self.sqrt_n = np.zeros(cap, np.float32)
        self.nnz = C.c_int64(0)
        self.weight_sum = C.c_float(0)
        self.delta_sum = C.c_float(0)

    def _entries(self, keys):
        idx = np.empty(len(keys), np.int64)
        for i, k in enumerate(keys.tolist()):
            e = self.index.get(k)
            if e is None:
                e = self.index[k] = len(self.index)
            idx[i] = e
        if len(self.index) > self.w.size:
            cap = 1 << (len(self.index) - 1).bit_length()
            for a in ("w", "z", "sqrt_n"):
                old = getattr(self, a)
                new = np.zeros(cap, np.float32)
                new[:old.size] = old
                setattr(self, a, new)
        return idx

    def push(self, keys: np.ndarray, grad: np.ndarray) -> int:
        idx = self._entries(np.asarray(keys, np.uint64))
        g = np.ascontiguousarray(grad, np.float32)
        return self.port.lib.port_ftrl_update(_ptr(idx), idx.size, _ptr(g), _ptr(self.w), _ptr(self.z),
                                              _ptr(self.sqrt_n), self.decay, self.alpha, self.beta,
                                              self.l1, self.l2, C.byref(self.nnz),
                                              C.byref(self.weight_sum), C.byref(self.delta_sum))

    def pull(self, keys: np.ndarray) -> np.ndarray:
        out = np.zeros(len(keys), np.float32)
        for i, k in enumerate(np.asarray(keys, np.uint64).tolist()):
            e = self.index.get(k)
            if e is not None:
                out[i] = self.w[e]
        return out


class Ref:
    """ctypes view of oracle/_ref/libpsref.so (reference headers, unmodified).

    Message-level API mirroring Message/Task/FilterConfig plus a RemoteNode-like
    chain driver; see oracle/ref_harness.cc."""

    def __init__(self, path: str = REF_SO):
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} (build with `make -C oracle ref`)")
        L = self.lib = C.CDLL(path)
        vp, sz, u64 = C.c_void_p, C.c_size_t, C.c_uint64
        sig = {
            "psref_last_error": ([], C.c_char_p),
            "psref_set_time": ([C.c_int64], None),
            "psref_crc32c": ([vp, sz], C.c_uint32),
            "psref_node_new": ([], vp),
            "psref_node_free": ([vp], None),
            "psref_msg_new": ([C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, u64, u64], vp),
            "psref_msg_free": ([vp], None),
            "psref_msg_clone": ([vp], vp),
            "psref_msg_set_key": ([vp, vp, sz, C.c_int], None),
            "psref_msg_add_value": ([vp, vp, sz, C.c_int], None),
            "psref_msg_key_bytes": ([vp], sz),
            "psref_msg_has_key_flag": ([vp], C.c_int),
            "psref_msg_key_type": ([vp], C.c_int),
            "psref_msg_copy_key": ([vp, vp], None),
            "psref_msg_num_values": ([vp], C.c_int),
            "psref_msg_value_bytes": ([vp, C.c_int], sz),
            "psref_msg_copy_value": ([vp, C.c_int, vp], None),
            "psref_msg_add_filter": ([vp, C.c_int], C.c_int),
            "psref_fc_set_num_bytes": ([vp, C.c_int, C.c_int], None),
            "psref_fc_set_clear_cache": ([vp, C.c_int, C.c_int], None),
            "psref_fc_set_noise": ([vp, C.c_int, C.c_float, C.c_float], None),
            "psref_fc_add_fixed_point": ([vp, C.c_int, C.c_int, C.c_float, C.c_int, C.c_float], None),
            "psref_fc_num_fixed_point": ([vp, C.c_int], C.c_int),
            "psref_fc_get_fixed_point": ([vp, C.c_int, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_float),
                                          C.POINTER(C.c_int), C.POINTER(C.c_float)], None),
            "psref_fc_get_signature": ([vp, C.c_int, C.POINTER(C.c_uint32)], C.c_int),
            "psref_fc_num_uncompressed": ([vp, C.c_int], C.c_int),
            "psref_fc_uncompressed": ([vp, C.c_int, C.c_int], u64),
            "psref_node_encode": ([vp, vp], C.c_int),
            "psref_node_decode": ([vp, vp], C.c_int),
            "psref_snappy_max": ([sz], sz),
            "psref_snappy_compress": ([vp, sz, vp], sz),
            "psref_snappy_uncompress": ([vp, sz, vp, sz, C.POINTER(sz)], C.c_int),
        }
        for name, (a, r) in sig.items():
            f = getattr(L, name)
            f.argtypes = a
            f.restype = r

    # -- thin helpers -------------------------------------------------------
    def set_time(self, t: int) -> None:
        self.lib.psref_set_time(t)

    def crc32c(self, b: bytes) -> int:
        a = np.frombuffer(bytes(b), dtype=np.uint8)
        return int(self.lib.psref_crc32c(_ptr(a) if a.size else None, a.size))

    def snappy_compress(self, b: bytes) -> bytes:
        a = np.frombuffer(bytes(b), dtype=np.uint8)
        out = np.empty(self.lib.psref_snappy_max(a.size), dtype=np.uint8)
        n = self.lib.psref_snappy_compress(_ptr(a) if a.size else None, a.size, _ptr(out))
        return out[:n].tobytes()

    def snappy_uncompress(self, b, cap: int = 1 << 26):
        return _uncompress(self.lib.psref_snappy_uncompress, b, cap)

    def last_error(self) -> str:
        return self.lib.psref_last_error().decode()

    def msg_new(self, request=True, push=False, has_param=True, key_channel=0, key_range=None):
        kr = key_range
        return self.lib.psref_msg_new(int(request), int(has_param), int(push), key_channel,
                                      int(kr is not None), 0 if kr is None else kr[0],
                                      0 if kr is None else kr[1])

    def msg_values(self, m):
        out = []
        for i in range(self.lib.psref_msg_num_values(m)):
            b = np.empty(self.lib.psref_msg_value_bytes(m, i), dtype=np.uint8)
            if b.size:
                self.lib.psref_msg_copy_value(m, i, _ptr(b))
            out.append(b)
        return out

    def msg_key(self, m):
        b = np.empty(self.lib.psref_msg_key_bytes(m), dtype=np.uint8)
        if b.size:
            self.lib.psref_msg_copy_key(m, _ptr(b))
        return b

    def fixed_points(self, m, idx):
        res = []
        for k in range(self.lib.psref_fc_num_fixed_point(m, idx)):
            hm, mn, hx, mx = C.c_int(), C.c_float(), C.c_int(), C.c_float()
            self.lib.psref_fc_get_fixed_point(m, idx, k, C.byref(hm), C.byref(mn), C.byref(hx), C.byref(mx))
            res.append((bool(hm.value), mn.value, bool(hx.value), mx.value))
        return res

    def signature(self, m, idx):
        s = C.c_uint32()
        has = self.lib.psref_fc_get_signature(m, idx, C.byref(s))
        return (bool(has), int(s.value))

    def ff_roundtrip(self, x: np.ndarray, nb: int, seed: int, fixed=None):
        """Run one FIXING_FLOAT-only message through encode then decode on a
        fresh node pair.  Returns dict(status, codes, min, max, decoded)."""
        L = self.lib
        self.set_time(seed)
        snd, rcv = L.psref_node_new(), L.psref_node_new()
        m = self.msg_new()
        dt = DT_FLOAT if x.dtype == np.float32 else DT_DOUBLE
        L.psref_msg_add_value(m, _ptr(x) if x.size else None, x.nbytes, dt)
        fi = L.psref_msg_add_filter(m, FIXING_FLOAT)
        L.psref_fc_set_num_bytes(m, fi, nb)
        if fixed is not None:
            mn, mx = fixed
            L.psref_fc_add_fixed_point(m, fi, mn is not None, 0.0 if mn is None else mn,
                                       mx is not None, 0.0 if mx is None else mx)
        res = {"status": 0}
        try:
            if L.psref_node_encode(snd, m) != 0:
                res.update(status=-1, error=self.last_error())
                return res
            res["codes"] = self.msg_values(m)[0]
            fp = self.fixed_points(m, fi)
            res["min"], res["max"] = fp[0][1], fp[0][3]
            w = L.psref_msg_clone(m)
            try:
                if L.psref_node_decode(rcv, w) != 0:
                    res.update(status=-2, error=self.last_error())
                    return res
                res["decoded"] = self.msg_values(w)[0].view(x.dtype)
            finally:
                L.psref_msg_free(w)
            return res
        finally:
            L.psref_msg_free(m)
            L.psref_node_free(snd)
            L.psref_node_free(rcv)
