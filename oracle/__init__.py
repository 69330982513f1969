"""ORACLE TEST INFRASTRUCTURE -- the parity checker, never the product.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package.

Parity status: the reference's filter path cannot be built in this image (it
needs glog, gflags, Eigen, the protobuf runtime and protoc-generated code;
SURVEY.md §8(c)), and its own tests hold no vectors for this path
(src/test/fixing_float_test.cc is stale and asserts nothing).  CRC32C is pinned
to the reference's own crc32c.cc, COMPRESSING's codec to snappy 1.1.8 and
NOISE's draws to libstdc++ (the libraries the reference calls); the rest is a
restatement, and parity is UNPINNED by the reference for FIXING_FLOAT,
KEY_CACHING's state machine and COMPRESSING's glue.  What is
here:

* ``Port`` -- ``oracle/psf_port.c`` + ``snappy_port.c``: a plain-C restatement
  of the reference's codec arithmetic (FIXING_FLOAT fixing_float.h:18-101,
  CRC32C crc32c.cc:292-335, NOISE add_noise.h:29-39 over libstdc++'s
  normal_distribution and this libm) and of snappy 1.1.8 (the third-party
  library the reference links for COMPRESSING).  Builds from this repo alone;
  travels to the GPU box.
* ``chain`` -- the message path (Message / RemoteNode / the four filters)
  restated in Python over ``Port``; tests/golden/scenarios.json is its record.
* ``RefCrc32c`` -- ``oracle/_ref/libcrc32c_ref.so``: the reference's own
  src/util/crc32c.cc compiled from /root/reference (it needs nothing else):
  pins CRC32C, KEY_CACHING's signature, against the reference itself.
* ``NoiseStd`` -- ``oracle/_port/libnoise_std.so`` (noise_std.cc): NOISE's
  two libstdc++ calls (std::default_random_engine, std::normal_distribution)
  made as add_noise.h:29-39 makes them, with the reference's flags.
* ``slicing`` -- SliceKOFVMessage / EvenDivide restated in numpy.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
PORT_SO = os.path.join(HERE, "_port", "libpsf_port.so")
CRC_REF_SO = os.path.join(HERE, "_ref", "libcrc32c_ref.so")
NOISE_STD_SO = os.path.join(HERE, "_port", "libnoise_std.so")

DT_FLOAT, DT_DOUBLE = 9, 10
KEY_CACHING, COMPRESSING, FIXING_FLOAT, NOISE = 1, 2, 3, 4

PORT_OK, PORT_ERR_ARG, PORT_ERR_NBYTES, PORT_ERR_BIN = 0, -1, -2, -3


def build(ref: bool | None = None) -> None:
    """Compile the C restatement (always), the reference's crc32c.cc (when
    /root/reference is present) and the adapter harness (when libpsf is
    built)."""
    subprocess.check_call(["make", "-s", "-C", HERE, "port"])
    if ref is None:
        ref = os.path.isfile("/root/reference/src/util/crc32c.cc")
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


class RefCrc32c:
    """ctypes view of oracle/_ref/libcrc32c_ref.so: the reference's own
    crc32c::Value (src/util/crc32c.cc:292-335, compiled in place)."""

    def __init__(self, path: str = CRC_REF_SO):
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} (build with `make -C oracle ref`)")
        self.lib = C.CDLL(path)
        self.lib.ref_crc32c.argtypes = [C.c_void_p, C.c_size_t]
        self.lib.ref_crc32c.restype = C.c_uint32

    def crc32c(self, b) -> int:
        a = np.frombuffer(bytes(b), dtype=np.uint8) if not isinstance(b, np.ndarray) else \
            np.ascontiguousarray(b).view(np.uint8)
        return int(self.lib.ref_crc32c(_ptr(a) if a.size else None, a.size))

    def key_signature(self, keys: np.ndarray) -> int:
        """KEY_CACHING's signature: the first min(bytes, 2048) key bytes (key_caching.h:18)."""
        b = np.ascontiguousarray(keys).view(np.uint8)
        return self.crc32c(b[:2048])


SNAPPY_SO = "/opt/conda/lib/libsnappy.so.1"


class Snappy118:
    """snappy 1.1.8 itself (the third-party library the reference's
    COMPRESSING calls through SArray::CompressTo / UncompressFrom,
    shared_array_inl.h:232-255), through its C API, where the image has it:
    it generated tests/golden/snappy*.npz and pins snappy_port.c."""

    def __init__(self, path: str = SNAPPY_SO):
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        L = self.lib = C.CDLL(path)
        sz = C.c_size_t
        L.snappy_compress.argtypes = [C.c_void_p, sz, C.c_void_p, C.POINTER(sz)]
        L.snappy_max_compressed_length.argtypes = [sz]
        L.snappy_max_compressed_length.restype = sz
        L.snappy_uncompressed_length.argtypes = [C.c_void_p, sz, C.POINTER(sz)]
        L.snappy_uncompress.argtypes = [C.c_void_p, sz, C.c_void_p, C.POINTER(sz)]

    def compress(self, b: bytes) -> bytes:
        a = np.frombuffer(bytes(b) + b"\0", dtype=np.uint8)
        cap = C.c_size_t(self.lib.snappy_max_compressed_length(len(b)))
        out = np.empty(cap.value, np.uint8)
        assert self.lib.snappy_compress(_ptr(a), len(b), _ptr(out), C.byref(cap)) == 0
        return out[:cap.value].tobytes()

    def uncompress(self, b: bytes, cap: int = 1 << 26):
        """(0, bytes) or (status != 0, b"") as RawUncompress accepts / rejects"""
        a = np.frombuffer(bytes(b) + b"\0", dtype=np.uint8)
        n = C.c_size_t()
        if self.lib.snappy_uncompressed_length(_ptr(a), len(b), C.byref(n)) != 0:
            return -1, b""
        if n.value > cap:
            return -2, b""
        out = np.empty(max(n.value, 1), np.uint8)
        if self.lib.snappy_uncompress(_ptr(a), len(b), _ptr(out), C.byref(n)) != 0:
            return -3, b""
        return 0, out[:n.value].tobytes()

    snappy_compress = compress      # Port's names
    snappy_uncompress = uncompress


class NoiseStd:
    """ctypes view of oracle/_port/libnoise_std.so: AddNoise through libstdc++'s
    own engine and distribution (add_noise.h:29-39)."""

    def __init__(self, path: str = NOISE_STD_SO):
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} (build with `make -C oracle port`)")
        self.lib = C.CDLL(path)
        self.lib.noise_std.argtypes = [C.c_void_p, C.c_size_t, C.c_int, C.c_float, C.c_float]
        self.lib.noise_std.restype = C.c_int

    def add_noise(self, x: np.ndarray, mean: float, sd: float) -> np.ndarray:
        y = np.array(x, copy=True)
        dt = DT_FLOAT if y.dtype == np.float32 else DT_DOUBLE
        assert self.lib.noise_std(_ptr(y), y.size, dt, mean, sd) == 0
        return y
