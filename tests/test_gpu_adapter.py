"""GPU: the reference-side drop-in (include/psf_ps_filter.h) compiled against
the PS filter interface, run side by side with the reference's unmodified
FixingFloatFilter on the same PS::Message (oracle/adapter_harness.cc):
identical codes, side-info and decoded values, and each side decodes the
other's wire output identically."""
import ctypes as C
import os

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

SO = os.path.join(ROOT, "oracle", "_ref", "libpsadapter.so")


@pytest.fixture(scope="module")
def harness():
    if not os.path.exists(SO):
        pytest.skip("adapter harness not built (make -C oracle adapter)")
    L = C.CDLL(SO)
    L.psadapter_compare_ff.argtypes = [C.c_void_p, C.c_size_t, C.c_int, C.c_int, C.c_int64,
                                       C.c_int, C.c_float, C.c_int, C.c_float]
    L.psadapter_compare_ff.restype = C.c_int
    L.psadapter_last_error.restype = C.c_char_p
    return L


def _run(L, x, nb, seed, mn=None, mx=None):
    dt = 9 if x.dtype == np.float32 else 10
    return L.psadapter_compare_ff(x.ctypes.data, x.nbytes, dt, nb, seed,
                                  mn is not None, 0.0 if mn is None else mn,
                                  mx is not None, 0.0 if mx is None else mx)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("nb", [1, 2, 3, 5])
def test_adapter_matches_reference_filter(harness, dtype, nb):
    x = np.random.default_rng(nb).standard_normal(100_003).astype(dtype)
    rc = _run(harness, x, nb, 12345)
    assert rc == 0, (rc, harness.psadapter_last_error())
    rc = _run(harness, x, nb, -77, -1.0, 1.0)
    assert rc == 0, (rc, harness.psadapter_last_error())


def test_adapter_rejects_like_reference(harness):
    x = np.full(64, 40.0, np.float32)  # fixing_float.h:71 CHECK_GT(bin, 0)
    assert _run(harness, x, 1, 1) == -1


def _sig(L):
    L.psadapter_compare_compress.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_int]
    L.psadapter_compare_compress.restype = C.c_int
    L.psadapter_compare_noise.argtypes = [C.c_void_p, C.c_size_t, C.c_int, C.c_float, C.c_float]
    L.psadapter_compare_noise.restype = C.c_int


@pytest.mark.parametrize("nkeys", [0, 5, 3000, 200_000])
def test_adapter_compressing_matches_reference(harness, nkeys):
    """CompressingFilter (compressing.h:8-37): same snappy bytes for keys and
    values, same uncompressed_size, each side decodes the other's output."""
    _sig(harness)
    rng = np.random.default_rng(nkeys)
    keys = np.sort(rng.choice(10**9, size=nkeys, replace=False)).astype(np.uint64)
    for vals in (rng.standard_normal(nkeys + 7).astype(np.float32),
                 np.clip(rng.standard_normal(70_000) * 20 + 128, 0, 255).astype(np.uint8),
                 np.zeros(0, np.float32)):
        rc = harness.psadapter_compare_compress(keys.ctypes.data if nkeys else None, keys.nbytes,
                                                vals.ctypes.data if vals.size else None, vals.nbytes, 9)
        assert rc == 0, (rc, harness.psadapter_last_error())


@pytest.mark.parametrize("dtype", [np.float32])
def test_adapter_noise_matches_reference(harness, dtype):
    _sig(harness)
    x = np.linspace(-1, 1, 5001).astype(dtype)
    rc = harness.psadapter_compare_noise(x.ctypes.data, x.nbytes, 9, 0.5, 2.0)
    assert rc == 0, (rc, harness.psadapter_last_error())
