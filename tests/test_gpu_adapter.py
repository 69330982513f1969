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
