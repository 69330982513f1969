"""parameter_server_amd -- MI355X-native (HIP/gfx950) filter codec chain of
dmlc/parameter_server (src/filter): FIXING_FLOAT, KEY_CACHING, COMPRESSING,
NOISE behind the reference's Filter/RemoteNode plugin surface.

The product is libpsf.so (HIP kernels + C++ host layer, C ABI in
include/psf.h).  This package only binds it; there is no CPU fallback.
"""
from ._lib import (COMPRESSING, DT_CHAR, DT_DOUBLE, DT_FLOAT, DT_UINT64, FIXING_FLOAT,  # noqa: F401
                   KEY_CACHING, NOISE, PSF_ERR_ARG, PSF_ERR_BIN, PSF_ERR_CHECK, PSF_ERR_HIP,
                   PSF_ERR_NBYTES, PSF_ERR_UNSUPPORTED, PSF_OK, PsfError, lib)

__all__ = ["lib", "PsfError", "FIXING_FLOAT", "KEY_CACHING", "COMPRESSING", "NOISE"]


def __getattr__(name):
    # torch-dependent wrappers load lazily so `import parameter_server_amd`
    # stays cheap for the C-ABI symbol checks
    if name in ("Context", "Message", "RemoteNode", "KVMap", "set_clock", "copy_out"):
        from . import filter as _f
        return getattr(_f, name)
    raise AttributeError(name)
