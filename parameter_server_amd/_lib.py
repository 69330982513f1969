"""ctypes binding of libpsf.so (include/psf.h).

The library is built in-tree (parameter_server_amd/libpsf.so) by
``parameter_server_amd.build``.  There is no CPU fallback: if the shared
library is missing, loading fails loudly.
"""
from __future__ import annotations

import ctypes as C
import os

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libpsf.so")
# tuning experiments only (tools/build_variants.sh): load an in-tree variant build
LIB_PATH = os.environ.get("PSF_LIBRARY_VARIANT") or LIB_PATH

PSF_OK = 0
PSF_ERR_ARG = -1
PSF_ERR_NBYTES = -2
PSF_ERR_BIN = -3
PSF_ERR_HIP = -4
PSF_ERR_CHECK = -5
PSF_ERR_UNSUPPORTED = -6
PSF_ERR_TIMEOUT = -7  # reserved: no entry point returns it
PSF_STREAM_GIVEN, PSF_STREAM_OWN, PSF_STREAM_SHARED = 0, 1, 2
PSF_EXCHANGE_RCCL, PSF_EXCHANGE_HOST = 0, 1

DT_UINT64, DT_FLOAT, DT_DOUBLE, DT_CHAR = 8, 9, 10, 11
KEY_CACHING, COMPRESSING, FIXING_FLOAT, NOISE = 1, 2, 3, 4
LOC_HOST, LOC_DEVICE = 0, 1


class PsfError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"psf error {code}: {msg}")
        self.code = code


class FixedPoint(C.Structure):
    _fields_ = [("has_min", C.c_int32), ("has_max", C.c_int32),
                ("min_value", C.c_float), ("max_value", C.c_float)]


vp, sz, i32, u32, u64 = C.c_void_p, C.c_size_t, C.c_int32, C.c_uint32, C.c_uint64
PI = C.POINTER(C.c_int)

# name -> (argtypes, restype); the exported surface of include/psf.h
SIGNATURES = {
    "psf_last_error": ([], C.c_char_p),
    "psf_version": ([], C.c_char_p),
    "psf_set_clock": ([C.c_int, C.c_int64], None),
    "psf_set_default_device": ([C.c_int], C.c_int),
    "psf_default_device": ([], C.c_int),
    "psf_context_create": ([C.c_int, vp, C.c_int, C.POINTER(vp)], C.c_int),
    "psf_context_destroy": ([vp], C.c_int),
    "psf_context_sync": ([vp], C.c_int),
    "psf_copy_to_host": ([vp, vp, vp, sz], C.c_int),
    "psf_copy_to_host_async": ([vp, vp, vp, sz], C.c_int),
    "psf_host_buffer_alloc": ([vp, sz, C.POINTER(vp), C.POINTER(vp)], C.c_int),
    "psf_host_buffer_release": ([vp], C.c_int),
    "psf_ff_encode": ([vp, vp, sz, C.c_int, C.c_int, C.POINTER(FixedPoint), i32, vp], C.c_int),
    "psf_ff_encode_async": ([vp, vp, sz, C.c_int, C.c_int, C.POINTER(FixedPoint), i32, vp, vp, vp], C.c_int),
    "psf_ff_decode": ([vp, vp, sz, C.c_int, C.c_int, C.c_float, C.c_float, vp], C.c_int),
    "psf_ff_decode_async": ([vp, vp, sz, C.c_int, C.c_int, vp, vp], C.c_int),
    "psf_crc32c": ([vp, vp, sz, C.POINTER(u32)], C.c_int),
    "psf_key_signature": ([vp, vp, sz, C.POINTER(u32)], C.c_int),
    "psf_snappy_max_compressed_length": ([sz], sz),
    "psf_snappy_compress": ([vp, vp, sz, vp, C.POINTER(sz)], C.c_int),
    "psf_snappy_uncompressed_length": ([vp, vp, sz, C.POINTER(sz)], C.c_int),
    "psf_snappy_compress_stored": ([vp, vp, sz, sz, C.POINTER(sz)], C.c_int),
    "psf_snappy_stored_capacity": ([sz], sz),
    "psf_snappy_uncompress": ([vp, vp, sz, vp, sz, C.POINTER(sz)], C.c_int),
    "psf_node_create": ([vp, C.POINTER(vp)], C.c_int),
    "psf_node_destroy": ([vp], C.c_int),
    "psf_node_encode": ([vp, vp], C.c_int),
    "psf_node_decode": ([vp, vp], C.c_int),
    "psf_msg_create": ([C.c_int, C.c_int, C.c_int, i32, C.c_int, u64, u64, C.POINTER(vp)], C.c_int),
    "psf_msg_destroy": ([vp], C.c_int),
    "psf_msg_clone": ([vp, C.POINTER(vp)], C.c_int),
    "psf_msg_set_key": ([vp, vp, sz, C.c_int, C.c_int], C.c_int),
    "psf_msg_add_value": ([vp, vp, sz, C.c_int, C.c_int], C.c_int),
    "psf_msg_set_value": ([vp, C.c_int, vp, sz, C.c_int], C.c_int),
    "psf_msg_recv_frame": ([vp, vp, sz, C.c_int], C.c_int),
    "psf_task_serialize": ([vp, vp, sz, C.POINTER(sz)], C.c_int),
    "psf_task_parse": ([vp, sz, C.POINTER(vp)], C.c_int),
    "psf_msg_key": ([vp, C.POINTER(vp), C.POINTER(sz), PI], C.c_int),
    "psf_msg_key_info": ([vp, PI, PI], C.c_int),
    "psf_msg_key_channel": ([vp, C.POINTER(i32)], C.c_int),
    "psf_task_value_count": ([vp, PI], C.c_int),
    "psf_msg_num_values": ([vp], C.c_int),
    "psf_msg_value": ([vp, C.c_int, C.POINTER(vp), C.POINTER(sz), PI], C.c_int),
    "psf_msg_add_filter": ([vp, C.c_int], C.c_int),
    "psf_fc_set_num_bytes": ([vp, C.c_int, C.c_int], C.c_int),
    "psf_fc_set_clear_cache": ([vp, C.c_int, C.c_int], C.c_int),
    "psf_fc_set_noise": ([vp, C.c_int, C.c_float, C.c_float], C.c_int),
    "psf_fc_add_fixed_point": ([vp, C.c_int, C.POINTER(FixedPoint)], C.c_int),
    "psf_fc_num_fixed_point": ([vp, C.c_int], C.c_int),
    "psf_fc_fixed_point": ([vp, C.c_int, C.c_int, C.POINTER(FixedPoint)], C.c_int),
    "psf_fc_signature": ([vp, C.c_int, PI, C.POINTER(u32)], C.c_int),
    "psf_fc_set_signature": ([vp, C.c_int, C.c_int, u32], C.c_int),
    "psf_fc_num_uncompressed": ([vp, C.c_int], C.c_int),
    "psf_fc_uncompressed": ([vp, C.c_int, C.c_int, C.POINTER(u64)], C.c_int),
    "psf_fc_add_uncompressed": ([vp, C.c_int, u64], C.c_int),
    "psf_node_roundtrip": ([vp, vp, C.POINTER(vp), C.c_int, C.c_int, C.POINTER(vp)], C.c_int),
    "psf_node_roundtrip_ex": ([vp, vp, C.POINTER(vp), C.c_int, C.c_int, C.POINTER(vp), C.POINTER(vp)], C.c_int),
    "psf_nodes_roundtrip_ex": ([C.POINTER(vp), C.POINTER(vp), C.POINTER(vp), C.c_int, PI, C.c_int, C.c_int,
                                C.POINTER(vp), C.POINTER(vp)], C.c_int),
    "psf_nodes_roundtrip_opts": ([C.POINTER(vp), C.POINTER(vp), C.POINTER(vp), C.c_int, PI, C.c_int, C.c_int,
                                  C.c_int, C.POINTER(vp), C.POINTER(vp)], C.c_int),
    "psf_range_even_divide": ([u64, u64, u64, u64, C.POINTER(u64), C.POINTER(u64)], C.c_int),
    "psf_msg_slice": ([vp, vp, C.POINTER(u64), C.c_int, C.c_int, C.POINTER(vp), PI], C.c_int),
    "psf_msgs_slice": ([vp, C.POINTER(vp), C.c_int, C.POINTER(u64), C.c_int, C.c_int, C.POINTER(vp), PI],
                       C.c_int),
    "psf_node_set_defer_dequant": ([vp, C.c_int], C.c_int),
    "psf_msg_pending": ([vp, C.c_int, PI, C.POINTER(C.c_float), C.POINTER(C.c_float)], C.c_int),
    "psf_msg_materialize": ([vp, vp], C.c_int),
    "psf_ordered_match": ([vp, vp, sz, vp, vp, sz, vp, C.c_int, C.c_int, C.c_int, C.POINTER(sz)], C.c_int),
    "psf_ff_decode_match": ([vp, vp, sz, vp, C.c_int, C.c_float, C.c_float, vp, sz, vp, C.c_int, C.c_int,
                             C.POINTER(sz)], C.c_int),
    "psf_msg_ordered_match": ([vp, vp, C.c_int, vp, sz, vp, C.c_int, C.c_int, C.c_int, C.POINTER(sz)],
                              C.c_int),
    "psf_kvmap_create": ([vp, sz, C.c_int, C.c_double, C.c_double, C.c_double, C.c_double, C.POINTER(vp)],
                         C.c_int),
    "psf_kvmap_destroy": ([vp], C.c_int),
    "psf_kvmap_set_value": ([vp, vp], C.c_int),
    "psf_kvmap_get_value": ([vp, vp], C.c_int),
    "psf_kvmap_push": ([vp, vp, sz, vp], C.c_int),
    "psf_kvmap_pull": ([vp, vp, sz, vp], C.c_int),
    "psf_kvmap_stats": ([vp, C.POINTER(C.c_int64), C.POINTER(C.c_double), C.POINTER(C.c_double),
                         C.POINTER(u64)], C.c_int),
    "psf_nodes_encode": ([C.POINTER(vp), C.POINTER(vp), C.c_int], C.c_int),
    "psf_nodes_decode": ([C.POINTER(vp), C.POINTER(vp), C.c_int], C.c_int),
    "psf_nodes_roundtrip": ([C.POINTER(vp), C.POINTER(vp), C.POINTER(vp), C.c_int, C.c_int], C.c_int),
    "psf_spill_pack": ([vp, C.POINTER(vp), PI, PI, C.c_int, C.c_int, C.POINTER(C.c_int64), C.POINTER(vp)],
                       C.c_int),
    "psf_spill_fill": ([vp, vp], C.c_int),
    "psf_spill_destroy": ([vp], C.c_int),
    "psf_spill_unpack": ([vp, vp, C.c_int, C.POINTER(C.c_int64), C.POINTER(vp), PI, C.c_int, PI], C.c_int),
    "psf_router_create": ([vp, C.POINTER(u64), C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(vp)], C.c_int),
    "psf_router_destroy": ([vp], C.c_int),
    "psf_router_keep_encoded": ([vp, C.c_int], C.c_int),
    "psf_router_encode": ([vp, C.POINTER(vp), C.c_int, C.POINTER(C.c_int64)], C.c_int),
    "psf_router_fill": ([vp, vp], C.c_int),
    "psf_router_decode_local": ([vp], C.c_int),
    "psf_router_decode_received": ([vp, vp, C.POINTER(C.c_int64)], C.c_int),
    "psf_router_step": ([vp, C.POINTER(vp), C.c_int, C.c_int], C.c_int),
    "psf_router_host_stats": ([vp, C.POINTER(C.c_int64)], C.c_int),
    "psf_router_host_stats_reset": ([vp], C.c_int),
    "psf_context_host_stats": ([vp, C.POINTER(C.c_int64), C.POINTER(C.c_int64)], C.c_int),
    "psf_context_host_stats_reset": ([vp], C.c_int),
    "psf_context_set_cache_limit": ([vp, u64, u64], C.c_int),
    "psf_context_memory_stats": ([vp, C.POINTER(u64)], C.c_int),
    "psf_set_device_cache_limit": ([C.c_int, u64, u64], C.c_int),
    "psf_device_memory_stats": ([C.c_int, C.POINTER(u64)], C.c_int),
    "psf_router_num_results": ([vp], C.c_int),
    "psf_router_result": ([vp, C.c_int, PI, C.POINTER(vp)], C.c_int),
    "psf_router_num_encoded": ([vp], C.c_int),
    "psf_router_encoded": ([vp, C.c_int, C.POINTER(i32), PI, C.POINTER(vp)], C.c_int),
    "psf_exchange_unique_id": ([vp, sz], C.c_int),
    "psf_exchange_create": ([vp, C.c_int, C.c_int, C.c_char_p, C.c_int, vp, u64, u64, C.POINTER(vp)], C.c_int),
    "psf_exchange_destroy": ([vp], C.c_int),
    "psf_exchange_stats": ([vp, C.POINTER(C.c_int64)], C.c_int),
    "psf_router_set_exchange": ([vp, vp], C.c_int),
    "psf_exchange_data_stats": ([vp, C.POINTER(C.c_int64)], C.c_int),
    "psf_router_set_store": ([vp, vp], C.c_int),
    "psf_router_pull": ([vp, C.POINTER(vp), C.c_int, C.c_int], C.c_int),
    "psf_router_pull_encode": ([vp, C.POINTER(vp), C.c_int, C.POINTER(C.c_int64)], C.c_int),
    "psf_router_pull_serve": ([vp, vp, C.POINTER(C.c_int64), C.POINTER(C.c_int64)], C.c_int),
    "psf_router_pull_finish": ([vp, vp, C.POINTER(C.c_int64)], C.c_int),
    "psf_router_num_pulled": ([vp], C.c_int),
    "psf_router_pulled": ([vp, C.c_int, C.POINTER(i32), C.POINTER(vp)], C.c_int),
    "psf_profile_enable": ([vp, C.c_int], C.c_int),
    "psf_profile_stride": ([vp, C.c_int], C.c_int),
    "psf_profile_reset": ([vp], C.c_int),
    "psf_profile_read": ([vp, C.c_int, C.POINTER(C.c_int64), C.POINTER(C.c_double),
                          C.POINTER(C.c_double)], C.c_int),
    "psf_profile_kernel_name": ([C.c_int], C.c_char_p),
}

KERNELS = ("ff_minmax_partials", "ff_encode", "ff_decode", "crc32c_chunks", "noise_add",
           "snappy_compress", "snappy_decompress", "ordered_match", "kvmap_push", "kvmap_get",
           "ff_decode_minmax", "ff_minmax_encode")
OP_ASSIGN, OP_PLUS, OP_MINUS, OP_TIMES, OP_DIVIDE = 0, 1, 2, 3, 4

_lib = None


def lib() -> C.CDLL:
    """Load libpsf.so (once).  Raises if the HIP library was not built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing: run `python -m parameter_server_amd.build` "
                              "(there is no CPU fallback)")
        L = C.CDLL(LIB_PATH)
        variant = LIB_PATH != os.path.join(os.path.dirname(os.path.abspath(__file__)), "libpsf.so")
        for name, (args, res) in SIGNATURES.items():
            if variant and not hasattr(L, name):
                continue  # an older build loaded for an A/B run lacks the newer entry points
            f = getattr(L, name)
            f.argtypes = args
            f.restype = res
        _lib = L
    return _lib


def check(status: int) -> int:
    if status < 0:
        raise PsfError(status, lib().psf_last_error().decode())
    return status
