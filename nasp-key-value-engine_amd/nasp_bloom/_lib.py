"""ctypes binding of libnasp_bloom.so (the C ABI in include/nasp_bloom.h).

This is the Python-side binding a maintainer would add; it
fails loudly when the HIP library is missing -- there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# NB_LIB: another build of the same library (same-box A/B of kernel variants)
LIB_PATH = os.environ.get("NB_LIB") or os.path.join(PKG_ROOT, "build", "libnasp_bloom.so")

NB_OK = 0
NB_ERR_ARG = -1
NB_ERR_HIP = -2
NB_ERR_NODEV = -3
NB_ERR_UNSUPPORTED = -4

BUILD_OVERWRITE = 1

FLAVOR_LIBSTDCXX = 0
FLAVOR_MSVC_FNV1A = 1
FLAVOR_MURMUR3_X64_128 = 2  # non-parity (include/nasp_bloom.h)

# every symbol include/nasp_bloom.h declares: (restype, argtypes)
_u8p = C.c_void_p
_SIGS = {
    "nb_abi_version": (C.c_int, []),
    "nb_device_count": (C.c_int, []),
    "nb_last_error": (C.c_char_p, []),
    "nb_shutdown": (C.c_int, []),
    "nb_device_build_count": (C.c_uint64, []),
    "nb_device_merkle_count": (C.c_uint64, []),
    "nb_set_knob": (C.c_int, [C.c_char_p, C.c_uint64]),
    "nb_get_knob": (C.c_int, [C.c_char_p, C.POINTER(C.c_uint64)]),
    "nb_size_of_bitset": (C.c_uint32, [C.c_uint32, C.c_double]),
    "nb_num_hashes": (C.c_uint32, [C.c_uint32, C.c_uint32]),
    "nb_seed_from_time": (C.c_uint64, [C.c_uint32]),
    "nb_std_hash": (C.c_uint64, [C.c_void_p, C.c_uint64, C.c_int]),
    "nb_build": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint64, C.c_uint32,
                           C.c_uint32, C.c_uint64, C.c_int, C.c_void_p, C.c_int]),
    "nb_build_sharded": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint64, C.c_uint32,
                                   C.c_uint32, C.c_uint64, C.c_int, C.c_void_p, C.c_int]),
    "nb_build_cpu": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint64, C.c_uint32,
                               C.c_uint32, C.c_uint64, C.c_int, C.c_void_p]),
    "nb_probe_cpu": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint64, C.c_uint32,
                               C.c_uint32, C.c_uint64, C.c_int, C.c_void_p, C.c_void_p]),
    "nb_probe": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint64, C.c_uint32,
                           C.c_uint32, C.c_uint64, C.c_int, C.c_void_p, C.c_void_p, C.c_int]),
    "nb_build_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint64, C.c_uint32,
                                  C.c_uint32, C.c_uint64, C.c_int, C.c_void_p, C.c_void_p]),
    "nb_build_device_ex": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint64, C.c_uint32,
                                     C.c_uint32, C.c_uint64, C.c_int, C.c_void_p, C.c_uint32,
                                     C.c_void_p]),
    "nb_probe_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint64, C.c_uint32,
                                  C.c_uint32, C.c_uint64, C.c_int, C.c_void_p, C.c_void_p,
                                  C.c_void_p]),
    "nb_or_merge_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32,
                                     C.c_uint64, C.c_void_p]),
    "nb_serialized_size": (C.c_size_t, [C.c_uint32]),
    "nb_serialize": (C.c_size_t, [C.c_uint32, C.c_uint32, C.c_double, C.c_uint32, C.c_uint64,
                                  C.c_void_p, C.c_void_p]),
    "nb_deserialize": (C.c_int, [C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p, C.c_void_p,
                                 C.c_void_p, C.c_void_p, C.c_void_p]),
    "nb_framed_filter_size": (C.c_size_t, [C.c_uint32, C.c_int, C.c_uint32]),
    "nb_frame_filter": (C.c_size_t, [C.c_uint32, C.c_uint32, C.c_double, C.c_uint32, C.c_uint64,
                                     C.c_void_p, C.c_int, C.c_uint32, C.c_void_p]),
    "nb_frame_filter_device": (C.c_int, [C.c_uint32, C.c_uint32, C.c_double, C.c_uint32,
                                         C.c_uint64, C.c_void_p, C.c_int, C.c_uint32,
                                         C.c_void_p, C.c_void_p]),
    "nb_builder_create": (C.c_int, [C.c_uint32, C.c_uint32, C.c_uint64, C.c_int, C.c_void_p,
                                    C.c_int, C.POINTER(C.c_void_p)]),
    "nb_builder_add": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64]),
    "nb_builder_add_batch": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32,
                                       C.c_uint64]),
    "nb_builder_add_batch_async": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32,
                                             C.c_uint64]),
    "nb_builder_sync_uploads": (C.c_int, [C.c_void_p]),
    "nb_builder_finish": (C.c_int, [C.c_void_p, C.c_void_p]),
    "nb_builder_destroy": (C.c_int, [C.c_void_p]),
    "nb_host_alloc": (C.c_int, [C.c_size_t, C.POINTER(C.c_void_p)]),
    "nb_host_free": (C.c_int, [C.c_void_p]),
    "nb_merkle_tree_size": (C.c_uint64, [C.c_uint64]),
    "nb_merkle_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint64, C.c_int,
                                   C.c_void_p, C.c_void_p]),
    "nb_merkle": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint64, C.c_int, C.c_void_p,
                            C.c_void_p, C.c_void_p, C.c_int]),
    "nb_merkle_cpu": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint64, C.c_int, C.c_void_p,
                                C.c_void_p, C.c_void_p]),
}

FRAME_RAW = 0
FRAME_COMP = 1

_LIB = None


class NaspBloomError(RuntimeError):
    pass


def lib() -> C.CDLL:
    """Load the HIP library (raises if it has not been built)."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise NaspBloomError(
                f"{LIB_PATH} is missing: build it with `make -C {PKG_ROOT}` "
                "(or __graft_entry__.build()); there is no CPU fallback")
        h = C.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(h, name)
            fn.restype = res
            fn.argtypes = args
        if h.nb_abi_version() != 1:
            raise NaspBloomError("ABI version mismatch")
        _LIB = h
    return _LIB


def check(rc: int, what: str) -> None:
    if rc != NB_OK:
        msg = lib().nb_last_error().decode(errors="replace")
        raise NaspBloomError(f"{what} failed (rc={rc}): {msg}")
