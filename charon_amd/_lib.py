"""ctypes binding of libhipbls.so (include/hipbls.h).

The library is built in-tree (charon_amd/lib/libhipbls.so, see charon_amd/build.py).  There is
no CPU fallback: if the library or a gfx950 device is missing, every entry point raises
HipBlsUnavailable.
"""

from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libhipbls.so")

# status codes (include/hipbls.h enum hbls_status)
OK = 0
BAD_PUBKEY = 1
BAD_SIGNATURE = 2
NOT_VERIFIED = 3
COMBINE_FAILED = 4
BAD_SECRET = 5
BAD_INPUT = 6

EXPORTS = (
    "hbls_init", "hbls_last_error", "hbls_available", "hbls_verify_batch", "hbls_threshold_aggregate_batch",
    "hbls_aggregate_batch", "hbls_verify_aggregate_batch", "hbls_sign_batch", "hbls_secret_to_public_key_batch",
    "hbls_threshold_split", "hbls_recover_secret", "hbls_hash_to_g2_device", "hbls_verify_device",
    "hbls_threshold_aggregate_device", "hbls_slot_device", "hbls_hm_entry_bytes", "hbls_sync",
    "hbls_timing", "hbls_timing_read",
)


class HipBlsUnavailable(RuntimeError):
    pass


class HipBlsRuntimeError(RuntimeError):
    pass


_lock = threading.Lock()
_lib = None


def _declare(lib):
    P = ctypes.c_void_p
    SZ = ctypes.c_size_t
    U32 = ctypes.c_uint32
    sig = {
        "hbls_init": ([ctypes.c_int], ctypes.c_int),
        "hbls_last_error": ([], ctypes.c_char_p),
        "hbls_available": ([], ctypes.c_int),
        "hbls_verify_batch": ([P, P, P, P, P, SZ, P], ctypes.c_int),
        "hbls_threshold_aggregate_batch": ([P, P, P, SZ, P, P], ctypes.c_int),
        "hbls_aggregate_batch": ([P, P, SZ, P, P], ctypes.c_int),
        "hbls_verify_aggregate_batch": ([P, P, P, P, P, P, SZ, P], ctypes.c_int),
        "hbls_sign_batch": ([P, P, P, P, SZ, P, P], ctypes.c_int),
        "hbls_secret_to_public_key_batch": ([P, SZ, P, P], ctypes.c_int),
        "hbls_threshold_split": ([P, P, U32, U32, P, P], ctypes.c_int),
        "hbls_recover_secret": ([P, P, SZ, P, P], ctypes.c_int),
        "hbls_hash_to_g2_device": ([P, P, P, SZ, P, P], ctypes.c_int),
        "hbls_verify_device": ([P, P, P, P, SZ, P, P], ctypes.c_int),
        "hbls_threshold_aggregate_device": ([P, P, P, SZ, SZ, P, P, P], ctypes.c_int),
        "hbls_slot_device": ([P, P, P, SZ, P, P, P, P, SZ, P, P, P, P, SZ, SZ, P, P, P], ctypes.c_int),
        "hbls_hm_entry_bytes": ([], SZ),
        "hbls_sync": ([P], ctypes.c_int),
        "hbls_timing": ([ctypes.c_int], ctypes.c_int),
        "hbls_timing_read": ([P, SZ, P], ctypes.c_int),
    }
    for name, (args, res) in sig.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res


def load_library(path: str = LIB_PATH):
    """Load the shared library without touching the GPU (safe on CPU-only hosts)."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(path):
                raise HipBlsUnavailable(f"{path} not built; run `python -m charon_amd.build`")
            lib = ctypes.CDLL(path)
            _declare(lib)
            _lib = lib
        return _lib


def lib():
    """The library, initialised on a gfx950 device; raises if that is impossible."""
    L = load_library()
    if L.hbls_init(-1) != 0:
        raise HipBlsUnavailable("hipbls: " + L.hbls_last_error().decode(errors="replace"))
    return L


def check(rc: int):
    if rc != 0:
        raise HipBlsRuntimeError("hipbls: " + _lib.hbls_last_error().decode(errors="replace"))
