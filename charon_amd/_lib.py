"""ctypes binding of libhipbls.so (include/hipbls.h).

The library is built in-tree (charon_amd/lib/libhipbls.so, see charon_amd/build.py).  There is
no CPU fallback: if the library or a gfx950 device is missing, every entry point raises
HipBlsUnavailable.
"""

from __future__ import annotations

import ctypes
import os
import re
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
UNCHECKED = 7

EXPORTS = (
    "hbls_init", "hbls_last_error", "hbls_available", "hbls_device_count", "hbls_verify_batch",
    "hbls_threshold_aggregate_batch", "hbls_aggregate_batch", "hbls_verify_aggregate_batch", "hbls_sign_batch",
    "hbls_secret_to_public_key_batch", "hbls_threshold_split", "hbls_recover_secret", "hbls_hash_to_g2_device",
    "hbls_verify_device", "hbls_threshold_aggregate_device", "hbls_verify_aggregate_device", "hbls_slot_device",
    "hbls_hm_entry_bytes", "hbls_sync", "hbls_status_bitmap",
    "hbls_timing", "hbls_timing_read", "hbls_comm_id_bytes", "hbls_comm_unique_id", "hbls_comm_init",
    "hbls_allgather_device", "hbls_comm_size", "hbls_comm_destroy", "hbls_stats", "hbls_fe_batch", "hbls_slot_msm", "hbls_adaptive", "hbls_rlc_lanes", "hbls_ta_joint", "hbls_attestation_signing_roots",
    "hbls_signing_roots", "hbls_attestation_signing_roots_device", "hbls_pk_entry_bytes",
    "hbls_decompress_pubkeys_device", "hbls_pubkey_cache_add", "hbls_pubkey_cache_clear", "hbls_pubkey_cache_size",
    "hbls_debug_split", "hbls_build_id", "hbls_sig_cache", "hbls_duty_signing_roots",
    "hbls_single_max", "hbls_dec_pair_max", "hbls_tune", "hbls_verify_batch_first_error",
    "hbls_verify_device_first_error",
)

ALL_DEVICES = 0xFFFFFFFF


class HblsSlot(ctypes.Structure):
    """struct hbls_slot (include/hipbls.h)."""
    _fields_ = [(name, ctypes.c_void_p if kind == "p" else ctypes.c_size_t) for name, kind in (
        ("msgs", "p"), ("msg_off", "p"), ("msg_len", "p"), ("n_msgs", "s"), ("hm", "p"),
        ("pks", "p"), ("sigs", "p"), ("msg_idx", "p"), ("n", "s"), ("vgrp_off", "p"), ("n_vgroups", "s"),
        ("vstatus", "p"), ("ta_sigs", "p"), ("ta_src", "p"), ("ta_idx", "p"), ("grp_off", "p"), ("n_groups", "s"),
        ("n_ta_partials", "s"), ("ta_out", "p"), ("ta_status", "p"), ("dv_pks", "p"), ("agg_vstatus", "p"),
        ("pk_table", "p"), ("pk_table_st", "p"), ("dv_pk_table", "p"), ("dv_pk_table_st", "p"))]


class HipBlsUnavailable(RuntimeError):
    pass


class HipBlsRuntimeError(RuntimeError):
    pass


BUILD_ID_PREFIX = "hbls-build:"


def source_build_id(root: str = "") -> str:
    """sha256 (first 16 hex digits) over every file of charon_amd/csrc and include/hipbls.h, names
    and contents, in sorted order: what charon_amd/build.py embeds as hbls_build_id()."""
    import hashlib

    root = root or os.path.dirname(_HERE)
    csrc = os.path.join(root, "charon_amd", "csrc")
    files = sorted(os.path.join(csrc, f) for f in os.listdir(csrc) if f.endswith((".h", ".hip")))
    files.append(os.path.join(root, "include", "hipbls.h"))
    h = hashlib.sha256()
    for f in files:
        h.update(os.path.relpath(f, root).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    return h.hexdigest()[:16]


def embedded_build_id(path: str) -> str:
    """The build id string inside a built library file, read from its bytes (no loading)."""
    with open(path, "rb") as f:
        data = f.read()
    m = re.search(rb"hbls-build:[0-9a-f]{16}(\+[A-Za-z0-9_=,.+-]*)?", data)
    return m.group(0).decode() if m else ""


def check_build_id(lib_id: str, root: str = "") -> None:
    """Raise HipBlsUnavailable unless lib_id was built from the sources in the tree (tuning
    variants carry '+defines' after the hash; only the hash is compared)."""
    want = source_build_id(root)
    got = lib_id[len(BUILD_ID_PREFIX):].split("+", 1)[0] if lib_id.startswith(BUILD_ID_PREFIX) else ""
    if got != want:
        raise HipBlsUnavailable(f"stale libhipbls.so: built from sources {got or '(unknown)'}, the tree is {want}; "
                                "run `python -m charon_amd.build`")


_lock = threading.Lock()
_lib = None


def _declare(lib):
    P = ctypes.c_void_p
    SZ = ctypes.c_size_t
    U32 = ctypes.c_uint32
    sig = {
        "hbls_init": ([ctypes.c_uint32], ctypes.c_int),
        "hbls_last_error": ([], ctypes.c_char_p),
        "hbls_available": ([], ctypes.c_int),
        "hbls_device_count": ([], ctypes.c_int),
        "hbls_verify_batch": ([P, P, P, P, P, SZ, P], ctypes.c_int),
        "hbls_verify_batch_first_error": ([P, P, P, P, P, SZ, P, P, P], ctypes.c_int),
        "hbls_verify_device_first_error": ([P, P, P, P, SZ, P, SZ, P, P, P], ctypes.c_int),
        "hbls_threshold_aggregate_batch": ([P, P, P, SZ, P, P], ctypes.c_int),
        "hbls_aggregate_batch": ([P, P, SZ, P, P], ctypes.c_int),
        "hbls_verify_aggregate_batch": ([P, P, P, P, P, P, SZ, P], ctypes.c_int),
        "hbls_sign_batch": ([P, P, P, P, SZ, P, P], ctypes.c_int),
        "hbls_secret_to_public_key_batch": ([P, SZ, P, P], ctypes.c_int),
        "hbls_threshold_split": ([P, P, U32, U32, P, P], ctypes.c_int),
        "hbls_recover_secret": ([P, P, SZ, P, P], ctypes.c_int),
        "hbls_hash_to_g2_device": ([P, P, P, SZ, P, P], ctypes.c_int),
        "hbls_verify_device": ([P, P, P, P, SZ, P, SZ, P, P], ctypes.c_int),
        "hbls_threshold_aggregate_device": ([P, P, P, SZ, SZ, P, P, P], ctypes.c_int),
        "hbls_verify_aggregate_device": ([P, P, SZ, P, P, P, P], ctypes.c_int),
        "hbls_attestation_signing_roots": ([P, SZ, P, SZ, P, P], ctypes.c_int),
        "hbls_signing_roots": ([P, SZ, P, SZ, P, P], ctypes.c_int),
        "hbls_attestation_signing_roots_device": ([P, SZ, P, SZ, P, P, P], ctypes.c_int),
        "hbls_pk_entry_bytes": ([], SZ),
        "hbls_decompress_pubkeys_device": ([P, SZ, P, P, P], ctypes.c_int),
        "hbls_pubkey_cache_add": ([P, SZ], ctypes.c_int),
        "hbls_pubkey_cache_clear": ([], ctypes.c_int),
        "hbls_pubkey_cache_size": ([], SZ),
        "hbls_debug_split": ([U32], ctypes.c_int),
        "hbls_slot_device": ([ctypes.POINTER(HblsSlot), P], ctypes.c_int),
        "hbls_hm_entry_bytes": ([], SZ),
        "hbls_sync": ([P], ctypes.c_int),
        "hbls_status_bitmap": ([P, SZ, P, P], ctypes.c_int),
        "hbls_timing": ([ctypes.c_int], ctypes.c_int),
        "hbls_timing_read": ([P, P, SZ, P], ctypes.c_int),
        "hbls_comm_id_bytes": ([], SZ),
        "hbls_comm_unique_id": ([P], ctypes.c_int),
        "hbls_comm_init": ([ctypes.c_int, ctypes.c_int, P], ctypes.c_int),
        "hbls_allgather_device": ([P, P, SZ, P], ctypes.c_int),
        "hbls_comm_size": ([], ctypes.c_int),
        "hbls_comm_destroy": ([], ctypes.c_int),
        "hbls_stats": ([P, SZ], ctypes.c_int),
        "hbls_fe_batch": ([SZ], SZ),
        "hbls_slot_msm": ([SZ], SZ),
        "hbls_adaptive": ([ctypes.c_int], ctypes.c_int),
        "hbls_rlc_lanes": ([SZ], SZ),
        "hbls_ta_joint": ([SZ], SZ),
        "hbls_build_id": ([], ctypes.c_char_p),
        "hbls_sig_cache": ([SZ], SZ),
        "hbls_single_max": ([SZ], SZ),
        "hbls_dec_pair_max": ([SZ], SZ),
        "hbls_tune": ([ctypes.c_char_p, SZ, P], ctypes.c_int),
        "hbls_duty_signing_roots": ([ctypes.c_int, P, P, P, SZ, P, SZ, P, P, P], ctypes.c_int),
    }
    for name, (args, res) in sig.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res


def load_library(path: str = ""):
    """Load the shared library without touching the GPU (safe on CPU-only hosts).  HBLS_LIBRARY
    names a tuning variant built by charon_amd.build (default: the in-tree product library).
    Refuses a library whose embedded build id (hbls_build_id) differs from the tree's sources."""
    path = path or os.environ.get("HBLS_LIBRARY") or LIB_PATH
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(path):
                raise HipBlsUnavailable(f"{path} not built; run `python -m charon_amd.build`")
            # One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64.so.  Loaded after
            # ours, it would bind to the runtime this library pulled in from /opt/rocm and find no
            # device ("No HIP GPUs are available"); loaded first, the library binds to torch's (same
            # soname) and both see the GPU.  Importing torch does not touch the GPU.
            try:
                import torch  # noqa: F401
            except ImportError:
                pass
            lib = ctypes.CDLL(path)
            _declare(lib)
            # provenance: the library must have been built from the sources in this tree
            if os.path.isdir(os.path.join(os.path.dirname(_HERE), "charon_amd", "csrc")):
                check_build_id(lib.hbls_build_id().decode())
            _lib = lib
        return _lib


def lib(device_mask: int = 0):
    """The library, initialised on its gfx950 devices (mask 0: HBLS_DEVICE_MASK or device 0);
    raises if that is impossible."""
    L = load_library()
    if L.hbls_init(device_mask) != 0:
        raise HipBlsUnavailable("hipbls: " + L.hbls_last_error().decode(errors="replace"))
    return L


def timing_read(L, max_n: int = 1 << 16):
    """[(kernel name, ms)] of the launches recorded since hbls_timing(1)."""
    names = (ctypes.c_char_p * max_n)()
    ms = (ctypes.c_float * max_n)()
    n = ctypes.c_size_t(0)
    check(L.hbls_timing_read(names, ms, max_n, ctypes.byref(n)))
    return [(names[i].decode(), float(ms[i])) for i in range(n.value)]


def check(rc: int):
    if rc != 0:
        raise HipBlsRuntimeError("hipbls: " + _lib.hbls_last_error().decode(errors="replace"))
