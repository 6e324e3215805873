"""charon_amd: MI355X-native BLS12-381 backend for charon's tbls hot path.

Layout:
  csrc/      gfx950 HIP kernels + C ABI (libhipbls.so; header include/hipbls.h)
  _lib.py    ctypes binding (fails loudly without the library / a gfx950 device)
  tbls.py    mirror of charon's tbls.Implementation (tbls/tbls.go:27-141) + batch API
  slot.py    device-resident slot pipeline (batch verify + threshold aggregate) used by bench.py
"""

__all__ = ["tbls"]
