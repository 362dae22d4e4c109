"""roctx ranges around the phases of VecEnvRLGames.step (SURVEY §5 tracing: "roctx ranges around
pre / physics / post"), so `rocprofv3 --marker-trace --kernel-trace` shows which kernels each
phase of the reference's step sequence (vec_env_rlgames.py:56-78) launched.

The ranges come from ROCm's roctx library (librocprofiler-sdk-roctx, the one rocprofv3
intercepts). They are on by default when the library loads; MI_ROCTX=0 turns them off. A range
costs two host calls (~1 us); it has no effect on the device work.
"""
from __future__ import annotations

import ctypes as C
import os
from contextlib import contextmanager

_LIB = None
_TRIED = False
_CANDIDATES = ("librocprofiler-sdk-roctx.so.1", "/opt/rocm/lib/librocprofiler-sdk-roctx.so.1",
               "libroctx64.so.4", "/opt/rocm/lib/libroctx64.so.4")


def lib():
    """The roctx library, or None (not installed, or MI_ROCTX=0)."""
    global _LIB, _TRIED
    if _TRIED:
        return _LIB
    _TRIED = True
    if os.environ.get("MI_ROCTX", "1") == "0":
        return None
    for name in _CANDIDATES:
        try:
            L = C.CDLL(name)
            L.roctxRangePushA.argtypes = [C.c_char_p]
            L.roctxRangePushA.restype = C.c_int
            L.roctxRangePop.argtypes = []
            L.roctxRangePop.restype = C.c_int
            _LIB = L
            break
        except (OSError, AttributeError):
            continue
    return _LIB


@contextmanager
def trace_range(name: str):
    """roctxRangePushA(name) ... roctxRangePop() (no-op without the library)."""
    L = lib()
    if L is None:
        yield
        return
    L.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        L.roctxRangePop()
