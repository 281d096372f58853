"""roctx ranges for the validators and the trainer (tracing).

`with roctx.range("gemm.timed"): ...` pushes a named range that rocprofv3
(`--marker-trace`) and rocprof timelines show over the GPU kernels it
encloses.  The library is dlopen'ed lazily; without it (build box) the ranges
are no-ops, so instrumented code runs unchanged everywhere.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
from typing import Optional

_LIBS = ("librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so", "libroctx64.so.4")
_lib: Optional[ctypes.CDLL] = None
_tried = False


def _load() -> Optional[ctypes.CDLL]:
    global _lib, _tried
    if _tried:
        return _lib
    _tried = True
    if os.environ.get("MXK8S_ROCTX", "1") == "0":
        return None
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    for name in _LIBS:
        for cand in (os.path.join(rocm, "lib", name), name):
            try:
                L = ctypes.CDLL(cand)
            except OSError:
                continue
            L.roctxRangePushA.argtypes = [ctypes.c_char_p]
            L.roctxRangePushA.restype = ctypes.c_int
            L.roctxRangePop.restype = ctypes.c_int
            L.roctxMarkA.argtypes = [ctypes.c_char_p]
            _lib = L
            return _lib
    return None


def available() -> bool:
    return _load() is not None


def push(name: str) -> None:
    L = _load()
    if L is not None:
        L.roctxRangePushA(name.encode())


def pop() -> None:
    L = _load()
    if L is not None:
        L.roctxRangePop()


def mark(name: str) -> None:
    L = _load()
    if L is not None:
        L.roctxMarkA(name.encode())


@contextlib.contextmanager
def range(name: str):  # noqa: A001 - mirrors the roctx API name
    push(name)
    try:
        yield
    finally:
        pop()
