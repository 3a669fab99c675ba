"""ctypes wrapper of oracle/libflsfast*.so: the FastLanes-shaped CPU decoder
timed as bench.py's cpu_baseline (flsfast.cpp).  TEST / BENCH INFRASTRUCTURE
ONLY; checked against the oracle (flsref.c) by tests/test_flsfast.py.

Two builds: libflsfast.so with the reference's flags for cwida/FastLanes
(generic x86-64, no -march=native: vcpkg_ports/fastlanes/portfile.cmake) and
libflsfast_v4.so (x86-64-v4, AVX-512), loaded only where the CPU has it.
"""
from __future__ import annotations

import ctypes as C
from pathlib import Path

import numpy as np

_HERE = Path(__file__).resolve().parent
BUILDS = {"generic": _HERE / "libflsfast.so", "avx512": _HERE / "libflsfast_v4.so"}
_libs: dict[str, C.CDLL] = {}


def host_has_avx512() -> bool:
    try:
        flags = next(l for l in open("/proc/cpuinfo") if l.startswith("flags")).split()
    except (OSError, StopIteration):
        return False
    return all(f in flags for f in ("avx512f", "avx512bw", "avx512dq", "avx512vl"))


def available() -> list[str]:
    return [b for b, p in BUILDS.items() if p.exists() and (b != "avx512" or host_has_avx512())]


def lib(build: str = "generic") -> C.CDLL:
    if build not in _libs:
        p = BUILDS[build]
        if not p.exists():
            raise ImportError(f"{p} not built: run `make -C {_HERE}`")
        lib_ = C.CDLL(str(p))
        lib_.flsfast_decode.restype = C.c_int64
        lib_.flsfast_decode.argtypes = [C.c_void_p, C.c_uint64, C.c_uint32, C.c_uint32, C.c_int,
                                        C.POINTER(C.c_void_p), C.POINTER(C.c_void_p)]
        lib_.flsfast_heap_bytes.restype = C.c_uint64
        lib_.flsfast_heap_bytes.argtypes = [C.c_void_p, C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32]
        _libs[build] = lib_
    return _libs[build]


class Decoder:
    """Output buffers for row groups [rg0, rg1) of an image (numpy, reused
    across calls: the bench times decode passes over the same buffers)."""

    def __init__(self, img, ptr: int, length: int, out_bytes: list[int], rows: int, rg0: int, rg1: int,
                 build: str = "generic"):
        self._keep = img
        self.ptr, self.len, self.rg0, self.rg1 = ptr, length, rg0, rg1
        self.lib = lib(build)
        self.outs = [np.empty(max(1, rows * ob), dtype=np.uint8) for ob in out_bytes]
        hb = [self.lib.flsfast_heap_bytes(ptr, length, rg0, rg1, c) for c in range(len(out_bytes))]
        self.heaps = [np.empty(h + 64, dtype=np.uint8) if h else None for h in hb]
        self._o = (C.c_void_p * len(self.outs))(*[o.ctypes.data for o in self.outs])
        self._h = (C.c_void_p * len(self.outs))(*[h.ctypes.data if h is not None else None for h in self.heaps])

    def decode(self, nthreads: int) -> int:
        n = self.lib.flsfast_decode(self.ptr, self.len, self.rg0, self.rg1, nthreads, self._o, self._h)
        if n < 0:
            raise ValueError("flsfast_decode failed")
        return n
