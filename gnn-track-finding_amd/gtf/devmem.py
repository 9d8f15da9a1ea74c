"""Device arrays without a framework: plain allocations from libgtf's HIP runtime
(gtf_malloc / gtf_memcpy_*, include/gtf.h), for the drop-in stage CLIs.

A drop-in CLI runs one stage over one directory and exits (run_gnn_trackml_mod.sh calls
each stage once per iteration). On the MI355X box `import torch` plus its first device
tensor take 1.9-2.0 s, most of the extrapolation CLI's 2.3 s, while the HIP runtime
comes up in 0.25-0.45 s (tools/cold_start.py). So ``DeviceGraph(mem="hip")``, which
gtf.dropin.run_dir uses in a process that has not imported torch, keeps its arrays in
:class:`HipArray` instead of torch tensors: the same kernels on the same bytes, through
the C-ABI only. Arrays expose the few tensor methods DeviceGraph's stage path uses
(``data_ptr``, ``numel``, ``element_size``, ``numpy``)."""
from __future__ import annotations

import ctypes
import sys

import numpy as np

from . import _native as nat


def default_mem() -> str:
    """the allocator a stage entry point picks when the caller gives none: "hip" in a
    process that has not imported torch (a drop-in CLI), else "torch", whose HIP runtime
    libgtf then shares. GTF_DROPIN_MEM=torch|hip overrides."""
    import os
    m = os.environ.get("GTF_DROPIN_MEM", "")
    if m in ("torch", "hip"):
        return m
    return "torch" if "torch" in sys.modules else "hip"


class HipArray:
    """a 1-D device array: an owning allocation, or a view into one (arena members)"""

    def __init__(self, n: int, dtype, base: "HipArray" = None, offset: int = 0):
        self.dtype = np.dtype(dtype)
        self.n = int(n)
        self._lib = nat.lib(lean=True)
        self._base = base
        if base is None:
            p = ctypes.c_void_p()
            nat.check(self._lib.gtf_malloc(ctypes.byref(p), ctypes.c_size_t(self.nbytes)))
            self._ptr = p.value
        else:
            self._ptr = base._ptr + offset

    @classmethod
    def from_numpy(cls, a: np.ndarray, stream=None) -> "HipArray":
        a = np.ascontiguousarray(a).reshape(-1)
        d = cls(a.size, a.dtype)
        d.upload(a, stream)
        return d

    @classmethod
    def zeros(cls, n: int, dtype, stream=None) -> "HipArray":
        d = cls(n, dtype)
        nat.check(d._lib.gtf_memset(ctypes.c_void_p(d._ptr), 0, ctypes.c_size_t(d.nbytes), stream))
        return d

    def view(self, offset: int, n: int, dtype) -> "HipArray":
        """n elements of dtype at byte offset (shares this allocation)"""
        return HipArray(n, dtype, base=self._base or self, offset=(self._ptr - (self._base or self)._ptr) + offset)

    @property
    def nbytes(self) -> int:
        return self.n * self.dtype.itemsize

    def data_ptr(self) -> int:
        return self._ptr

    def numel(self) -> int:
        return self.n

    def element_size(self) -> int:
        return self.dtype.itemsize

    def upload(self, a: np.ndarray, stream=None):
        a = np.ascontiguousarray(a, dtype=self.dtype).reshape(-1)
        if a.size != self.n:
            raise ValueError("upload of %d elements into a %d-element device array" % (a.size, self.n))
        nat.check(self._lib.gtf_memcpy_htod(ctypes.c_void_p(self._ptr), a.ctypes.data_as(ctypes.c_void_p),
                                            ctypes.c_size_t(self.nbytes), stream))
        # the copy is stream-ordered: keep the host buffer alive until the next synchronisation
        self._pending = a

    def copy_from(self, other: "HipArray", stream=None):
        if other.nbytes != self.nbytes:
            raise ValueError("device copy between arrays of %d and %d bytes" % (other.nbytes, self.nbytes))
        nat.check(self._lib.gtf_memcpy_dtod(ctypes.c_void_p(self._ptr), ctypes.c_void_p(other._ptr),
                                            ctypes.c_size_t(self.nbytes), stream))

    def numpy(self, stream=None) -> np.ndarray:
        """a host copy (synchronises the stream)"""
        out = np.empty(self.n, self.dtype)
        nat.check(self._lib.gtf_memcpy_dtoh(out.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(self._ptr),
                                            ctypes.c_size_t(self.nbytes), stream))
        self._pending = None
        return out

    def free(self):
        if self._base is None and self._ptr is not None and not sys.is_finalizing():
            self._lib.gtf_free(ctypes.c_void_p(self._ptr))
        self._ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:   # interpreter shutdown: the runtime may be gone
            pass
