"""Measurement helper: device tensors in a chosen kind of device memory
(tools/membw.hip membw_alloc: 0 hipMalloc, 1 fine-grained, 2 uncached,
3 contiguous), exposed to torch through the CUDA array interface. Round 5
measured the batch kernels' outputs and the builder's frames in uncached
memory (tools/uc_ab.py): no gain in the parse, losses for
partial-line writes, so the library keeps ordinary device memory."""
import ctypes
import os

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_mb = None
UNCACHED = 2


def _lib():
    global _mb
    if _mb is None:
        _mb = ctypes.CDLL(os.path.join(ROOT, "tools", "libmembw.so"))
        _mb.membw_alloc.restype = ctypes.c_void_p
        _mb.membw_alloc.argtypes = [ctypes.c_uint64, ctypes.c_int]
        _mb.membw_free.argtypes = [ctypes.c_void_p]
    return _mb


class _Mem:
    def __init__(self, nbytes, kind):
        self.ptr = _lib().membw_alloc(max(int(nbytes), 1), kind)
        if not self.ptr:
            raise RuntimeError("membw_alloc failed")
        self.__cuda_array_interface__ = {"shape": (max(int(nbytes), 1),), "typestr": "|u1",
                                         "data": (self.ptr, False), "version": 3,
                                         "strides": None}

    def __del__(self):
        if getattr(self, "ptr", None):
            _lib().membw_free(self.ptr)
            self.ptr = None


def empty(shape, dtype=torch.uint8, device="cuda", kind=UNCACHED):
    """Uninitialised tensor of `shape` in membw_alloc memory of `kind` (on the
    current device)."""
    shape = tuple(shape) if isinstance(shape, (tuple, list)) else (int(shape),)
    nbytes = int(np.prod(shape, dtype=np.int64)) * torch.empty((), dtype=dtype).element_size()
    t = torch.as_tensor(_Mem(nbytes, kind), device=device)[:nbytes]
    return t.view(dtype).view(shape)
