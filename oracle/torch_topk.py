"""torch.topk's CPU row selection (oracle; test infrastructure only).

ctypes binding of oracle/torch_topk.cpp, which calls libstdc++'s std::partial_sort /
std::nth_element + std::sort exactly as torch's CPU topk kernel does
(aten/src/ATen/native/cpu/SortingKernel.cpp topk_impl_loop), so exact ties come out in
torch's order. The reference ranks with torch.topk per row (main.py:335,365,375).
Pinned by tests/golden/torch_topk.npz (torch.topk's own outputs) and the reference's
own results in tests/golden/colpali_full.npz.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "libtorch_topk.so")
_lib = None


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            subprocess.run(["make", "-C", _HERE], check=True, stdout=subprocess.DEVNULL)
        lib = ctypes.CDLL(_LIB)
        lib.oracle_torch_topk.restype = ctypes.c_int
        lib.oracle_torch_topk.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                          ctypes.c_int64, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        _lib = lib
    return _lib


def topk(s: np.ndarray, k: int, sort_k_minus_1: bool = True):
    """(idx int64 [rows, k], val fp32 [rows, k]) of torch.topk(row, k) for every row of s."""
    s = np.ascontiguousarray(s, dtype=np.float32)
    if s.ndim == 1:
        s = s[None]
    rows, n = s.shape
    idx = np.empty((rows, k), np.int64)
    val = np.empty((rows, k), np.float32)
    rc = _load().oracle_torch_topk(s.ctypes.data, rows, n, n, k, int(sort_k_minus_1), idx.ctypes.data,
                                   val.ctypes.data)
    if rc:
        raise ValueError(f"oracle_torch_topk: bad arguments (k={k}, n={n})")
    return idx, val


def hits(s: np.ndarray, tgt_count: int, ks=(1, 5, 10), row_offset: int = 0) -> np.ndarray:
    """[rows, len(ks)] bool: target column block (row + offset) * tgt_count .. + tgt_count in
    torch.topk(row, min(k, n)) -- one selection per k, as compute_metrics_detailed calls it
    (main.py:331-378)."""
    n = s.shape[1]
    rows = np.arange(s.shape[0]) + row_offset
    out = []
    for k in ks:
        idx, _ = topk(s, min(k, n))
        out.append(((idx // tgt_count) == rows[:, None]).any(1))
    return np.stack(out, 1)
