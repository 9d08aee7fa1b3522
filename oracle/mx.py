"""MX-fp8 format restated on the CPU (oracle — TEST INFRASTRUCTURE ONLY).

The reference has no fp8 path: every model runs in bf16 (main.py:808-820,
torch_dtype=DTYPE). The fp8 mode is BASELINE.json configs[4] ("Apple-DFN5B-H
fp8 weights on CDNA4 fp8 MFMA"), so parity for it is two-level:
  * the quantiser is pinned BIT-EXACTLY to this restatement of the format
    documented in include/mme.h (config 5 section): OCP e4m3fn values with
    round-to-nearest-even after clamping to +-448 (torch.float8_e4m3fn's cast,
    itself checked against an exhaustive nearest-value table in
    tests/test_mx_oracle.py), E8M0 block scales chosen as the smallest power
    of two that keeps the block's absmax within 448;
  * the fp8 GEMM against an fp64 product of the dequantised operands, and the
    fp8 towers against the fp32 oracle encoders with the tolerance stated in
    tests/test_gpu_mx.py ("parity unpinned" against the reference itself,
    which has no such mode).
"""
from __future__ import annotations

import numpy as np
import torch


def e4m3_table() -> np.ndarray:
    """float value of every e4m3fn byte (0x7f / 0xff = NaN)."""
    v = np.arange(256)
    s = np.where(v >> 7, -1.0, 1.0)
    e = (v >> 3) & 15
    m = v & 7
    mag = np.where(e == 0, m * 2.0 ** -9, (1 + m / 8.0) * 2.0 ** (e - 7.0))
    out = s * mag
    out[(v & 0x7f) == 0x7f] = np.nan
    return out.astype(np.float32)


def scale_bytes(amax: np.ndarray) -> np.ndarray:
    """E8M0 byte per block: clamp(expfield(a) - 8 + (mantissa(a) > 0x600000), 1, 254); 127 for a == 0."""
    a = np.asarray(amax, dtype=np.float32)
    u = a.view(np.uint32)
    e = ((u >> 23) & 255).astype(np.int64) - 8 + ((u & 0x7FFFFF) > 0x600000)
    e = np.clip(e, 1, 254)
    return np.where(a == 0, 127, e).astype(np.uint8)


def encode_e4m3(x: np.ndarray) -> np.ndarray:
    """RNE to e4m3fn after clamping to +-448 (u8 bytes)."""
    xc = np.clip(np.asarray(x, dtype=np.float32), -448.0, 448.0)
    return torch.from_numpy(np.ascontiguousarray(xc)).to(torch.float8_e4m3fn).view(torch.uint8).numpy()


def srow(r: np.ndarray) -> np.ndarray:
    """Position of row r in a scale plane (include/mme.h, round 4): inside each 128-row group, row r
    is stored at (r % 32) * 4 + (r % 128) // 32 (the 4 rows i * 32 + r of an MFMA lane adjacent)."""
    r = np.asarray(r)
    return (r & ~127) | ((r & 31) << 2) | ((r >> 5) & 3)


def quantize(x: np.ndarray, rows_pad: int = 0):
    """x: float32 [R, K] (bf16-valued) -> (q u8 [R, K], scales u8 [K/32, rows_pad], rows in srow order)."""
    x = np.asarray(x, dtype=np.float32)
    R, K = x.shape
    assert K % 32 == 0
    rp = rows_pad or max(256, (R + 255) // 256 * 256)
    blocks = x.reshape(R, K // 32, 32)
    sb = scale_bytes(np.abs(blocks).max(axis=2))                      # [R, K/32]
    scaled = np.ldexp(blocks, (127 - sb.astype(np.int32))[:, :, None]).astype(np.float32)
    q = encode_e4m3(scaled.reshape(R, K))
    planes = np.zeros((K // 32, rp), dtype=np.uint8)
    planes[:, srow(np.arange(R))] = sb.T
    return q, planes


def dequantize(q: np.ndarray, planes: np.ndarray, rows: int) -> np.ndarray:
    """mx8 -> float64 [rows, K]."""
    tab = e4m3_table().astype(np.float64)
    vals = tab[q[:rows]]
    K = vals.shape[1]
    sc = np.ldexp(1.0, planes[:, srow(np.arange(rows))].T.astype(np.int64) - 127)   # [rows, K/32]
    return vals * np.repeat(sc, 32, axis=1)[:, :K]


def gemm_ref(aq, asc, M, bq, bsc, N) -> np.ndarray:
    """fp64 product of the dequantised operands: A [M,K] . B[N,K]^T."""
    return dequantize(aq, asc, M) @ dequantize(bq, bsc, N).T
