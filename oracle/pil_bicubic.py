"""PIL-exact bicubic resize + HF rescale/normalise, in numpy (integer arithmetic).

Restates what processor(images=...) does in the reference (main.py:407):
transformers PilBackend._preprocess (image_processing_backends.py:619-656)
-> np_resize -> PIL Image.resize(BICUBIC) (Pillow libImaging/Resample.c:
precompute_coeffs, normalize_coeffs_8bpc, ImagingResampleHorizontal_8bpc /
Vertical_8bpc; PRECISION_BITS = 22, bicubic a = -0.5), then
image_transforms.rescale (float64 * 1/255 -> float32) and normalize
((x - mean) / std in float32). Pinned by tests/golden/preprocess.npz.
"""
from __future__ import annotations

import math

import numpy as np

PREC = 22


def _bicubic(x: float) -> float:
    a = -0.5
    if x < 0.0:
        x = -x
    if x < 1.0:
        return ((a + 2.0) * x - (a + 3.0)) * x * x + 1
    if x < 2.0:
        return (((x - 5) * x + 8) * x - 4) * a
    return 0.0


def coeffs(in_size: int, out_size: int):
    """(xmin[out], count[out], int32 kk[out, ksize]) exactly as Pillow computes them."""
    scale = in_size / out_size
    fs = max(scale, 1.0)
    support = 2.0 * fs
    ksize = int(math.ceil(support)) * 2 + 1
    xmin_a = np.zeros(out_size, np.int64)
    cnt_a = np.zeros(out_size, np.int64)
    kk = np.zeros((out_size, ksize), np.int64)
    for xx in range(out_size):
        center = (xx + 0.5) * scale
        ss = 1.0 / fs
        xmin = int(center - support + 0.5)
        xmin = max(xmin, 0)
        xmax = int(center + support + 0.5)
        xmax = min(xmax, in_size) - xmin
        w = [_bicubic((x + xmin - center + 0.5) * ss) for x in range(xmax)]
        ww = 0.0
        for v in w:
            ww += v
        for x in range(xmax):
            k = w[x] / ww if ww != 0.0 else w[x]
            kk[xx, x] = int(-0.5 + k * (1 << PREC)) if k < 0 else int(0.5 + k * (1 << PREC))
        xmin_a[xx], cnt_a[xx] = xmin, xmax
    return xmin_a, cnt_a, kk


def _pass(src: np.ndarray, axis: int, out_size: int) -> np.ndarray:
    """One separable pass over `axis` of a uint8 HxWxC array."""
    xmin, cnt, kk = coeffs(src.shape[axis], out_size)
    s = np.moveaxis(src.astype(np.int64), axis, 0)
    acc = np.full((out_size,) + s.shape[1:], 1 << (PREC - 1), np.int64)
    for j in range(kk.shape[1]):
        valid = j < cnt
        idx = np.where(valid, xmin + j, 0)
        k = np.where(valid, kk[:, j], 0)
        acc += s[idx] * k.reshape((-1,) + (1,) * (s.ndim - 1))
    out = np.clip(acc >> PREC, 0, 255).astype(np.uint8)
    return np.moveaxis(out, 0, axis)


def resize_bicubic(img: np.ndarray, out_h: int, out_w: int) -> np.ndarray:
    """uint8 [H, W, 3] -> uint8 [out_h, out_w, 3]; horizontal pass first, like Pillow."""
    H, W = img.shape[:2]
    x = img
    if out_w != W:
        x = _pass(x, 1, out_w)
    if out_h != H:
        x = _pass(x, 0, out_h)
    return x.copy() if x is img else x


def geometry(H: int, W: int, size: int, mode: str):
    """(rh, rw, top, left): SigLIP square resize, or CLIP shortest-edge resize + center crop
    (transformers get_resize_output_image_size(default_to_square=False), center_crop)."""
    if mode == "square":
        return size, size, 0, 0
    short, long = (W, H) if W <= H else (H, W)
    new_short, new_long = size, int(size * long / short)
    rh, rw = (new_long, new_short) if W <= H else (new_short, new_long)
    return rh, rw, (rh - size) // 2, (rw - size) // 2


def preprocess_u8(img: np.ndarray, size: int, mode: str) -> np.ndarray:
    rh, rw, top, left = geometry(img.shape[0], img.shape[1], size, mode)
    r = resize_bicubic(img, rh, rw)
    return r[top:top + size, left:left + size]


def normalize(u8: np.ndarray, mean, std) -> np.ndarray:
    """uint8 [S,S,3] -> float32 pixel_values [3,S,S] (rescale 1/255 in float64, normalise in float32)."""
    r = (u8.astype(np.float64) * (1 / 255)).astype(np.float32)
    m = np.asarray(mean, np.float32)
    s = np.asarray(std, np.float32)
    return np.ascontiguousarray(((r - m) / s).transpose(2, 0, 1))
