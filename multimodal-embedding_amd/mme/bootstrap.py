"""Bootstrap recall on the device.

run_bootstrap_benchmark (main.py:563-660) draws n_iterations resamples of the n
images WITH replacement (main.py:588), re-scores the sampled embeddings
(compute_similarity_scores, main.py:620-624) and runs compute_metrics_detailed
(main.py:305-383) on every resample — hours on the CPU for 1 000 iterations
(README.md:70-72). A resample's score matrices are index gathers of the full
matrices, so here the full T2I [n, n] and I2T [n, 5n] matrices are computed once
(mme_gemm, or MaxSim for ColPali) and each batch of resamples is
mme_gather_scores -> mme_topk_rows_torch (one selection per k, in torch.topk's CPU
order) -> mme_recall_hits_groups; only the 9 x iterations hit counts leave the device.

Sampled positions: resample b's image i is samples[b, i]; its T2I query is that
image's caption-0 row, its I2T targets the 5 positions of that image's captions
(img_to_caps_map, main.py:601-609), I2T-Sym is the transposed T2I matrix
(main.py:624). Ties — a duplicated image scores exactly like its copies — decide
many rows; the reference's torch.topk keeps the copy its libstdc++ partial_sort /
nth_element leaves (a different selection per k), and mme_topk_rows_torch replays
exactly that, so every resample's counts equal the reference's.

The confidence interval (bootstrap_confidence_interval, main.py:259-278: 10 000
resamples of the per-iteration values, 2.5 / 97.5 percentiles) is host statistics
over 9 x n_iterations numbers (the CSV stage), seeded here.
"""
from __future__ import annotations

from typing import Dict, Optional, Sequence

import numpy as np
import torch

from . import ops

KS = (1, 5, 10)
NAMES = [f"{p}_R@{k}" for p in ("T2I", "I2T", "I2T_Sym") for k in KS]


def full_scores(img: torch.Tensor, t2i: torch.Tensor, all_txt: torch.Tensor):
    """Dense models: (T2I [n_t2i, n_img], I2T [n_img, n_cap]) fp32 on the device (main.py:471-473)."""
    return ops.gemm(t2i.contiguous(), img.contiguous(), out_f32=True), \
        ops.gemm(img.contiguous(), all_txt.contiguous(), out_f32=True)


def sample_indices(n: int, iterations: int, seed: Optional[int] = 0, device="cuda") -> torch.Tensor:
    """int32 [iterations, n] resamples with replacement (np.random.choice(n, n, replace=True) per
    iteration, main.py:588; the reference is unseeded — here a seeded generator)."""
    rng = np.random.default_rng(seed)
    return torch.from_numpy(rng.integers(0, n, (iterations, n)).astype(np.int32)).to(device)


def ops_ws_bytes(rows: int, cols: int, k: int) -> int:
    """mme_topk_rows_torch's workspace for one resample's [rows, cols] matrix (rows·cols·8 B when
    torch's nth_element branch, k·64 > cols, runs; else 0)."""
    return 8 * rows * cols if k * 64 > cols else 0


@torch.no_grad()
def bootstrap_hits(s_t2i: torch.Tensor, s_i2t: torch.Tensor, samples: torch.Tensor, caps_per_image: int = 5,
                   ks: Sequence[int] = KS, batch: Optional[int] = None) -> torch.Tensor:
    """int64 [iterations, 9] hit counts (T2I, I2T, I2T-Sym) x ks for every resample."""
    iters, n = samples.shape
    if s_t2i.shape != (n, n) or s_i2t.shape != (n, caps_per_image * n):
        raise ValueError("bootstrap_hits: expected T2I [n, n] and I2T [n, caps*n] score matrices")
    s_sym = s_t2i.t().contiguous()
    if batch is None:  # ~2 GiB per batch: one gathered matrix at a time + its torch-order selection workspace
        per = max(4 * n * c + ops_ws_bytes(n, c, min(max(ks), c)) for c in (n, caps_per_image * n))
        batch = max(1, min(iters, (2 << 30) // max(1, per)))
    out = torch.empty(iters, 3 * len(ks), dtype=torch.int64, device=samples.device)
    for b0 in range(0, iters, batch):
        smp = samples[b0:b0 + batch].contiguous()
        for j, (S, g) in enumerate(((s_t2i, 1), (s_i2t, caps_per_image), (s_sym, 1))):
            G = ops.gather_scores(S, smp, smp, g)
            for q, k in enumerate(ks):  # one torch.topk per row and k (main.py:331-378)
                kk = min(k, G.shape[1])
                idx, _ = ops.topk_rows_torch(G, kk)
                out[b0:b0 + smp.shape[0], j * len(ks) + q:j * len(ks) + q + 1] = ops.recall_hits_groups(
                    idx, n, g, [kk])
            del G
    return out


def confidence_interval(values: np.ndarray, confidence: float = 0.95, n_boot: int = 10000, seed: int = 0):
    """bootstrap_confidence_interval (main.py:259-278): mean, 2.5 / 97.5 percentiles of resampled means."""
    rng = np.random.default_rng(seed)
    values = np.asarray(values, np.float64)
    means = values[rng.integers(0, len(values), (n_boot, len(values)))].mean(1)
    a = (1 - confidence) / 2
    return float(values.mean()), float(np.percentile(means, a * 100)), float(np.percentile(means, (1 - a) * 100))


def bootstrap_row(hits: torch.Tensor, n: int, ks: Sequence[int] = KS, seed: int = 0) -> Dict[str, float]:
    """Per-metric _mean / _lower / _upper / _std over the resamples (main.py:641-651 column order)."""
    h = hits.cpu().numpy().astype(np.float64) * (100.0 / n)
    names = [f"{p}_R@{k}" for p in ("T2I", "I2T", "I2T_Sym") for k in ks]
    row: Dict[str, float] = {}
    for j, name in enumerate(names):
        m, lo, hi = confidence_interval(h[:, j], seed=seed + j)
        row[f"{name}_mean"], row[f"{name}_lower"], row[f"{name}_upper"] = m, lo, hi
        row[f"{name}_std"] = float(np.std(h[:, j]))
    return row
