"""Winoground 2x2 decision rule (oracle; test infrastructure only).

run_winoground, run_benchmark_grand_slam_v28_publication_ready.py:443-452:
s = torch.matmul(te.to(DTYPE), ie.to(DTYPE).t()) on L2-normalised bf16 embeddings,
then strict comparisons. Pinned by tests/golden/winoground.npz (the reference's own
run_winoground over tiny models, load_dataset patched to synthetic examples).
"""
from __future__ import annotations

import numpy as np
import torch


def scores(te: torch.Tensor, ie: torch.Tensor) -> torch.Tensor:
    """te, ie: [2, D] bf16 -> [2, 2] fp32 of the bf16 matmul (fp32 accumulation, one rounding)."""
    return (te.float() @ ie.float().t()).to(torch.bfloat16).float()


def decide(s) -> tuple:
    s = np.asarray(s, dtype=np.float32).reshape(2, 2)
    txt = bool(s[0, 0] > s[0, 1] and s[1, 1] > s[1, 0])
    img = bool(s[0, 0] > s[1, 0] and s[1, 1] > s[0, 1])
    return txt, img, txt and img


def metrics(all_scores) -> dict:
    d = np.array([decide(s) for s in all_scores], dtype=np.int64).reshape(-1, 3)
    n = max(1, d.shape[0])
    return {"Wino Text": 100.0 * d[:, 0].sum() / n, "Wino Image": 100.0 * d[:, 1].sum() / n,
            "Wino Group": 100.0 * d[:, 2].sum() / n}
