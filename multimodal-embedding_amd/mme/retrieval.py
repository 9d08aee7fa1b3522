"""Similarity + top-k recall on the device.

Mirrors compute_similarity_scores (main.py:440-475) and the recall part of
compute_metrics_detailed (main.py:305-383) with the I2T orientation of v28
(run_benchmark_grand_slam_v28_publication_ready.py:391): scores_i2t =
img @ all_txt.T (main.py:622-623's trailing .t() is the KeyError bug of
SURVEY.md §0.1 and is not reproduced). Recall is computed on the identity
sample (every item once), the only sample for which the reference's result is
defined reproducibly.

The fused kernel never materialises the score matrix: mme_sim_topk returns
the 10 best columns per row (score desc, column asc) and mme_recall_hits
counts rows whose first k columns contain a target.
"""
from __future__ import annotations

from typing import Dict, Sequence

import torch

from . import ops

KS = (1, 5, 10)


def compute_similarity_scores(img_embeds: torch.Tensor, txt_embeds: torch.Tensor, m_info=None,
                              processor=None) -> torch.Tensor:
    """scores [n_txt, n_img] fp32 = txt @ img.T (main.py:471-473), on the device.

    ColPali (m_info['type'] == 'colpali') routes to processor.score (MaxSim)."""
    if m_info is not None and m_info.get("type") == "colpali":
        return processor.score(txt_embeds, img_embeds)
    dev = img_embeds.device if img_embeds.is_cuda else torch.device("cuda")
    a = txt_embeds.to(dev, torch.bfloat16).contiguous()
    b = img_embeds.to(dev, torch.bfloat16).contiguous()
    if a.shape[1] % 64:  # the GEMM's K steps are 64 deep; zero columns leave the dot products unchanged
        pad = -a.shape[1] % 64
        a, b = torch.nn.functional.pad(a, (0, pad)), torch.nn.functional.pad(b, (0, pad))
    return ops.gemm(a, b, out_f32=True)


def topk_rows(q: torch.Tensor, d: torch.Tensor, k: int, col_offset: int = 0):
    """(idx, score) of the k best columns of q @ d.T per row."""
    return ops.sim_topk(q.contiguous(), d.contiguous(), k, col_offset)


def recall_counts(img: torch.Tensor, t2i_txt: torch.Tensor, all_txt: torch.Tensor, caps_per_image: int = 5,
                  ks: Sequence[int] = KS, img_row_offset: int = 0, t2i_row_offset: int = 0,
                  img_all: torch.Tensor = None) -> Dict[str, torch.Tensor]:
    """Device hit counters for the three protocols of compute_metrics_detailed.

    img / t2i_txt rows are this process's (sharded) rows starting at the given
    global offsets; all_txt and img_all are the full (all-gathered) tables."""
    img_all = img if img_all is None else img_all
    n_img_all, n_t2i_all, n_cap_all = img_all.shape[0], None, all_txt.shape[0]
    kmax = max(ks)
    out = {}
    # T2I (main.py:331-358): query caption i -> target image i
    k = min(kmax, img_all.shape[0])
    idx, _ = topk_rows(t2i_txt, img_all, k)
    out["T2I"] = ops.recall_hits(idx, 1, [min(x, k) for x in ks], row_offset=t2i_row_offset)
    # I2T multi-caption (main.py:361-368): image i -> captions [5i, 5i+5)
    k = min(kmax, n_cap_all)
    idx, _ = topk_rows(img, all_txt, k)
    out["I2T"] = ops.recall_hits(idx, caps_per_image, [min(x, k) for x in ks], row_offset=img_row_offset)
    return out


def recall_sym_counts(img: torch.Tensor, t2i_all: torch.Tensor, ks: Sequence[int] = KS, img_row_offset: int = 0):
    """I2T symmetric (main.py:371-378): scores_t2i.t() -> image i vs single caption i."""
    k = min(max(ks), t2i_all.shape[0])
    idx, _ = topk_rows(img, t2i_all, k)
    return ops.recall_hits(idx, 1, [min(x, k) for x in ks], row_offset=img_row_offset)


def counts_to_metrics(counts: Dict[str, torch.Tensor], n_img: int, n_t2i: int, ks: Sequence[int] = KS
                      ) -> Dict[str, float]:
    """Hit counters -> the reference's metric dict (key order of main.py:358,368,378)."""
    res = {}
    for name, denom in (("T2I", n_t2i), ("I2T", n_img), ("I2T_Sym", n_img)):
        c = counts[name].tolist()
        for j, k in enumerate(ks):
            res[f"{name}_R@{k}"] = 100.0 * c[j] / denom
    return res


def compute_metrics(img: torch.Tensor, t2i_txt: torch.Tensor, all_txt: torch.Tensor, caps_per_image: int = 5,
                    ks: Sequence[int] = KS) -> Dict[str, float]:
    """Single-process R@k for T2I, I2T (multi-caption) and I2T-Sym on the identity sample."""
    dev = torch.device("cuda")
    img, t2i_txt, all_txt = (t.to(dev, torch.bfloat16).contiguous() for t in (img, t2i_txt, all_txt))
    counts = recall_counts(img, t2i_txt, all_txt, caps_per_image, ks)
    counts["I2T_Sym"] = recall_sym_counts(img, t2i_txt, ks)
    return counts_to_metrics(counts, img.shape[0], t2i_txt.shape[0], ks)
