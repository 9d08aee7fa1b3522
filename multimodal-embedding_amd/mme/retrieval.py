"""Similarity + top-k recall on the device.

Mirrors compute_similarity_scores (main.py:440-475) and the recall part of
compute_metrics_detailed (main.py:305-383) with the I2T orientation of v28
(run_benchmark_grand_slam_v28_publication_ready.py:391): scores_i2t =
img @ all_txt.T (main.py:622-623's trailing .t() is the KeyError bug of
SURVEY.md §0.1 and is not reproduced). Recall is computed on the identity
sample (every item once), the only sample for which the reference's result is
defined reproducibly.

The fused kernel never materialises the score matrix: mme_sim_topk returns
the 11 best columns per row (score desc, column asc) and mme_recall_hits
counts rows whose first k columns contain a target. The reference ranks with
torch.topk(row, k) once per k (main.py:335,365,375), whose order among EXACTLY
tied scores is its libstdc++ selection's, not column order: rows whose top 11
hold an exact tie (duplicated images or captions tie in every row) are flagged
(mme_tie_rows), their full score rows recomputed bit-identically
(mme_sim_scores) and re-selected in torch's order once per k
(mme_topk_rows_torch). Pinned by tests/golden/dense_ties.npz.
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
    """(idx, score) of the k best columns of q @ d.T per row, order (score desc, column asc)."""
    return ops.sim_topk(q.contiguous(), d.contiguous(), k, col_offset)


# bound on the fp32 score rows recomputed at once for tied rows (nd columns each)
TIE_ROWS_BYTES = 1 << 30


class Ranked:
    """rank_rows' result: hit counters per k, the top-kmax table in torch.topk's order, the rows
    that were re-selected in that order (with their per-k index lists), and the fused pass's
    top-(kmax+1) scores per row (descending)."""

    def __init__(self, hits, idx, tie_rows, tie_idx, score=None):
        self.hits, self.idx, self.tie_rows, self.tie_idx, self.score = hits, idx, tie_rows, tie_idx, score


def rank_rows(q: torch.Tensor, d: torch.Tensor, tgt_count: int, ks: Sequence[int] = KS, row_offset: int = 0,
              hits: torch.Tensor = None) -> Ranked:
    """compute_metrics_detailed's ranking of the rows of q @ d.T (main.py:331-378) on the device.

    Row r (global row r + row_offset) targets columns [(r + row_offset)·tgt_count, +tgt_count); for each
    k, a hit when torch.topk(row, min(k, nd)) holds a target. One fused sim/top-(kmax+1) pass ranks
    every row; rows without an exact tie in it have a unique top-k for every k (counted from that
    table). Rows with one (mme_tie_rows) are recomputed (mme_sim_scores: the same fp32 scores) and
    re-selected in torch.topk's CPU order, once per k (mme_topk_rows_torch). ``hits`` (int64
    [len(ks)]) accumulates when given."""
    q, d = q.contiguous(), d.contiguous()
    nq, nd = q.shape[0], d.shape[0]
    kmax = min(max(ks), nd)
    kk = [min(x, nd) for x in ks]
    if hits is None:
        hits = torch.zeros(len(ks), dtype=torch.int64, device=q.device)
    idx, sc = ops.sim_topk(q, d, min(kmax + 1, nd))
    flags = ops.tie_rows(sc)
    ops.recall_hits(idx, tgt_count, kk, row_offset=row_offset, hits=hits, skip=flags)
    idx = idx[:, :kmax]
    tie = flags.nonzero()[:, 0]  # the one host sync of the ranking: how many rows need torch's order
    tie_idx = {}
    if tie.numel():
        idx = idx.contiguous()
        per = max(1, TIE_ROWS_BYTES // (4 * nd))
        parts = {k: [] for k in kk}
        for lo in range(0, tie.numel(), per):
            rows = tie[lo:lo + per]
            S = ops.sim_scores(q.index_select(0, rows), d)
            tstart = ((rows + row_offset) * tgt_count).to(torch.int32)
            sel = {}
            for k in parts:  # one selection per distinct k (kk repeats k when nd < max(ks))
                sel[k] = ops.topk_rows_torch(S, k)[0]
                parts[k].append(sel[k])
            for j, k in enumerate(kk):  # but a hit counter per requested k
                ops.recall_hits(sel[k], tgt_count, [k], tgt_start=tstart, hits=hits[j:j + 1])
            idx.index_copy_(0, rows, parts[kmax][-1])  # torch.topk(row, kmax): the table's own order
        tie_idx = {k: torch.cat(v) for k, v in parts.items()}
    return Ranked(hits, idx, tie, tie_idx, sc)


def recall_counts(img: torch.Tensor, t2i_txt: torch.Tensor, all_txt: torch.Tensor, caps_per_image: int = 5,
                  ks: Sequence[int] = KS, img_row_offset: int = 0, t2i_row_offset: int = 0,
                  img_all: torch.Tensor = None) -> Dict[str, torch.Tensor]:
    """Device hit counters for the T2I and I2T protocols of compute_metrics_detailed.

    img / t2i_txt rows are this process's (sharded) rows starting at the given
    global offsets; all_txt and img_all are the full (all-gathered) tables."""
    img_all = img if img_all is None else img_all
    return {
        # T2I (main.py:331-358): query caption i -> target image i
        "T2I": rank_rows(t2i_txt, img_all, 1, ks, t2i_row_offset).hits,
        # I2T multi-caption (main.py:361-368): image i -> captions [5i, 5i+5)
        "I2T": rank_rows(img, all_txt, caps_per_image, ks, img_row_offset).hits}


def recall_sym_counts(img: torch.Tensor, t2i_all: torch.Tensor, ks: Sequence[int] = KS, img_row_offset: int = 0):
    """I2T symmetric (main.py:371-378): scores_t2i.t() -> image i vs single caption i."""
    return rank_rows(img, t2i_all, 1, ks, img_row_offset).hits


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
