"""Similarity + top-k recall restated in numpy (oracle; test infrastructure only).

compute_similarity_scores dense branch (main.py:471-473): fp32 matmul of the
bf16 embeddings; compute_metrics_detailed recall loops (main.py:331-378): for
each k in (1, 5, 10) and each row, torch.topk(row, min(k, ncols)); hit if a
target column is among them, R@k = 100 * hits / rows. I2T uses the v28
orientation (run_benchmark_grand_slam_v28_publication_ready.py:391).

Ranking follows torch.topk's CPU order exactly, exact ties included (the order
torch's libstdc++ partial_sort / nth_element leaves tied values in; neither
column order nor its reverse): a row whose top-(k+1) values are all distinct has
ONE top-k in one order, found by argpartition + (score desc, column asc) sort;
a row with an exact tie among them is re-selected by torch's own algorithm
(oracle/torch_topk.cpp), once per k as compute_metrics_detailed calls it.
Pinned by tests/golden/retrieval.npz, full_retrieval.npz and dense_ties.npz
(exact duplicates: repeated images / captions, both of torch's branches).
"""
from __future__ import annotations

from typing import Dict, Sequence

import numpy as np

KS = (1, 5, 10)


def bf16_to_f32(bits: np.ndarray) -> np.ndarray:
    return (bits.astype(np.uint32) << 16).view(np.float32)


def scores(q: np.ndarray, d: np.ndarray) -> np.ndarray:
    return q.astype(np.float32) @ d.astype(np.float32).T


def _lex_topk(s: np.ndarray, k: int):
    """(idx, score) of the k largest per row, ordered (score desc, column asc).

    Wide rows: argpartition to k + 16 candidates, exact ordering among them; a row whose
    last candidate ties the k-th value (a tie could straddle the cut) is ordered in full."""
    k = min(k, s.shape[1])
    kk = k + 16

    def full(x):
        cols = np.arange(x.shape[1])
        order = np.lexsort((np.broadcast_to(cols, x.shape), -x), axis=1)[:, :k]
        return order.astype(np.int32), np.take_along_axis(x, order, 1)
    if s.shape[1] <= 4 * kk:
        return full(s)
    cand = np.argpartition(-s, kk - 1, axis=1)[:, :kk]
    cs = np.take_along_axis(s, cand, 1)
    order = np.lexsort((cand, -cs), axis=1)
    cand, cs = np.take_along_axis(cand, order, 1), np.take_along_axis(cs, order, 1)
    idx, sc = cand[:, :k].astype(np.int32), cs[:, :k].copy()
    redo = np.nonzero(cs[:, kk - 1] >= cs[:, k - 1])[0]
    if redo.size:
        idx[redo], sc[redo] = full(s[redo])
    return idx, sc


def _tied(sc: np.ndarray) -> np.ndarray:
    """Rows of a sorted top-list holding an exact tie between neighbours."""
    return (sc[:, 1:] == sc[:, :-1]).any(1) if sc.shape[1] > 1 else np.zeros(sc.shape[0], bool)


def topk(s: np.ndarray, k: int):
    """(idx int32, score fp32) [rows, min(k, ncols)] = torch.topk(row, k) for every row, in torch's
    CPU order (main.py:335,365,375)."""
    s = np.ascontiguousarray(s, np.float32)
    k = min(k, s.shape[1])
    idx, sc = _lex_topk(s, min(k + 1, s.shape[1]))
    tie = np.nonzero(_tied(sc))[0]
    idx, sc = idx[:, :k].copy(), sc[:, :k].copy()
    if tie.size:
        from . import torch_topk
        ti, tv = torch_topk.topk(s[tie], k)
        idx[tie], sc[tie] = ti.astype(np.int32), tv
    return idx, sc


def hits(s: np.ndarray, tgt_count: int, ks: Sequence[int] = KS, row_offset: int = 0) -> np.ndarray:
    """[rows, len(ks)] bool: row r's target columns [(r + row_offset)·tgt_count, +tgt_count) lie in
    torch.topk(row, min(k, ncols)) -- compute_metrics_detailed's per-k selection (main.py:331-378).
    Rows whose top-(kmax+1) values are distinct take every k from one ordered list; rows with an exact
    tie there are selected per k in torch's order."""
    s = np.ascontiguousarray(s, np.float32)
    n = s.shape[1]
    kmax = min(max(ks), n)
    idx, sc = _lex_topk(s, min(kmax + 1, n))
    rows = np.arange(s.shape[0]) + row_offset
    tgt = (idx[:, :kmax] // tgt_count) == rows[:, None]
    first = np.where(tgt.any(1), tgt.argmax(1), kmax)
    out = np.stack([first < min(k, n) for k in ks], 1)
    tie = np.nonzero(_tied(sc))[0]
    if tie.size:
        from . import torch_topk
        st = s[tie]
        out[tie] = np.stack([((torch_topk.topk(st, min(k, n))[0] // tgt_count) == rows[tie, None]).any(1)
                             for k in ks], 1)
    return out


def compare_topk(idx: np.ndarray, ref_idx: np.ndarray, ref_score: np.ndarray, rel_tol: float = 1e-5,
                 exact_rows: np.ndarray = None, dev_score: np.ndarray = None, oracle_only: list = None,
                 unflagged: list = None):
    """Row-wise parity of a top-k index table against the reference's.

    ref_idx / ref_score hold the reference's top-(k+1) per row (score desc). A row is a
    near-tie when two neighbouring scores among those k+1 differ by <= rel_tol·|s_1| but are
    not equal: a different fp32 summation order may legitimately swap them (SURVEY §7,
    "exact-index parity"). EXACT ties are not exempt on rows the compared side found tied too
    (exact_rows, bool per row: mme.retrieval.Ranked.tie_rows): their order is torch.topk's, which
    the device replays. A reference exact tie on a row the compared side did NOT flag is a near tie
    (its summation order separated the pair); oracle_only (a list, optional) receives those rows.
    dev_score (optional), the compared side's own top-(k+1) scores, checks the flags themselves:
    a row whose own scores hold an exact tie must be flagged; unflagged (a list, optional)
    receives the rows that are not (a tie_rows defect; callers assert it stays empty). Returns
    (identical [rows] bool, near_tie [rows] bool); every row that is not a near-tie must be
    identical. With no (k+1)-th reference column (fewer columns than k + 1) only the gaps that
    exist are compared."""
    k = idx.shape[1]
    same = (idx == ref_idx[:, :k]).all(1)
    kk = min(k + 1, ref_score.shape[1])
    gaps = ref_score[:, :kk - 1] - ref_score[:, 1:kk]
    unequal = gaps != 0
    if exact_rows is not None:
        flagged = np.asarray(exact_rows, bool)
        only = ~flagged[:, None] & (gaps == 0)
        if oracle_only is not None:
            oracle_only.extend(np.nonzero(only.any(1))[0].tolist())
        if dev_score is not None and unflagged is not None:
            kd = min(kk, dev_score.shape[1])
            dtied = (dev_score[:, :kd - 1] == dev_score[:, 1:kd]).any(1)
            unflagged.extend(np.nonzero(dtied & ~flagged)[0].tolist())
        unequal = unequal | only
    near = ((gaps <= rel_tol * np.abs(ref_score[:, :1])) & unequal).any(1)
    return same, near


def recall(idx: np.ndarray, tgt_count: int, ks: Sequence[int] = KS, row_offset: int = 0) -> np.ndarray:
    """Hit counts per k from ONE ordered top-k table (exact only for rows without a tie at a k-th
    place; `hits` is the per-k selection)."""
    rows = np.arange(idx.shape[0]) + row_offset
    lo = rows * tgt_count
    hit = (idx >= lo[:, None]) & (idx < lo[:, None] + tgt_count)
    first = np.where(hit.any(1), hit.argmax(1), idx.shape[1])
    return np.array([(first < min(k, idx.shape[1])).sum() for k in ks], np.int64)


def metrics(img: np.ndarray, t2i: np.ndarray, all_txt: np.ndarray, caps: int = 5, ks=KS) -> Dict[str, float]:
    """The 9 R@k values of compute_metrics_detailed on the identity sample."""
    n = img.shape[0]
    out = {}
    for name, q, d, tc, denom in (("T2I", t2i, img, 1, t2i.shape[0]), ("I2T", img, all_txt, caps, n),
                                  ("I2T_Sym", img, t2i, 1, n)):
        h = hits(scores(q, d), tc, ks).sum(0)
        for j, k in enumerate(ks):
            out[f"{name}_R@{k}"] = 100.0 * h[j] / denom
    return out


def l2norm_bf16(x_bits: np.ndarray) -> np.ndarray:
    """bf16 bits -> bf16 bits of x / bf16(||x||) (main.py:414 semantics on a bf16 tensor)."""
    import torch
    x = torch.from_numpy(x_bits.view(np.int16)).view(torch.bfloat16)
    n = torch.sqrt((x.float() ** 2).sum(-1, keepdim=True)).to(torch.bfloat16)
    y = (x.float() / n.float()).to(torch.bfloat16)
    return y.view(torch.int16).numpy().view(np.uint16)
