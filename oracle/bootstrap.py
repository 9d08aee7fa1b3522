"""Bootstrap resampling of the recall metrics (oracle; test infrastructure only).

Restates the loop of run_bootstrap_benchmark (main.py:586-634) on precomputed
full score matrices: resample b's T2I matrix is s_t2i[s][:, s], its I2T matrix
s_i2t[s][:, caption positions of s] (img_to_caps_map, main.py:601-609), I2T-Sym
the transposed T2I matrix (main.py:624); compute_metrics_detailed (main.py:305-383)
counts a hit when a target column is among torch.topk(row, k).

Ties: a duplicated image (sampling with replacement) scores exactly like its copy,
so which copy torch.topk keeps decides many rows. `resample_hits` ranks every row
in torch.topk's own CPU order (oracle/torch_topk.cpp: the libstdc++ partial_sort /
nth_element torch runs), one selection per k as compute_metrics_detailed calls it;
`ambiguous` still counts the rows whose target tie group straddles the k-th place
(where a column-order rule would be a guess). Pinned against
tests/golden/bootstrap.npz (the reference's compute_metrics_detailed on resampled
matrices built by its own compute_similarity_scores): every value identical.
"""
from __future__ import annotations

from typing import Sequence, Tuple

import numpy as np

KS = (1, 5, 10)


def _rank_info(S: np.ndarray, tgt_lo: np.ndarray, tc: int) -> Tuple[np.ndarray, np.ndarray]:
    """Per row: (rank of the best target under the position rule, number of columns tied with it)."""
    rows = np.arange(S.shape[0])
    cols = tgt_lo[:, None] + np.arange(tc)[None, :]
    tv = S[rows[:, None], cols]                        # [R, tc]
    best = tv.argmax(1)                                # first max -> lowest position among equal targets
    v = tv[rows, best]
    p = cols[rows, best]
    greater = (S > v[:, None]).sum(1)
    pos = np.arange(S.shape[1])[None, :]
    equal_before = ((S == v[:, None]) & (pos < p[:, None])).sum(1)
    ties = (S == v[:, None]).sum(1) - 1
    return greater + equal_before, np.stack([greater, ties], 1)


def resample_hits(s_t2i: np.ndarray, s_i2t: np.ndarray, sample: np.ndarray, caps: int = 5,
                  ks: Sequence[int] = KS) -> Tuple[np.ndarray, np.ndarray]:
    """(hits [9], ambiguous [9]) of one resample (T2I, I2T, I2T-Sym) x ks."""
    n = sample.shape[0]
    t2i = s_t2i[np.ix_(sample, sample)]
    capcols = (caps * sample[:, None] + np.arange(caps)[None, :]).reshape(-1)
    i2t = s_i2t[np.ix_(sample, capcols)]
    sym = t2i.T
    from oracle import torch_topk as TT
    hits, amb = [], []
    for S, tc in ((t2i, 1), (i2t, caps), (sym, 1)):
        _, gt = _rank_info(S, np.arange(n) * tc, tc)
        greater, ties = gt[:, 0], gt[:, 1]
        hits.extend(TT.hits(np.ascontiguousarray(S), tc, ks).sum(0).tolist())
        for k in ks:
            k = min(k, S.shape[1])
            # where a column-order rule would guess: the target's tie group spans the k-th place
            amb.append(int(((greater < k) & (greater + ties >= k) & (ties > 0)).sum()))
    return np.array(hits, np.int64), np.array(amb, np.int64)
