"""Multi-GPU sharding of the encode + retrieval job (one process per GPU).

The reference is single-process (main.py:92); this is build-only scope
(SURVEY.md §8e). Partitioning: rank r owns images [lo, hi), their caption-0
T2I queries and captions [5·lo, 5·hi) — caption ownership follows image
ownership, so encoding needs no communication at all. Exchange, once per job:
  * all-gather of the text embeddings (T2I and all captions) and of the image
    embeddings (bf16, 69 MB + 11.5 MB at SigLIP D = 1152) over RCCL/xGMI;
  * every rank then ranks ITS rows against the full tables (T2I: its caption-0
    rows vs all images; I2T / I2T-Sym: its images vs all captions) — no
    cross-rank top-k merge is needed;
  * one all-reduce(SUM) of the 9 int64 hit counters.
The compute callbacks are injectable so the orchestration is testable on the
CPU with gloo (tests/test_distributed.py).
"""
from __future__ import annotations

from typing import Callable, Dict, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

KS = (1, 5, 10)


def shard_range(n: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous balanced split of n items (first n % world ranks get one more)."""
    q, r = divmod(n, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def all_gather_rows(x: torch.Tensor, world: int, group=None) -> torch.Tensor:
    """Concatenate every rank's [n_r, D] rows in rank order (ragged n_r allowed)."""
    if world == 1:
        return x
    return _gather_ragged(x, world, group)


def _gather_ragged(x: torch.Tensor, world: int, group=None) -> torch.Tensor:
    """all_gather_rows' collective: exchange the row counts, gather rows padded to the largest,
    strip the padding (device tensors: one all_gather_into_tensor over RCCL)."""
    if x.is_cuda and dist.get_backend(group) == "gloo":  # gloo gathers host tensors (CPU rehearsal of N > 1)
        return _gather_ragged(x.cpu(), world, group).to(x.device)
    n = torch.tensor([x.shape[0]], dtype=torch.int64, device=x.device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    sizes = [int(s.item()) for s in sizes]
    mx = max(sizes)
    xp = x if x.shape[0] == mx else torch.cat([x, x.new_zeros(mx - x.shape[0], *x.shape[1:])])
    xp = xp.contiguous()
    if x.is_cuda:
        out = x.new_empty(world * mx, *x.shape[1:])
        dist.all_gather_into_tensor(out, xp, group=group)
        parts = out.split(mx)
    else:
        parts = [torch.empty_like(xp) for _ in range(world)]
        dist.all_gather(parts, xp, group=group)
    return torch.cat([p[:s] for p, s in zip(parts, sizes)])


def all_reduce_(t: torch.Tensor, op=dist.ReduceOp.SUM, group=None) -> torch.Tensor:
    """In-place all-reduce; gloo (CPU rehearsal of the N > 1 path) reduces a host copy of device tensors."""
    if t.is_cuda and dist.get_backend(group) == "gloo":
        h = t.cpu()
        dist.all_reduce(h, op=op, group=group)
        t.copy_(h)
        return t
    dist.all_reduce(t, op=op, group=group)
    return t


class DeviceOps:
    """Default compute: libmme fused sim/top-k + recall counters, in torch.topk's order on exact ties
    (mme.retrieval.rank_rows)."""

    def rank(self, q: torch.Tensor, d: torch.Tensor, tgt_count: int, ks: Sequence[int], row_offset: int):
        """(hit counts int64 [len(ks)], top-max(ks) index table in torch.topk's order)."""
        from .retrieval import rank_rows
        r = rank_rows(q, d, tgt_count, ks, row_offset)
        return r.hits, r.idx


def rank_hit_counts(img_l: torch.Tensor, t2i_l: torch.Tensor, img_all: torch.Tensor, t2i_all: torch.Tensor,
                    all_all: torch.Tensor, row_offset: int, caps_per_image: int = 5, ks: Sequence[int] = KS,
                    compute: Optional[object] = None, return_idx: bool = False):
    """One rank's share of the 9 hit counters: ITS rows ranked against the full tables.

    T2I: the rank's caption-0 queries vs all images; I2T: its images vs all captions;
    I2T-Sym: its images vs all T2I captions. ``row_offset`` = the rank's first global
    image (targets are global indices). ``compute.rank(q, d, tgt_count, ks, row_offset)``
    returns (hit counts, top-k table) with compute_metrics_detailed's per-k torch.topk
    semantics. Returns int64 [3·len(ks)] (and the top-k index tables when ``return_idx``)."""
    compute = compute or DeviceOps()
    res, idxs = [], {}
    for name, q, d, tcount in (("T2I", t2i_l, img_all, 1), ("I2T", img_l, all_all, caps_per_image),
                               ("I2T_Sym", img_l, t2i_all, 1)):
        if q.shape[0]:
            h, idx = compute.rank(q, d, tcount, ks, row_offset)
            idxs[name] = idx
        else:
            h = torch.zeros(len(ks), dtype=torch.int64, device=q.device)
        res.append(h.to(torch.int64))
    counts = torch.cat(res)
    return (counts, idxs) if return_idx else counts


def counts_to_metrics(counts: Sequence[int], n_img: int, ks: Sequence[int] = KS) -> Dict[str, float]:
    """R@k = 100 · hits / n for the 9 counters in (T2I, I2T, I2T_Sym) × ks order (main.py:358,368,378)."""
    c = [int(x) for x in counts]
    out = {}
    for j, name in enumerate(("T2I", "I2T", "I2T_Sym")):
        for i, k in enumerate(ks):
            out[f"{name}_R@{k}"] = 100.0 * c[j * len(ks) + i] / n_img
    return out


def sharded_recall(img_l: torch.Tensor, t2i_l: torch.Tensor, all_l: torch.Tensor, rank: int, world: int,
                   n_img: int, caps_per_image: int = 5, ks: Sequence[int] = KS, group=None,
                   compute: Optional[object] = None, return_tables: bool = False):
    """Global R@k from per-rank shards (see module docstring). With return_tables the tables dict
    also carries "gather_events": device events around the three all-gathers (None on the CPU)."""
    lo, _ = shard_range(n_img, rank, world)
    evs = None
    if img_l.is_cuda:
        evs = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        evs[0].record()
    img_all = all_gather_rows(img_l, world, group)
    t2i_all = all_gather_rows(t2i_l, world, group)
    all_all = all_gather_rows(all_l, world, group)
    if evs is not None:
        evs[1].record()
    counts = rank_hit_counts(img_l, t2i_l, img_all, t2i_all, all_all, lo, caps_per_image, ks, compute)
    if world > 1:
        all_reduce_(counts, dist.ReduceOp.SUM, group)
    out = counts_to_metrics(counts.tolist(), n_img, ks)
    if return_tables:
        return out, {"img": img_all, "t2i": t2i_all, "all": all_all, "gather_events": evs}
    return out


def env_rank_world() -> Tuple[int, int, int]:
    """(rank, world_size, local_rank) from torchrun's environment (defaults 0/1/0)."""
    from .launch import env_rank_world as _erw
    return _erw()


class MaxSimOps:
    """Default compute of the ColPali recall: libmme MaxSim, row top-k and recall counters.

    Recall ranks every row in torch.topk's CPU order (mme_topk_rows_torch), one selection per k
    as compute_metrics_detailed calls it (main.py:331-378): MaxSim sums are bf16-quantised, so
    exact ties at the k-th place are common and the reference's tie order decides them."""

    def maxsim(self, Q, ql, D, dl, flags):
        from . import ops
        return ops.maxsim(Q, ql, D, dl, flags)

    def recall(self, s: torch.Tensor, tgt_count: int, ks: Sequence[int], row_offset: int) -> torch.Tensor:
        from . import ops
        return ops.recall_hits_torch(s.contiguous(), tgt_count, ks, row_offset)

    def topk(self, s: torch.Tensor, k: int) -> torch.Tensor:
        from . import ops
        return ops.topk_rows(s, k)[0]

    def hits(self, idx: torch.Tensor, tgt_count: int, ks: Sequence[int], row_offset: int) -> torch.Tensor:
        from . import ops
        return ops.recall_hits(idx, tgt_count, ks, row_offset=row_offset)


def sharded_colpali_recall(img_D: torch.Tensor, img_len: torch.Tensor, t2i_Q: torch.Tensor, t2i_len: torch.Tensor,
                           all_D: torch.Tensor, all_len: torch.Tensor, all_pad: torch.Tensor, rank: int, world: int,
                           n_img: int, caps_per_image: int = 5, ks: Sequence[int] = KS, chunk: int = 10, group=None,
                           compute: Optional[object] = None, return_scores: bool = False):
    """Recall@k of the colpali branch of run_bootstrap_benchmark (main.py:618-624 with the
    v28 I2T orientation) from per-rank shards of per-item multi-vector tables.

    Rank r holds images [lo, hi) (img_D [n_r, Ld, 128], valid rows img_len), their T2I
    caption queries (t2i_Q / t2i_len, valid rows first) and their captions (all_D / all_len,
    all_pad = each caption's padded length L_b in the reference's left-padded batch).
    Exchange: one all-gather of each table (bf16; 266 MB of image vectors at n = 1000),
    then every rank scores ITS rows (MaxSim is asymmetric, so I2T-Sym = columns of T2I:
    all T2I queries against the rank's images, transposed) and one all-reduce of the
    9 hit counters. Zero-padding semantics of processor.score's pad_sequence are global:
    doc chunks of `chunk` run over the full, rank-ordered doc lists."""
    from .colpali import chunk_zero_flags
    compute = compute or MaxSimOps()
    lo, hi = shard_range(n_img, rank, world)
    D_all, dl_all = all_gather_rows(img_D, world, group), all_gather_rows(img_len, world, group)
    Qt_all, qtl_all = all_gather_rows(t2i_Q, world, group), all_gather_rows(t2i_len, world, group)
    Qa_all, qal_all = all_gather_rows(all_D, world, group), all_gather_rows(all_len, world, group)
    qap_all = all_gather_rows(all_pad, world, group)
    img_flags = chunk_zero_flags(dl_all, chunk)
    cap_flags = chunk_zero_flags(qap_all, chunk) | (qap_all > qal_all).to(torch.uint8)
    kmax = max(ks)
    s_t2i = compute.maxsim(t2i_Q, t2i_len, D_all, dl_all, img_flags)        # [n_r, n]
    s_i2t = compute.maxsim(img_D, img_len, Qa_all, qal_all, cap_flags)     # [n_r, 5n]
    if world == 1:
        s_sym = s_t2i.t().contiguous()
    else:  # column block [lo, hi) of the global T2I matrix
        s_sym = compute.maxsim(Qt_all, qtl_all, img_D, img_len, img_flags[lo:hi].contiguous()).t().contiguous()
    res = []
    for s, tc in ((s_t2i, 1), (s_i2t, caps_per_image), (s_sym, 1)):
        k = min(kmax, s.shape[1])
        kk = [min(x, k) for x in ks]
        if s.shape[0] and hasattr(compute, "recall"):
            res.append(compute.recall(s, tc, kk, lo).to(torch.int64))
        elif s.shape[0]:
            res.append(compute.hits(compute.topk(s, k), tc, kk, lo).to(torch.int64))
        else:
            res.append(torch.zeros(len(ks), dtype=torch.int64, device=s.device))
    counts = torch.cat(res)
    if world > 1:
        all_reduce_(counts, dist.ReduceOp.SUM, group)
    c = counts.tolist()
    out = {}
    for j, name in enumerate(("T2I", "I2T", "I2T_Sym")):
        for i, k in enumerate(ks):
            out[f"{name}_R@{k}"] = 100.0 * c[j * len(ks) + i] / n_img
    if return_scores:
        return out, {"t2i": s_t2i, "i2t": s_i2t}
    return out
