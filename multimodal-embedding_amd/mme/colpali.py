"""ColPali late-interaction scoring (MaxSim) on the device.

Reference: compute_similarity_scores' colpali branch (main.py:451-470) calls
colpali_engine's processor.score(q_chunk, d_chunk) on 10 x 10 chunks, which
zero-pads each chunk with pad_sequence and evaluates
einsum("bnd,csd->bcns").max(dim=3)[0].sum(dim=2) in bf16 (in-container port:
TF:models/colpali/processing_colpali.py:256-270; colpali_engine itself is not
installed — pinned >=0.2.0 in requirements.txt:9, 0.3.1 in paper.md:146).

Padding semantics reproduced exactly:
  * zero query rows contribute max(0·D) = 0 -> dropped (q_lens);
  * zero doc rows join the max as a 0 whenever the doc is shorter than the
    longest doc of its chunk -> per-doc `d_zero` flag.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch

from . import ops

DIM = 128


def pack_multivectors(vs: Sequence[torch.Tensor], multiple: int = 16, device="cuda"
                      ) -> Tuple[torch.Tensor, torch.Tensor]:
    """List of [T_i, 128] -> (zero-padded bf16 [n, Lpad, 128], int32 lens [n]) on the device."""
    dev = torch.device(device)
    vs = [v.reshape(-1, v.shape[-1]) for v in vs]
    lens = [v.shape[0] for v in vs]
    L = max(lens) if lens else 1
    Lp = max(multiple, (L + multiple - 1) // multiple * multiple)
    out = torch.zeros(len(vs), Lp, DIM, dtype=torch.bfloat16, device=dev)
    for i, v in enumerate(vs):
        out[i, : v.shape[0]] = v.to(dev, torch.bfloat16)
    return out, torch.tensor(lens, dtype=torch.int32, device=dev)


def chunk_zero_flags(d_lens: torch.Tensor, chunk: int) -> torch.Tensor:
    """u8 flag per doc: shorter than the longest doc of its `chunk`-sized group."""
    n = d_lens.numel()
    pad = (-n) % chunk
    l = torch.nn.functional.pad(d_lens.to(torch.int64), (0, pad), value=-1).view(-1, chunk)
    mx = l.max(dim=1, keepdim=True).values.expand_as(l).reshape(-1)[:n]
    return (d_lens.to(torch.int64) < mx).to(torch.uint8)


def maxsim_scores(Q: torch.Tensor, q_lens: torch.Tensor, D: torch.Tensor, d_lens: torch.Tensor,
                  doc_chunk: Optional[int] = 10) -> torch.Tensor:
    """fp32 [nq, nd] MaxSim with the reference's chunked zero-padding (doc_chunk=None: whole list is one chunk)."""
    flags = chunk_zero_flags(d_lens, doc_chunk or d_lens.numel())
    return ops.maxsim(Q, q_lens, D, d_lens, flags)


KS = (1, 5, 10)


def colpali_recall(img_D: torch.Tensor, img_len: torch.Tensor, t2i_Q: torch.Tensor, t2i_len: torch.Tensor,
                   all_D: torch.Tensor, all_len: torch.Tensor, all_pad: torch.Tensor,
                   caps_per_image: int = 5, ks: Sequence[int] = KS, chunk: int = 10):
    """Single-process Recall@k of the colpali branch (mme.distributed.sharded_colpali_recall
    at world size 1). Returns (hit counters dict, score matrices dict)."""
    from .distributed import sharded_colpali_recall
    return sharded_colpali_recall(img_D, img_len, t2i_Q, t2i_len, all_D, all_len, all_pad, 0, 1, img_D.shape[0],
                                  caps_per_image, ks, chunk, return_scores=True)


class ColPaliScorer:
    """The processor.score surface used at main.py:467 (plus a one-call fast path)."""

    def __init__(self, device="cuda"):
        self.device = torch.device(device)

    def score(self, qs: Sequence[torch.Tensor], ps: Sequence[torch.Tensor], **_) -> torch.Tensor:
        """One reference call: qs / ps are one chunk each (padded as a whole). Returns CPU fp32."""
        Q, ql = pack_multivectors(qs, device=self.device)
        D, dl = pack_multivectors(ps, device=self.device)
        return maxsim_scores(Q, ql, D, dl, doc_chunk=None).cpu()

    def score_chunked(self, qs: Sequence[torch.Tensor], ps: Sequence[torch.Tensor], chunk: int = 10
                      ) -> torch.Tensor:
        """Equivalent of the reference's whole 10 x 10 chunk loop (main.py:462-469) in one launch."""
        Q, ql = pack_multivectors(qs, device=self.device)
        D, dl = pack_multivectors(ps, device=self.device)
        return maxsim_scores(Q, ql, D, dl, doc_chunk=chunk)
