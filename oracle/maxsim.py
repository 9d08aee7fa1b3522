"""ColPali MaxSim restated (oracle).

colpali_engine processor.score -> score_multi_vector (in-container port
TF:models/colpali/processing_colpali.py:256-270): per chunk, pad_sequence
(zeros) queries and docs, einsum("bnd,csd->bcns") in bf16, max over doc
tokens, sum over query tokens (bf16), cast to fp32. Chunking of the reference
loop (main.py:451-470): 10 queries x 10 docs per call. Pinned by
tests/golden/maxsim.npz.
"""
from __future__ import annotations

from typing import List

import numpy as np
import torch


def score_chunk(qs: List[torch.Tensor], ds: List[torch.Tensor]) -> torch.Tensor:
    Q = torch.nn.utils.rnn.pad_sequence(qs, batch_first=True, padding_value=0)
    D = torch.nn.utils.rnn.pad_sequence(ds, batch_first=True, padding_value=0)
    return torch.einsum("bnd,csd->bcns", Q, D).max(dim=3)[0].sum(dim=2).to(torch.float32)


def score_reference_chunks(qs: List[torch.Tensor], ds: List[torch.Tensor], chunk: int = 10) -> torch.Tensor:
    rows = []
    for i in range(0, len(qs), chunk):
        rows.append(torch.cat([score_chunk(qs[i:i + chunk], ds[j:j + chunk]) for j in range(0, len(ds), chunk)], 1))
    return torch.cat(rows, 0)


def split(bits: np.ndarray, lens: np.ndarray) -> List[torch.Tensor]:
    x = torch.from_numpy(bits.view(np.int16)).view(torch.bfloat16)
    out, o = [], 0
    for l in lens:
        out.append(x[o:o + l])
        o += l
    return out
