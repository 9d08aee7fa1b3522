"""encode_data with the reference's semantics on the libmme path.

Restates main.py:386-438: batches of m_info['batch_size'], processor ->
get_image_features / get_text_features, CLS row if 3-D, L2-normalise in the
model dtype, cast to DTYPE (bf16) and move to the host (the reference's
output contract: CPU bf16 tensors). The normalisation runs in libmme
(mme_l2norm, bit-exact bf16 semantics) instead of torch.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import torch

from . import ops


@torch.no_grad()
def encode_data(model, processor, m_info: dict, images: Sequence, texts: Sequence, device="cuda"
                ) -> Tuple[torch.Tensor, torch.Tensor]:
    bs = m_info["batch_size"]
    if m_info.get("type") == "colpali":
        return encode_colpali(model, processor, bs, images, texts, device)
    img_list: List[torch.Tensor] = []
    for i in range(0, len(images), bs):
        inputs = processor(images=images[i:i + bs], return_tensors="pt", padding=True).to(device)
        out = model.get_image_features(**inputs)
        if out.dim() == 3:
            out = out[:, 0, :]
        img_list.append(ops.l2norm(out.contiguous()).cpu())
    txt_list: List[torch.Tensor] = []
    for i in range(0, len(texts), bs):
        inputs = processor(text=texts[i:i + bs], return_tensors="pt", padding=True, truncation=True).to(device)
        out = model.get_text_features(**inputs)
        if out.dim() == 3:
            out = out[:, 0, :]
        txt_list.append(ops.l2norm(out.contiguous()).cpu())
    img = torch.cat(img_list) if img_list else torch.empty(0)
    txt = torch.cat(txt_list) if txt_list else torch.empty(0)
    return img, txt


@torch.no_grad()
def encode_colpali(model, processor, bs: int, images: Sequence, texts: Sequence, device="cuda"
                   ) -> Tuple[List[torch.Tensor], List[torch.Tensor]]:
    """The colpali branch (main.py:402-405,422-425): process_images / process_queries ->
    model(**inputs) -> one [T, 128] CPU tensor per item (padding rows included, zero).
    The per-item lists are returned intact: main.py:416,436 torch.cat them into one
    [sum T, 128] tensor, which compute_similarity_scores then splits into single rows
    (SURVEY.md §0.2); mme keeps the list the scorer needs."""
    img_list: List[torch.Tensor] = []
    for i in range(0, len(images), bs):
        out = model(**processor.process_images(images[i:i + bs]).to(device))
        img_list.extend([o.cpu() for o in out])
    txt_list: List[torch.Tensor] = []
    for i in range(0, len(texts), bs):
        out = model(**processor.process_queries(texts[i:i + bs]).to(device))
        txt_list.extend([o.cpu() for o in out])
    return img_list, txt_list
