"""Winoground 2x2 scorer.

Restates run_winoground (run_benchmark_grand_slam_v28_publication_ready.py:413-461):
per example, the two captions and the two images are encoded as one batch each
(padding to the longer caption), L2-normalised in the model dtype, scored with a
bf16 torch.matmul (s[t][i] = bf16 <text_t, image_i>), and counted with the
reference's strict comparisons: text s00>s01 & s11>s10, image s00>s10 & s11>s01,
group both. ColPali scores the pair with processor.score (MaxSim).

Dense models run batched on the device: all 2n images through encode_images,
all 2n captions through encode_texts with reference batches of 2 (each example's
own padding reproduced), then one mme_winoground launch. The dataset
(facebook/winoground) is not available offline; examples are any iterable of
dicts with image_0 / image_1 (PIL or HxWx3 u8) and caption_0 / caption_1
(strings or token-id lists).
"""
from __future__ import annotations

from typing import Dict, Iterable, List

import numpy as np
import torch

from . import ops


def _counts_to_metrics(text: int, image: int, group: int, total: int) -> Dict[str, float]:
    return {"Wino Text": 100.0 * text / total, "Wino Image": 100.0 * image / total,
            "Wino Group": 100.0 * group / total}


@torch.no_grad()
def winoground_scores(model, processor, examples: List[dict]):
    """Device path for the dual encoders: (scores fp32 [n, 4], counts int64 [3])."""
    from .processor import to_u8_nhwc
    n = len(examples)
    imgs = [to_u8_nhwc(ex[f"image_{j}"]) for ex in examples for j in (0, 1)]
    emb_i = torch.empty(2 * n, model.spec.proj_dim, dtype=torch.bfloat16, device=model.device)
    for idx, u8 in processor.images_to_u8(imgs):  # groups of equal-size images
        e = model.encode_images(u8)
        emb_i[torch.tensor(idx, device=model.device)] = e
    rows = processor.tokenize([ex[f"caption_{j}"] for ex in examples for j in (0, 1)])
    lens = [len(r) for r in rows]
    pad = model.spec.text.pad_id
    ids = torch.full((2 * n, max(lens)), pad, dtype=torch.int64)
    for i, r in enumerate(rows):
        ids[i, : len(r)] = torch.tensor(r, dtype=torch.int64)
    emb_t = model.encode_texts(ids.to(model.device), torch.tensor(lens), ref_batch=2)
    return ops.winoground(emb_t.view(n, 2, -1), emb_i.view(n, 2, -1))


@torch.no_grad()
def run_winoground(model, processor, m_info: dict, examples: Iterable[dict]) -> Dict[str, float]:
    """The reference's run_winoground over the given examples (metrics in percent)."""
    examples = list(examples)
    if not examples:
        return {}
    if m_info.get("type") == "colpali":
        t = i = g = 0
        for ex in examples:
            bi = processor.process_images([ex["image_0"], ex["image_1"]]).to(model.device)
            bq = processor.process_queries([ex["caption_0"], ex["caption_1"]]).to(model.device)
            s = processor.score(model(**bq), model(**bi)).float().cpu()
            txt = bool(s[0, 0] > s[0, 1] and s[1, 1] > s[1, 0])
            img = bool(s[0, 0] > s[1, 0] and s[1, 1] > s[0, 1])
            t, i, g = t + txt, i + img, g + (txt and img)
        return _counts_to_metrics(t, i, g, len(examples))
    _, counts = winoground_scores(model, processor, examples)
    c = counts.tolist()
    return _counts_to_metrics(c[0], c[1], c[2], len(examples))


def synthetic_examples(n: int, caption_ids: bool = True, seed: int = 0, size: int = 64, vocab=(3, 990),
                       lens=(4, 12)) -> List[dict]:
    """Deterministic stand-in examples (u8 images, token-id captions)."""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        ex = {f"image_{j}": rng.integers(0, 256, (size, size, 3), dtype=np.uint8) for j in (0, 1)}
        for j in (0, 1):
            ex[f"caption_{j}"] = rng.integers(vocab[0], vocab[1], int(rng.integers(*lens))).tolist()
        out.append(ex)
    return out
