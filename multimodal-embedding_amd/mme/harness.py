"""Benchmark driver: the data layout, timing region and CSV of the reference.

Restates run_bootstrap_benchmark (main.py:478-667) for the device-resident
path:
  * images in dataset order; captions all_captions[5i + j] = caption j of
    image i; T2I queries = caption 0 of each image (main.py:503-529);
  * timed region = encode n images + n T2I captions + 5n captions
    (main.py:534-559) plus both score directions and recall (the v28
    definition the published QPS uses, …v28_publication_ready.py:305-408);
    warmup runs outside the region (v28);
  * metrics on the identity sample, I2T orientation fixed;
  * CSV columns of main.py:642-665 (identity sample: mean = lower = upper,
    std = 0).
"""
from __future__ import annotations

import csv
import time
from typing import Dict, List, Optional

import torch

from .retrieval import KS, compute_metrics

METRIC_KEYS = [f"{p}_R@{k}" for p in ("T2I", "I2T", "I2T_Sym") for k in KS]


def encode_job(model, images_u8: torch.Tensor, caption_ids: torch.Tensor, caption_lens: Optional[torch.Tensor] = None,
               caps_per_image: int = 5, img_batch: Optional[int] = None, txt_batch: Optional[int] = None):
    """Encode n images, their caption-0 T2I queries and all 5n captions (main.py:551-557). Execution
    batches default to the measured geometry bench.py runs (mme.config.exec_batches)."""
    from .config import exec_batches
    eb_img, eb_txt = exec_batches(model.spec)
    img_batch = eb_img if img_batch is None else img_batch
    txt_batch = eb_txt if txt_batch is None else txt_batch
    n = images_u8.shape[0]
    img = model.encode_images(images_u8, batch=img_batch)
    sel = torch.arange(0, caps_per_image * n, caps_per_image, device=caption_ids.device)
    t2i_ids = caption_ids.index_select(0, sel)
    t2i_lens = None if caption_lens is None else caption_lens.index_select(0, sel.to(caption_lens.device))
    t2i = model.encode_texts(t2i_ids, t2i_lens, exec_batch=txt_batch)
    all_txt = model.encode_texts(caption_ids, caption_lens, exec_batch=txt_batch)
    return img, t2i, all_txt


def run_benchmark(model, images_u8: torch.Tensor, caption_ids: torch.Tensor, caption_lens=None,
                  caps_per_image: int = 5, warmup: bool = True, n_iterations: int = 0, seed: int = 0,
                  **kw) -> Dict[str, object]:
    """One timed encode + retrieval job; returns the reference's result row.

    n_iterations > 0: the metrics are the bootstrap of run_bootstrap_benchmark
    (main.py:563-651: resamples with replacement, mean / 95 % CI / std per metric) on
    the device (mme.bootstrap); 0: the identity sample (mean = lower = upper, std 0)."""
    name = model.spec.name
    if warmup:  # v28: warmup outside the timed region
        encode_job(model, images_u8[:2], caption_ids[: 2 * caps_per_image], None if caption_lens is None else
                   caption_lens[: 2 * caps_per_image], caps_per_image, **kw)
    torch.cuda.synchronize()
    t0 = time.time()
    img, t2i, all_txt = encode_job(model, images_u8, caption_ids, caption_lens, caps_per_image, **kw)
    torch.cuda.synchronize()
    t_enc = time.time() - t0
    n = images_u8.shape[0]
    row: Dict[str, object] = {"Model": name}
    if n_iterations > 0:
        from . import bootstrap as mb
        s_t2i, s_i2t = mb.full_scores(img, t2i, all_txt)
        hits = mb.bootstrap_hits(s_t2i, s_i2t, mb.sample_indices(n, n_iterations, seed, img.device), caps_per_image)
        row.update(mb.bootstrap_row(hits, n, seed=seed))
    else:
        metrics = compute_metrics(img, t2i, all_txt, caps_per_image)
        for k in METRIC_KEYS:
            v = metrics[k]
            row[f"{k}_mean"], row[f"{k}_lower"], row[f"{k}_upper"], row[f"{k}_std"] = v, v, v, 0.0
    torch.cuda.synchronize()
    t_total = time.time() - t0
    row["Time"] = t_total
    row["QPS"] = n / t_total
    row["Encoding_Time"] = t_enc
    row["Img_per_sec"] = n / t_enc
    row["_failure_analysis"] = {}
    return row


def write_csv(rows: List[Dict[str, object]], path: str) -> None:
    """pd.DataFrame(final_results).to_csv(path) equivalent (main.py:835-836; index column kept)."""
    if not rows:
        return
    cols = list(rows[0].keys())
    for r in rows[1:]:
        for k in r:
            if k not in cols:
                cols.append(k)
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow([""] + cols)
        for i, r in enumerate(rows):
            w.writerow([i] + [r.get(c, "") for c in cols])
