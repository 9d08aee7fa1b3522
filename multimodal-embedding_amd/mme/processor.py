"""Processor duck type: processor(images=...) / processor(text=...).

Images: the PIL-exact bicubic resize + crop + rescale + normalise of the HF
PIL backend (main.py:407 -> image_processing_backends.PilBackend._preprocess)
runs on the device (libmme mme_preprocess_u8); this module only turns PIL
images / arrays into a u8 NHWC tensor and computes the resize geometry.

Text: the reference tokenizes with the model's HF tokenizer (main.py:427,
padding=True, truncation=True). A caller that has the checkpoint's tokenizer
passes it (`Processor(spec, tokenizer=tok)`, `load_model(..., tokenizer=tok)`):
any HF-compatible callable `tok(batch, padding=..., truncation=..., max_length=...)`
returning `input_ids` / `attention_mask`. A batch of strings is then handed to it
whole, exactly as main.py:427 does, and its padding / mask come back unchanged.
Pre-tokenized id lists pass through unchanged, padded here with HF's semantics:
right padding to the batch's longest row with pad_id, attention_mask 1/0,
truncation to max_pos keeping the trailing eos. Strings with no tokenizer raise:
the offline vocab-free stand-in (`HashTokenizer`, deterministic word hashes with
the model's special tokens) must be asked for explicitly with
`allow_hash_tokenizer=True`, so real captions are never silently hashed.
"""
from __future__ import annotations

import zlib
from typing import List, Optional, Sequence, Tuple, Union

import numpy as np
import torch

from . import ops
from .config import ImageProcConfig, ModelSpec


def image_geometry(H: int, W: int, ip: ImageProcConfig) -> Tuple[int, int, int, int]:
    """(resize_h, resize_w, crop_top, crop_left) for an H x W image.

    square: resize to S x S (SigLIP, image_processing_pil_siglip.py:26-35).
    shortest_edge: transformers get_resize_output_image_size(default_to_square=False)
    then center_crop (S, S) (image_processing_pil_clip.py:24-39)."""
    S = ip.size
    if ip.mode == "square":
        return S, S, 0, 0
    short, long = (W, H) if W <= H else (H, W)
    new_short, new_long = S, int(S * long / short)
    rh, rw = (new_long, new_short) if W <= H else (new_short, new_long)
    top = (rh - S) // 2
    left = (rw - S) // 2
    return rh, rw, top, left


class BatchFeature(dict):
    """Minimal transformers.BatchFeature: a dict with .to(device)."""

    def to(self, device):
        return BatchFeature({k: (v.to(device) if isinstance(v, torch.Tensor) else v) for k, v in self.items()})

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e


def to_u8_nhwc(img) -> np.ndarray:
    """PIL image / HxWx3 array -> contiguous uint8 RGB HxWx3 (convert_rgb as HF does)."""
    if hasattr(img, "convert"):  # PIL
        img = np.asarray(img.convert("RGB"))
    a = np.asarray(img)
    if a.dtype != np.uint8 or a.ndim != 3 or a.shape[2] != 3:
        raise ValueError(f"expected uint8 HxWx3 image, got {a.dtype} {a.shape}")
    return np.ascontiguousarray(a)


class HashTokenizer:
    """Deterministic offline stand-in for the model tokenizer (no vocab files offline)."""

    def __init__(self, vocab: int, bos: Optional[int], eos: int, pad: int, max_len: int, reserved: int = 3):
        self.vocab, self.bos, self.eos, self.pad, self.max_len = vocab, bos, eos, pad, max_len
        specials = {x for x in (bos, eos, pad) if x is not None}
        self.lo = reserved
        self.hi = min(specials | {vocab}) if min(specials) > reserved else vocab
        if self.hi - self.lo < 16:
            self.lo, self.hi = max(specials) + 1, vocab

    def encode(self, text: str) -> List[int]:
        span = self.hi - self.lo
        return [self.lo + zlib.crc32(w.encode()) % span for w in text.lower().split()]


def _as_rows(x) -> List[List[int]]:
    """input_ids of a tokenizer's output (tensor, array or nested lists) -> list of int lists."""
    if isinstance(x, torch.Tensor):
        x = x.tolist()
    elif isinstance(x, np.ndarray):
        x = x.tolist()
    return [[int(v) for v in r] for r in x]


def _ids(enc):
    """`input_ids` of a BatchEncoding / dict / object returned by a tokenizer."""
    try:
        return enc["input_ids"]
    except (KeyError, TypeError):
        return enc.input_ids


def _mask(enc):
    try:
        return enc["attention_mask"]
    except (KeyError, TypeError):
        return getattr(enc, "attention_mask", None)


def no_string_tokenizer(what: str) -> ValueError:
    return ValueError(
        f"{what} got caption strings but no tokenizer: pass the checkpoint's tokenizer (tokenizer=...), "
        "pre-tokenized id lists, or allow_hash_tokenizer=True for the offline word-hash stand-in")


class Processor:
    """processor(images=..., text=..., return_tensors='pt', padding=True, truncation=True).

    tokenizer: the model's HF-compatible tokenizer (called on batches of strings, main.py:427);
    allow_hash_tokenizer: without one, hash strings with the offline stand-in instead of raising."""

    def __init__(self, spec: ModelSpec, device="cuda", tokenizer=None, allow_hash_tokenizer: bool = False):
        self.spec = spec
        self.device = torch.device(device)
        t = spec.text
        self.text_tokenizer = tokenizer
        self.tokenizer = HashTokenizer(t.vocab, t.bos_id, t.eos_id, t.pad_id, t.max_pos) \
            if tokenizer is None and allow_hash_tokenizer else None

    # ---- images
    def images_to_u8(self, images) -> List[torch.Tensor]:
        """Group images by size -> list of (indices, u8 [n,H,W,3] device tensor)."""
        if isinstance(images, torch.Tensor):
            return [(list(range(images.shape[0])), images.to(self.device))]
        arrs = [to_u8_nhwc(im) for im in images]
        groups = {}
        for i, a in enumerate(arrs):
            groups.setdefault(a.shape, []).append(i)
        out = []
        for shape, idx in groups.items():
            stack = np.stack([arrs[i] for i in idx])
            out.append((idx, torch.from_numpy(stack).to(self.device)))
        return out

    def pixel_values(self, images) -> torch.Tensor:
        ip = self.spec.image_proc
        groups = self.images_to_u8(images)
        n = sum(len(i) for i, _ in groups)
        pv = torch.empty(n, 3, ip.size, ip.size, dtype=torch.float32, device=self.device)
        for idx, u8 in groups:
            _, H, W, _ = u8.shape
            rh, rw, top, left = image_geometry(H, W, ip)
            res = ops.preprocess_u8(u8, resize=(rh, rw), crop=(top, left), size=ip.size, mean=ip.mean, std=ip.std)
            pv[torch.tensor(idx, device=self.device)] = res
        return pv

    # ---- text
    def tokenize(self, texts: Sequence[Union[str, Sequence[int]]], truncation: bool = True) -> List[List[int]]:
        """Unpadded id rows; strings go to the tokenizer (padding=False) or the explicit hash stand-in."""
        t = self.spec.text
        strs = [x for x in texts if isinstance(x, str)]
        delegated = iter(())
        if strs and self.text_tokenizer is not None:
            delegated = iter(_as_rows(_ids(self.text_tokenizer(
                strs, padding=False, truncation=truncation, max_length=t.max_pos))))
        elif strs and self.tokenizer is None:
            raise no_string_tokenizer("Processor")
        rows = []
        for x in texts:
            if isinstance(x, str) and self.text_tokenizer is not None:
                rows.append(next(delegated))
            elif isinstance(x, str):
                body = self.tokenizer.encode(x)
                pre = [t.bos_id] if t.bos_id is not None else []
                room = t.max_pos - len(pre) - 1
                if truncation:
                    body = body[:max(room, 0)]
                rows.append(pre + body + [t.eos_id])
            else:
                ids = [int(v) for v in x]
                if truncation and len(ids) > t.max_pos:
                    ids = ids[: t.max_pos - 1] + [ids[-1]]  # keep the trailing eos
                rows.append(ids)
        return rows

    def pad(self, rows: List[List[int]]) -> BatchFeature:
        t = self.spec.text
        L = max(len(r) for r in rows)
        ids = torch.full((len(rows), L), t.pad_id, dtype=torch.int64)
        mask = torch.zeros((len(rows), L), dtype=torch.int64)
        for i, r in enumerate(rows):
            ids[i, : len(r)] = torch.tensor(r, dtype=torch.int64)
            mask[i, : len(r)] = 1
        return BatchFeature(input_ids=ids, attention_mask=mask)

    def __call__(self, images=None, text=None, return_tensors: str = "pt", padding: bool = True,
                 truncation: bool = True, **_) -> BatchFeature:
        if images is not None and text is not None:
            raise ValueError("call the processor with images or text, not both (main.py:407,427)")
        if images is not None:
            return BatchFeature(pixel_values=self.pixel_values(images))
        if text is None:
            raise ValueError("processor needs images= or text=")
        if isinstance(text, str):
            text = [text]
        if self.text_tokenizer is not None and text and all(isinstance(x, str) for x in text):
            # main.py:427: the checkpoint's tokenizer pads and masks the batch itself
            enc = self.text_tokenizer(list(text), padding=padding, truncation=truncation,
                                      max_length=self.spec.text.max_pos, return_tensors="pt")
            ids = torch.as_tensor(_ids(enc), dtype=torch.int64)
            m = _mask(enc)
            mask = torch.ones_like(ids) if m is None else torch.as_tensor(m, dtype=torch.int64)
            return BatchFeature(input_ids=ids, attention_mask=mask)
        return self.pad(self.tokenize(text, truncation=truncation))


def synthetic_images(n: int, H: int = 224, W: int = 224, seed: int = 0) -> np.ndarray:
    """SURVEY.md §8d synthetic images: default_rng(seed).integers(0,256,(n,H,W,3),uint8)."""
    return np.random.default_rng(seed).integers(0, 256, (n, H, W, 3), dtype=np.uint8)


def synthetic_caption_ids(spec: ModelSpec, n: int, seed: int = 1) -> np.ndarray:
    """SURVEY.md §8d synthetic captions (fixed length, no padding).

    CLIP: [bos] + 75 ids ~ U[1, eos-2] + [eos] (L = 77);
    SigLIP: 63 ids ~ U[2, vocab-1] + [eos] (L = 64, the truncation limit)."""
    t = spec.text
    rng = np.random.default_rng(seed)
    L = t.max_pos
    if t.bos_id is not None:
        body = rng.integers(1, min(t.bos_id, t.eos_id), (n, L - 2), dtype=np.int64)
        return np.concatenate([np.full((n, 1), t.bos_id), body, np.full((n, 1), t.eos_id)], axis=1)
    body = rng.integers(2, t.vocab, (n, L - 1), dtype=np.int64)
    return np.concatenate([body, np.full((n, 1), t.eos_id)], axis=1)
