"""ColPali-v1.3 encoder on the device (the §8a-11 output contract).

The colpali branch of encode_data (main.py:400-405,420-425) calls
`processor.process_images(batch)` / `processor.process_queries(batch)` and then
`model(**inputs)`, which must return a TENSOR [B, L, 128]: per-token embeddings,
L2-normalised, multiplied by attention_mask. The model is ColPali over
PaliGemma-3B (colpali_engine; in-container port
TF:models/colpali/modeling_colpali.py:89-146):

  pixel_values -> SigLIP-448 tower without head (mme.models.VisionTower.forward_tokens)
               -> multi_modal_projector (mme_gemm)                          [B*1024, 2048]
  ids          -> mme_gemma_embed: image features at the <image> slots, bf16(tok * sqrt(d)) elsewhere
  18 x Gemma layer (all libmme): mme_rmsnorm -> QKV mme_gemm -> mme_rope (positions 1..L)
               -> mme_attention_mqa (8 query heads, ONE K/V head, hd 256, bidirectional + key padding)
               -> o_proj mme_gemm (+residual fused) -> mme_rmsnorm
               -> gate|up mme_gemm with the GeGLU epilogue -> down mme_gemm (+residual fused)
  final mme_rmsnorm -> embedding_proj_layer mme_gemm (2048 -> 128) -> mme_l2norm_masked

Weights stay in HBM in kernel layout: q|k|v concatenated [(8+2)*256, 2048];
gate/up interleaved in groups of 4 rows (the GeGLU epilogue pairs them inside
one 16-B output chunk) [2*16384, 2048]. Nothing here computes on the host.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import ops
from ._lib import ACT_GEGLU_TANH
from .config import ColPaliSpec, get_spec
from .models import VisionTower, balanced
from .weights import VisionW, _pad_cols, _sub, pack_layer

BF16 = torch.bfloat16


@dataclass
class GemmaLayerW:
    ln1: torch.Tensor     # input_layernorm.weight [d]
    qkv_w: torch.Tensor   # [(H+2)*hd, d]: q heads | k | v
    o_w: torch.Tensor     # [d, H*hd]
    ln2: torch.Tensor     # post_attention_layernorm.weight
    gu_w: torch.Tensor    # [2I, d]: gate/up interleaved by 4 rows
    down_w: torch.Tensor  # [d, I]


@dataclass
class ColPaliW:
    vision: VisionW
    mmp_w: torch.Tensor   # multi_modal_projector.linear [D, d_vision]
    mmp_b: torch.Tensor
    tok: torch.Tensor     # embed_tokens [V, D]
    layers: List[GemmaLayerW]
    norm_w: torch.Tensor
    head_w: torch.Tensor  # embedding_proj_layer [128, D]
    head_b: torch.Tensor


def interleave_gate_up(gate: torch.Tensor, up: torch.Tensor) -> torch.Tensor:
    """[I, d] x 2 -> [2I, d] with rows 8k..8k+3 = gate 4k..4k+3 and 8k+4..8k+7 = up 4k..4k+3 (mme.h GeGLU)."""
    I, d = gate.shape
    if I % 4:
        raise ValueError("GeGLU: intermediate size must be a multiple of 4")
    return torch.cat([gate.reshape(I // 4, 4, d), up.reshape(I // 4, 4, d)], 1).reshape(2 * I, d).contiguous()


def from_hf_state_dict(spec: ColPaliSpec, sd: Dict[str, torch.Tensor], device="cuda") -> ColPaliW:
    """Pack a transformers ColPaliForRetrieval state dict (vlm.* / embedding_proj_layer.*)."""
    dev = torch.device(device)
    v, t = spec.vision, spec.text

    def b(name):
        return sd[name].to(device=dev, dtype=BF16)

    pre = "vlm.vision_tower."
    vision = VisionW(
        patch_w=_pad_cols(b(pre + "embeddings.patch_embedding.weight").reshape(v.hidden, -1), v.kpad),
        patch_b=b(pre + "embeddings.patch_embedding.bias"), pos=b(pre + "embeddings.position_embedding.weight"),
        cls=None, pre_ln_g=None, pre_ln_b=None,
        layers=[pack_layer(v, _sub(sd, f"{pre}encoder.layers.{i}."), dev) for i in range(v.layers)],
        post_ln_g=b(pre + "post_layernorm.weight"), post_ln_b=b(pre + "post_layernorm.bias"), head=None, proj_w=None)
    layers = []
    for i in range(t.layers):
        p = f"vlm.language_model.layers.{i}."
        layers.append(GemmaLayerW(
            ln1=b(p + "input_layernorm.weight"),
            qkv_w=torch.cat([b(p + "self_attn.q_proj.weight"), b(p + "self_attn.k_proj.weight"),
                             b(p + "self_attn.v_proj.weight")], 0).contiguous(),
            o_w=b(p + "self_attn.o_proj.weight").contiguous(),
            ln2=b(p + "post_attention_layernorm.weight"),
            gu_w=interleave_gate_up(b(p + "mlp.gate_proj.weight"), b(p + "mlp.up_proj.weight")),
            down_w=b(p + "mlp.down_proj.weight").contiguous()))
    return ColPaliW(vision=vision, mmp_w=b("vlm.multi_modal_projector.linear.weight"),
                    mmp_b=b("vlm.multi_modal_projector.linear.bias"), tok=b("vlm.language_model.embed_tokens.weight"),
                    layers=layers, norm_w=b("vlm.language_model.norm.weight"),
                    head_w=b("embedding_proj_layer.weight"), head_b=b("embedding_proj_layer.bias"))


def random_state_dict(spec: ColPaliSpec, seed: int = 0, device="cuda") -> Dict[str, torch.Tensor]:
    """Seeded random weights with the HF ColPaliForRetrieval names (offline stand-in for
    from_pretrained('vidore/colpali-v1.3'))."""
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    dev = torch.device(device)
    sd: Dict[str, torch.Tensor] = {}

    def lin(name, out_f, in_f, bias=True):
        a = math.sqrt(6.0 / (in_f + out_f))
        sd[name + ".weight"] = (torch.rand(out_f, in_f, generator=g, device=dev) * 2 - 1).mul_(a).to(BF16)
        if bias:
            sd[name + ".bias"] = (torch.randn(out_f, generator=g, device=dev) * 0.02).to(BF16)

    def ln(name, d):
        sd[name + ".weight"] = torch.ones(d, dtype=BF16, device=dev)
        sd[name + ".bias"] = torch.zeros(d, dtype=BF16, device=dev)

    v, t = spec.vision, spec.text
    d, pre = v.hidden, "vlm.vision_tower."
    sd[pre + "embeddings.patch_embedding.weight"] = (
        torch.randn(d, 3, v.patch, v.patch, generator=g, device=dev) / math.sqrt(3 * v.patch ** 2)).to(BF16)
    sd[pre + "embeddings.patch_embedding.bias"] = torch.zeros(d, dtype=BF16, device=dev)
    sd[pre + "embeddings.position_embedding.weight"] = (
        torch.randn(v.num_patches, d, generator=g, device=dev) / math.sqrt(d)).to(BF16)
    for i in range(v.layers):
        p = f"{pre}encoder.layers.{i}."
        ln(p + "layer_norm1", d)
        ln(p + "layer_norm2", d)
        for n in ("q_proj", "k_proj", "v_proj", "out_proj"):
            lin(p + "self_attn." + n, d, d)
        lin(p + "mlp.fc1", v.intermediate, d)
        lin(p + "mlp.fc2", d, v.intermediate)
    ln(pre + "post_layernorm", d)
    D, H, hd = t.hidden, t.heads, t.head_dim
    lin("vlm.multi_modal_projector.linear", D, d)
    lm = "vlm.language_model."
    sd[lm + "embed_tokens.weight"] = (torch.randn(t.vocab, D, generator=g, device=dev) / D).to(BF16)
    for i in range(t.layers):
        p = f"{lm}layers.{i}."
        sd[p + "input_layernorm.weight"] = torch.zeros(D, dtype=BF16, device=dev)  # HF init: (1 + 0)
        sd[p + "post_attention_layernorm.weight"] = torch.zeros(D, dtype=BF16, device=dev)
        lin(p + "self_attn.q_proj", H * hd, D, bias=False)
        lin(p + "self_attn.k_proj", hd, D, bias=False)
        lin(p + "self_attn.v_proj", hd, D, bias=False)
        lin(p + "self_attn.o_proj", D, H * hd, bias=False)
        lin(p + "mlp.gate_proj", t.intermediate, D, bias=False)
        lin(p + "mlp.up_proj", t.intermediate, D, bias=False)
        lin(p + "mlp.down_proj", D, t.intermediate, bias=False)
    sd[lm + "norm.weight"] = torch.zeros(D, dtype=BF16, device=dev)
    lin("embedding_proj_layer", spec.dim, D)
    return sd


class _DecBufs:
    def __init__(self, rows: int, spec: ColPaliSpec, device):
        t = spec.text
        self.h = torch.empty(rows, t.hidden, dtype=BF16, device=device)
        self.qkv = torch.empty(rows, (t.heads + 2) * t.head_dim, dtype=BF16, device=device)
        self.attn = torch.empty(rows, t.heads * t.head_dim, dtype=BF16, device=device)
        self.mid = torch.empty(rows, t.intermediate, dtype=BF16, device=device)


def _key_range(attention_mask: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """attention_mask [B, L] (one contiguous block of ones per row, left or right padded)
    -> int32 kstart, kend."""
    m = attention_mask.to(torch.int64)
    B, L = m.shape
    lens = m.sum(1)
    ar = torch.arange(L, device=m.device)
    kstart = torch.where(m.bool(), ar, torch.full_like(ar, L)).amin(1)
    if not torch.equal(m.bool(), (ar >= kstart[:, None]) & (ar < (kstart + lens)[:, None])):
        raise ValueError("attention_mask must be one contiguous run of ones per row")
    if int(lens.min()) == 0:
        raise ValueError("attention_mask has an empty row")
    return kstart.to(torch.int32), (kstart + lens).to(torch.int32)


class ColPaliModel:
    """`model(**inputs) -> Tensor[B, L, 128]` (main.py:404,424), plus fast device paths."""

    family = "colpali"

    def __init__(self, spec: ColPaliSpec, weights: ColPaliW, device="cuda"):
        self.spec = self.config = spec
        self.device = torch.device(device)
        self.w = weights
        self.vision = VisionTower(spec, weights.vision)
        self.dtype = BF16
        self.embed_scale = float(torch.tensor(spec.text.hidden ** 0.5).to(BF16))  # GemmaTextScaledWordEmbedding

    @classmethod
    def from_spec(cls, spec, seed: int = 0, device="cuda", state_dict=None) -> "ColPaliModel":
        spec = get_spec(spec) if isinstance(spec, str) else spec
        sd = state_dict if state_dict is not None else random_state_dict(spec, seed, device)
        return cls(spec, from_hf_state_dict(spec, sd, device), device)

    def eval(self):
        return self

    def to(self, *args, **kwargs):
        return self

    # ---- the decoder stack
    def _decode(self, ids: torch.Tensor, kstart: Optional[torch.Tensor], kend: Optional[torch.Tensor],
                mask_rows: Optional[torch.Tensor], img_feats: Optional[torch.Tensor]) -> torch.Tensor:
        """ids int64 [B, L] on device -> embeddings bf16 [B*L, 128]."""
        spec, t, w = self.spec, self.spec.text, self.w
        B, L = ids.shape
        P = spec.image_seq_len if img_feats is not None else 0
        x = ops.gemma_embed(ids, w.tok, self.embed_scale, img=img_feats, img_prefix=P)
        bufs = _DecBufs(B * L, spec, self.device)
        H, hd = t.heads, t.head_dim
        for lw in w.layers:
            h = ops.rmsnorm(x, lw.ln1, t.eps, out=bufs.h)
            qkv = ops.gemm(h, lw.qkv_w, out=bufs.qkv)
            ops.rope_(qkv, L, H + 1, hd, 1, t.theta)  # q heads + the k head, PaliGemma positions 1..L
            a = ops.attention_mqa(qkv, B, L, H, hd, kstart=kstart, kend=kend, out=bufs.attn)
            ops.gemm(a, lw.o_w, residual=x, out=x)
            h = ops.rmsnorm(x, lw.ln2, t.eps, out=bufs.h)
            mid = ops.gemm(h, lw.gu_w, act=ACT_GEGLU_TANH, out=bufs.mid,
                           algo_flops=2.0 * B * L * t.hidden * 2 * t.intermediate)
            ops.gemm(mid, lw.down_w, residual=x, out=x)
        h = ops.rmsnorm(x, w.norm_w, t.eps, out=bufs.h)
        e = ops.gemm(h, w.head_w, w.head_b)
        return ops.l2norm_masked(e, mask_rows, out=e)

    def _image_features(self, patches: torch.Tensor, B: int) -> torch.Tensor:
        feats = self.vision.forward_tokens(patches, B)
        return ops.gemm(feats, self.w.mmp_w, self.w.mmp_b)  # multi_modal_projector

    # ---- HF / colpali_engine surface
    @torch.no_grad()
    def __call__(self, input_ids: torch.Tensor, attention_mask: Optional[torch.Tensor] = None,
                 pixel_values: Optional[torch.Tensor] = None, token_type_ids: Optional[torch.Tensor] = None,
                 **_) -> torch.Tensor:
        spec = self.spec
        ids = input_ids.to(self.device, torch.int64)
        B, L = ids.shape
        if token_type_ids is not None and bool((token_type_ids != 0).any()):
            raise NotImplementedError("suffix (token_type_ids == 1) tokens: ColPali inputs are all prefix")
        if attention_mask is None:
            attention_mask = torch.ones(B, L, dtype=torch.int64, device=self.device)
        am = attention_mask.to(self.device, torch.int64)
        kstart, kend = _key_range(am)
        img = None
        if pixel_values is not None:
            P = spec.image_seq_len
            if not bool((ids[:, :P] == spec.image_token_id).all()) or bool((ids[:, P:] == spec.image_token_id).any()):
                raise ValueError(f"expected the {P} <image> tokens to lead every sequence (ColPali layout)")
            pv = pixel_values.to(self.device)
            img = self._image_features(ops.im2col(pv, spec.vision.patch, spec.vision.kpad), B)
        e = self._decode(ids, kstart, kend, am.reshape(-1), img)
        return e.view(B, L, spec.dim)

    # ---- fast device paths
    @torch.no_grad()
    def encode_images(self, images_u8: torch.Tensor, batch: int = 16) -> torch.Tensor:
        """u8 [n, H, W, 3] device images -> per-token embeddings bf16 [n, L_img, 128]
        (L_img = 1024 image tokens + bos + prompt + newline; no padding)."""
        from .processor import image_geometry
        spec = self.spec
        v, ip = spec.vision, spec.image_proc
        n, H, W, _ = images_u8.shape
        rh, rw, top, left = image_geometry(H, W, ip)
        toks = torch.tensor(spec.image_tokens, dtype=torch.int64, device=self.device)
        L = toks.numel()
        out = torch.empty(n, L, spec.dim, dtype=BF16, device=self.device)
        batch = balanced(n, batch)
        for i in range(0, n, batch):
            chunk = images_u8[i:i + batch]
            b = chunk.shape[0]
            patches = ops.preprocess_u8(chunk, resize=(rh, rw), crop=(top, left), size=ip.size, mean=ip.mean,
                                        std=ip.std, patch=v.patch, kpad=v.kpad)
            img = self._image_features(patches, b)
            e = self._decode(toks.expand(b, L).contiguous(), None, None, None, img)
            out[i:i + b] = e.view(b, L, spec.dim)
        return out

    @torch.no_grad()
    def encode_queries(self, captions: Sequence[Sequence[int]], ref_batch: Optional[int] = None,
                       exec_batch: int = 256, width: Optional[int] = None
                       ) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        """Caption token lists -> (Q bf16 [n, Lmax, 128] valid rows first then zeros,
        lens int32 [n] (valid rows), padded int32 [n] (the caption's padded length L_b)).

        Reproduces processor.process_queries(batch) per reference batch of `ref_batch`
        (main.py:420-424): left padding to the batch-longest, positions 1..L_b over the
        padded row; captions with equal L_b run in one execution batch (their
        embeddings depend only on L_b). width: fixed row count of Q (a multiple of 16 >= the
        longest query; equal widths let ranks all-gather their tables)."""
        spec = self.spec
        ref_batch = ref_batch or spec.batch_size
        rows = [spec.query_tokens(c) for c in captions]
        n = len(rows)
        lens = np.array([len(r) for r in rows], np.int64)
        padded = np.empty(n, np.int64)
        for s in range(0, n, ref_batch):
            padded[s:s + ref_batch] = lens[s:s + ref_batch].max()
        Lmax = -(-int(lens.max()) // 16) * 16 if n else 16  # zero rows up to a multiple of 16 (mme_maxsim)
        if width is not None:
            if width % 16 or width < Lmax:
                raise ValueError(f"width {width} must be a multiple of 16 >= {Lmax}")
            Lmax = width
        Q = torch.zeros(n, Lmax, spec.dim, dtype=BF16, device=self.device)
        for Lb in sorted(set(padded.tolist())):
            idx = np.nonzero(padded == Lb)[0]
            eb = balanced(len(idx), exec_batch)
            for j in range(0, len(idx), eb):
                part = idx[j:j + eb]
                b = len(part)
                ids = np.full((b, Lb), spec.pad_id, np.int64)
                for r, i in enumerate(part):
                    ids[r, Lb - lens[i]:] = rows[i]
                ks = torch.from_numpy((Lb - lens[part]).astype(np.int32)).to(self.device)
                ke = torch.full((b,), Lb, dtype=torch.int32, device=self.device)
                e = self._decode(torch.from_numpy(ids).to(self.device), ks, ke, None, None)
                # compact the valid (right-aligned) rows to the front: one gather per batch
                src = np.full((b, Lmax), b * Lb, np.int64)  # b*Lb -> an appended zero row
                for r, i in enumerate(part):
                    src[r, : lens[i]] = r * Lb + (Lb - lens[i]) + np.arange(lens[i])
                ez = torch.cat([e, torch.zeros(1, spec.dim, dtype=BF16, device=self.device)])
                Q[torch.from_numpy(part).to(self.device)] = ez.index_select(
                    0, torch.from_numpy(src.reshape(-1)).to(self.device)).view(b, Lmax, spec.dim)
        lens_t = torch.from_numpy(lens.astype(np.int32)).to(self.device)
        return Q, lens_t, torch.from_numpy(padded.astype(np.int32)).to(self.device)


class ColPaliProcessor:
    """process_images / process_queries / score (main.py:403,423,467) over the device path.

    Images: u8 arrays / PIL -> pixel_values by the PIL-exact preprocess kernel (448 square).
    Queries: pre-tokenized id lists (the spec adds bos, the query prefix ids, the augmentation pads and
    the newline), or strings through the checkpoint's tokenizer (`tokenizer=`: an HF-compatible
    callable). A string is laid out the way ColPaliProcessor.__call__ does it,
    f"{bos_token}{query_prefix}{query}{pad_token * 10}\n" (TF:models/colpali/processing_colpali.py,
    __call__), and that WHOLE string is tokenized in one call (`add_special_tokens=False`: the bos is
    in the text), so SentencePiece merges across the prefix / query seam exactly as for the reference.
    Without a tokenizer, strings raise unless `allow_hash_tokenizer=True` selects the offline
    word-hash stand-in (body hashed, spec layout). Left padding to the batch-longest."""

    def __init__(self, spec: ColPaliSpec, device="cuda", tokenizer=None, allow_hash_tokenizer: bool = False):
        from .colpali import ColPaliScorer
        from .config import TextConfig
        from .processor import HashTokenizer, Processor
        self.spec = spec
        self.device = torch.device(device)
        t = spec.text
        self.text_tokenizer = tokenizer
        self.tokenizer = None
        if tokenizer is None and allow_hash_tokenizer:
            self.tokenizer = HashTokenizer(t.vocab, spec.bos_id, spec.eos_id, spec.pad_id, 1 << 20, reserved=3)
            self.tokenizer.hi = min(self.tokenizer.hi, spec.image_token_id)  # never emit <image>
            self.tokenizer.lo = max(self.tokenizer.lo, spec.newline_id + 1)
        shim = type("S", (), {"image_proc": spec.image_proc,
                              "text": TextConfig(hidden=1, intermediate=1, layers=0, heads=1, act="none", eps=0.0)})
        self._img = Processor(shim, device=device)
        self._scorer = ColPaliScorer(device=device)

    def _batch(self, rows: List[Sequence[int]]):
        from .processor import BatchFeature
        L = max(len(r) for r in rows)
        ids = torch.full((len(rows), L), self.spec.pad_id, dtype=torch.int64)
        mask = torch.zeros((len(rows), L), dtype=torch.int64)
        for i, r in enumerate(rows):
            ids[i, L - len(r):] = torch.tensor(list(r), dtype=torch.int64)
            mask[i, L - len(r):] = 1
        return BatchFeature(input_ids=ids, attention_mask=mask, token_type_ids=torch.zeros_like(ids))

    def process_images(self, images, **_):
        b = self._batch([self.spec.image_tokens] * len(images))
        b["pixel_values"] = self._img.pixel_values(images)
        return b

    def process_queries(self, queries, **_):
        from .processor import _as_rows, _ids, no_string_tokenizer
        strs = [q for q in queries if isinstance(q, str)]
        full = iter(())
        if strs and self.text_tokenizer is not None:
            full = iter(_as_rows(_ids(self.text_tokenizer([self.query_string(q) for q in strs],
                                                          add_special_tokens=False, padding=False, truncation=False))))
        elif strs and self.tokenizer is None:
            raise no_string_tokenizer("ColPaliProcessor.process_queries")
        rows = [(list(next(full)) if self.text_tokenizer is not None else
                 self.spec.query_tokens(self.tokenizer.encode(q)))
                if isinstance(q, str) else self.spec.query_tokens([int(x) for x in q]) for q in queries]
        return self._batch(rows)

    def query_string(self, query: str) -> str:
        """ColPaliProcessor.__call__'s text layout: bos + query prefix + query + 10 augmentation pads + newline."""
        tok = self.text_tokenizer
        bos = getattr(tok, "bos_token", None) or "<bos>"
        pad = getattr(tok, "pad_token", None) or "<pad>"
        return f"{bos}{self.spec.query_prefix}{query}{pad * self.spec.n_aug}\n"

    def score(self, qs, ps, **kw):
        return self._scorer.score(qs, ps, **kw)


def load_colpali(name: str = "ColPali-v1.3", seed: int = 0, device="cuda", state_dict=None, tokenizer=None,
                 allow_hash_tokenizer: bool = False):
    """(model, processor) — the offline counterpart of ColPali.from_pretrained / ColPaliProcessor
    (main.py:808-812); `tokenizer` / `allow_hash_tokenizer` as ColPaliProcessor."""
    spec = get_spec(name)
    return ColPaliModel.from_spec(spec, seed=seed, device=device, state_dict=state_dict), \
        ColPaliProcessor(spec, device=device, tokenizer=tokenizer, allow_hash_tokenizer=allow_hash_tokenizer)
