"""PyTorch-CPU restatement of the SigLIP / CLIP towers + encode_data (oracle).

Follows the transformers 5.15 modules the reference instantiates through
from_pretrained (main.py:808-820):
  * SiglipVisionEmbeddings / SiglipTextEmbeddings  TF:models/siglip/modeling_siglip.py:116-224
  * attention (SDPA, fp32 softmax)               TF:models/siglip/modeling_siglip.py:228-247
  * SiglipEncoderLayer (pre-LN)                    TF:models/siglip/modeling_siglip.py:325-357
  * SiglipTextTransformer pooling h[:, -1] + head  TF:models/siglip/modeling_siglip.py:520-546
  * post_layernorm + MAP head                      TF:models/siglip/modeling_siglip.py:611-644
  * CLIPVisionEmbeddings + pre_layrnorm, CLS pool,
    visual_projection                              TF:models/clip/modeling_clip.py:203-218,642-656,751
  * CLIP text causal mask + EOT pooling            TF:models/clip/modeling_clip.py:543-581,713
and encode_data (main.py:386-438): batches of bs, L2-normalise in the model
dtype, cast to bf16.

dtype=float32 is the parity oracle; dtype=bfloat16 is the timed CPU baseline
(the reference's own CPU path runs these modules in bf16). Pinned against
tests/golden/tiny-*.npz (outputs of the reference's encode_data).
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch
import torch.nn.functional as F

from . import pil_bicubic


def _act(name: str, x: torch.Tensor) -> torch.Tensor:
    if name == "gelu_pytorch_tanh":
        return F.gelu(x, approximate="tanh")
    if name == "quick_gelu":
        return x * torch.sigmoid(1.702 * x)
    if name == "gelu":
        return F.gelu(x)
    raise ValueError(name)


def _attn(x, p, cfg, mask: Optional[torch.Tensor]):
    B, T, d = x.shape
    H = cfg.heads
    hd = d // H
    q = F.linear(x, p["self_attn.q_proj.weight"], p["self_attn.q_proj.bias"]).view(B, T, H, hd).transpose(1, 2)
    k = F.linear(x, p["self_attn.k_proj.weight"], p["self_attn.k_proj.bias"]).view(B, T, H, hd).transpose(1, 2)
    v = F.linear(x, p["self_attn.v_proj.weight"], p["self_attn.v_proj.bias"]).view(B, T, H, hd).transpose(1, 2)
    # scaled_dot_product_attention: the attention the reference's from_pretrained models run by
    # default (attn_implementation="sdpa", TF:models/siglip/modeling_siglip.py:228-247 is its eager
    # twin); its CPU kernel keeps the softmax in fp32 and never materialises [B, H, T, T]
    o = F.scaled_dot_product_attention(q, k, v, attn_mask=mask, scale=hd ** -0.5)
    o = o.transpose(1, 2).reshape(B, T, d)
    return F.linear(o, p["self_attn.out_proj.weight"], p["self_attn.out_proj.bias"])


def _layer(x, p, cfg, mask):
    h = F.layer_norm(x, (x.shape[-1],), p["layer_norm1.weight"], p["layer_norm1.bias"], cfg.eps)
    x = x + _attn(h, p, cfg, mask)
    h = F.layer_norm(x, (x.shape[-1],), p["layer_norm2.weight"], p["layer_norm2.bias"], cfg.eps)
    h = F.linear(_act(cfg.act, F.linear(h, p["mlp.fc1.weight"], p["mlp.fc1.bias"])), p["mlp.fc2.weight"],
                 p["mlp.fc2.bias"])
    return x + h


def _sub(sd, prefix):
    n = len(prefix)
    return {k[n:]: v for k, v in sd.items() if k.startswith(prefix)}


def _ln(x, sd, name, eps):
    return F.layer_norm(x, (x.shape[-1],), sd[name + ".weight"], sd[name + ".bias"], eps)


def vision_forward(spec, sd: Dict[str, torch.Tensor], pixel_values: torch.Tensor) -> torch.Tensor:
    v = spec.vision
    dt = sd["vision_model.post_layernorm.weight"].dtype
    x = F.conv2d(pixel_values.to(dt), sd["vision_model.embeddings.patch_embedding.weight"],
                 sd.get("vision_model.embeddings.patch_embedding.bias"), stride=v.patch)
    x = x.flatten(2).transpose(1, 2)
    B = x.shape[0]
    if spec.family == "clip":
        cls = sd["vision_model.embeddings.class_embedding"].expand(B, 1, -1)
        x = torch.cat([cls, x], 1)
    x = x + sd["vision_model.embeddings.position_embedding.weight"]
    if spec.family == "clip":
        x = _ln(x, sd, "vision_model.pre_layrnorm", v.eps)
    for i in range(v.layers):
        x = _layer(x, _sub(sd, f"vision_model.encoder.layers.{i}."), v, None)
    if spec.family == "clip":
        pooled = _ln(x[:, 0], sd, "vision_model.post_layernorm", v.eps)
        return F.linear(pooled, sd["visual_projection.weight"])
    x = _ln(x, sd, "vision_model.post_layernorm", v.eps)
    d = v.hidden
    probe = sd["vision_model.head.probe"].expand(B, 1, d)
    in_w, in_b = sd["vision_model.head.attention.in_proj_weight"], sd["vision_model.head.attention.in_proj_bias"]
    H, hd = v.heads, d // v.heads
    q = F.linear(probe, in_w[:d], in_b[:d]).view(B, 1, H, hd).transpose(1, 2)
    k = F.linear(x, in_w[d:2 * d], in_b[d:2 * d]).view(B, -1, H, hd).transpose(1, 2)
    val = F.linear(x, in_w[2 * d:], in_b[2 * d:]).view(B, -1, H, hd).transpose(1, 2)
    w = torch.softmax(torch.matmul(q, k.transpose(-1, -2)) * hd ** -0.5, dim=-1, dtype=torch.float32).to(q.dtype)
    a = torch.matmul(w, val).transpose(1, 2).reshape(B, 1, d)
    y = F.linear(a, sd["vision_model.head.attention.out_proj.weight"], sd["vision_model.head.attention.out_proj.bias"])
    z = _ln(y, sd, "vision_model.head.layernorm", v.eps)
    z = F.linear(_act(v.act, F.linear(z, sd["vision_model.head.mlp.fc1.weight"], sd["vision_model.head.mlp.fc1.bias"])),
                 sd["vision_model.head.mlp.fc2.weight"], sd["vision_model.head.mlp.fc2.bias"])
    return (y + z)[:, 0]


def text_forward(spec, sd: Dict[str, torch.Tensor], ids: torch.Tensor,
                 attention_mask: Optional[torch.Tensor] = None) -> torch.Tensor:
    t = spec.text
    B, L = ids.shape
    x = sd["text_model.embeddings.token_embedding.weight"][ids] + \
        sd["text_model.embeddings.position_embedding.weight"][:L]
    dt = x.dtype
    neg = torch.finfo(dt).min
    mask = torch.zeros(B, 1, L, L, dtype=dt)
    if attention_mask is not None:
        mask = mask.masked_fill(attention_mask[:, None, None, :] == 0, neg)
    if t.causal:
        mask = mask.masked_fill(torch.triu(torch.ones(L, L, dtype=torch.bool), 1), neg)
    use_mask = bool(t.causal or (attention_mask is not None and not bool(attention_mask.all())))
    for i in range(t.layers):
        x = _layer(x, _sub(sd, f"text_model.encoder.layers.{i}."), t, mask if use_mask else None)
    x = _ln(x, sd, "text_model.final_layer_norm", t.eps)
    if t.pool == "last":
        pooled = x[:, -1]
    elif t.pool == "argmax":
        pooled = x[torch.arange(B), ids.argmax(-1)]
    else:
        pooled = x[torch.arange(B), (ids == t.eos_id).int().argmax(-1)]
    if spec.family == "siglip":
        return F.linear(pooled, sd["text_model.head.weight"], sd["text_model.head.bias"])
    return F.linear(pooled, sd["text_projection.weight"])


def l2normalize_bf16(out: torch.Tensor, dtype=torch.bfloat16) -> torch.Tensor:
    """`out / out.norm(dim=-1, keepdim=True)` then `.to(DTYPE)` (main.py:414-415)."""
    return (out / out.norm(dim=-1, keepdim=True)).to(dtype)


def pad_ids(rows: Sequence[Sequence[int]], pad_id: int):
    L = max(len(r) for r in rows)
    ids = torch.full((len(rows), L), pad_id, dtype=torch.int64)
    mask = torch.zeros((len(rows), L), dtype=torch.int64)
    for i, r in enumerate(rows):
        ids[i, : len(r)] = torch.tensor(list(r))
        mask[i, : len(r)] = 1
    return ids, mask


@torch.no_grad()
def encode_data(spec, sd, images_u8: Sequence[np.ndarray], captions: Sequence[Sequence[int]], bs: int,
                out_dtype=torch.bfloat16):
    """main.py:386-438 with the oracle processor (PIL-exact numpy preprocessing)."""
    ip = spec.image_proc
    imgs = []
    for i in range(0, len(images_u8), bs):
        pv = np.stack([pil_bicubic.normalize(pil_bicubic.preprocess_u8(a, ip.size, ip.mode), ip.mean, ip.std)
                       for a in images_u8[i:i + bs]])
        out = vision_forward(spec, sd, torch.from_numpy(pv))
        imgs.append(l2normalize_bf16(out, out_dtype))
    txts = []
    for i in range(0, len(captions), bs):
        ids, mask = pad_ids(captions[i:i + bs], spec.text.pad_id)
        out = text_forward(spec, sd, ids, mask)
        txts.append(l2normalize_bf16(out, out_dtype))
    cat = lambda xs: torch.cat(xs) if xs else torch.empty(0)
    return cat(imgs), cat(txts)
