"""PyTorch-CPU restatement of the ColPali encoder (oracle, test infrastructure only).

ColPali-v1.3 (colpali_engine ColPali over PaliGemma-3B) is what the colpali
branch of encode_data (main.py:402-405,422-425) calls as `model(**inputs)`.
colpali_engine is not installed (requirements.txt:9 pins >=0.2.0); the
in-container port transformers 5.15 ColPaliForRetrieval is followed instead:
  * SigLIP vision tower, no head, post_layernorm       TF:models/siglip/modeling_siglip.py:553-619
  * multi_modal_projector Linear(1152 -> 2048)          TF:models/paligemma/modeling_paligemma.py:90-98,141-149
  * masked_scatter of image features, positions + 1     TF:models/paligemma/modeling_paligemma.py:223-246
  * GemmaTextScaledWordEmbedding (* bf16(sqrt d))        TF:models/gemma/modeling_gemma.py:50-61
  * GemmaRMSNorm (1 + w), fp32 statistics               TF:models/gemma/modeling_gemma.py:64-78
  * RoPE (cos/sin cast to the activation dtype)         TF:models/gemma/modeling_gemma.py:100-187
  * MQA attention, bidirectional + key padding          TF:models/gemma/modeling_gemma.py:202-292,
                                                        TF:models/paligemma/configuration_paligemma.py:92-95
  * GeGLU MLP                                           TF:models/gemma/modeling_gemma.py:84-97
  * final norm, embedding_proj_layer, L2, x mask        TF:models/colpali/modeling_colpali.py:132-140
Pinned against tests/golden/tiny-colpali.npz (the reference's encode_data run
over transformers' ColPaliForRetrieval, tests/golden/make_goldens.py).
"""
from __future__ import annotations

from typing import Dict, Optional

import torch
import torch.nn.functional as F

from . import encoders as venc


def _rms(x, w, eps):
    xf = x.float()
    y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    return (y * (1.0 + w.float())).to(x.dtype)


def _rope(x, pos, theta):
    """x [B, H, L, hd]; pos [L] (float)."""
    hd = x.shape[-1]
    inv = 1.0 / (theta ** (torch.arange(0, hd, 2, dtype=torch.float) / hd))
    f = pos[:, None].float() * inv[None, :]
    emb = torch.cat([f, f], -1)
    cos, sin = emb.cos().to(x.dtype), emb.sin().to(x.dtype)
    x1, x2 = x[..., : hd // 2], x[..., hd // 2:]
    rot = torch.cat([-x2, x1], -1)
    return x * cos + rot * sin


def _gemma_layer(x, p, tc, pos, mask):
    B, L, d = x.shape
    H, hd = tc.heads, tc.head_dim
    h = _rms(x, p["input_layernorm.weight"], tc.eps)
    q = F.linear(h, p["self_attn.q_proj.weight"]).view(B, L, H, hd).transpose(1, 2)
    k = F.linear(h, p["self_attn.k_proj.weight"]).view(B, L, 1, hd).transpose(1, 2)
    v = F.linear(h, p["self_attn.v_proj.weight"]).view(B, L, 1, hd).transpose(1, 2)
    q, k = _rope(q, pos, tc.theta), _rope(k, pos, tc.theta)
    k, v = k.expand(B, H, L, hd), v.expand(B, H, L, hd)
    w = torch.matmul(q, k.transpose(-1, -2)) * hd ** -0.5
    if mask is not None:
        w = w + mask
    w = torch.softmax(w, dim=-1, dtype=torch.float32).to(q.dtype)
    o = torch.matmul(w, v).transpose(1, 2).reshape(B, L, H * hd)
    x = x + F.linear(o, p["self_attn.o_proj.weight"])
    h = _rms(x, p["post_attention_layernorm.weight"], tc.eps)
    g = F.gelu(F.linear(h, p["mlp.gate_proj.weight"]), approximate="tanh")
    u = F.linear(h, p["mlp.up_proj.weight"])
    return x + F.linear(g * u, p["mlp.down_proj.weight"])


def vision_tokens(spec, sd: Dict[str, torch.Tensor], pixel_values: torch.Tensor) -> torch.Tensor:
    """SiglipVisionTransformer without head -> post-LN hidden [B, P, d]."""
    v = spec.vision
    pre = "vlm.vision_tower."
    dt = sd[pre + "post_layernorm.weight"].dtype
    x = F.conv2d(pixel_values.to(dt), sd[pre + "embeddings.patch_embedding.weight"],
                 sd[pre + "embeddings.patch_embedding.bias"], stride=v.patch)
    x = x.flatten(2).transpose(1, 2) + sd[pre + "embeddings.position_embedding.weight"]
    for i in range(v.layers):
        x = venc._layer(x, venc._sub(sd, f"{pre}encoder.layers.{i}."), v, None)
    return F.layer_norm(x, (x.shape[-1],), sd[pre + "post_layernorm.weight"], sd[pre + "post_layernorm.bias"], v.eps)


@torch.no_grad()
def forward(spec, sd: Dict[str, torch.Tensor], input_ids: torch.Tensor, attention_mask: Optional[torch.Tensor] = None,
            pixel_values: Optional[torch.Tensor] = None) -> torch.Tensor:
    """ColPaliForRetrieval.forward(...).embeddings: [B, L, 128] in the weights' dtype."""
    tc = spec.text
    B, L = input_ids.shape
    emb_w = sd["vlm.language_model.embed_tokens.weight"]
    dt = emb_w.dtype
    ids = input_ids.clone()
    is_img = ids == spec.image_token_id
    ids[ids >= emb_w.shape[0]] = 0
    x = emb_w[ids] * torch.tensor(tc.hidden ** 0.5, dtype=torch.float32).to(dt)
    if pixel_values is not None:
        feats = vision_tokens(spec, sd, pixel_values)
        feats = F.linear(feats, sd["vlm.multi_modal_projector.linear.weight"],
                         sd["vlm.multi_modal_projector.linear.bias"]).to(dt)
        x = x.masked_scatter(is_img[..., None], feats.reshape(-1, feats.shape[-1]))
    pos = torch.arange(L, dtype=torch.float) + 1  # PaliGemma positions are 1-indexed
    mask = None
    if attention_mask is not None and not bool(attention_mask.all()):
        mask = torch.zeros(B, 1, L, L, dtype=dt)
        mask = mask.masked_fill(attention_mask[:, None, None, :] == 0, torch.finfo(dt).min)
    for i in range(tc.layers):
        x = _gemma_layer(x, venc._sub(sd, f"vlm.language_model.layers.{i}."), tc, pos, mask)
    x = _rms(x, sd["vlm.language_model.norm.weight"], tc.eps)
    e = F.linear(x, sd["embedding_proj_layer.weight"], sd["embedding_proj_layer.bias"])
    e = e / e.norm(dim=-1, keepdim=True)
    if attention_mask is not None:
        e = e * attention_mask[..., None]
    return e


@torch.no_grad()
def encode_query_batch(spec, sd: Dict[str, torch.Tensor], captions) -> list:
    """One reference batch of ColPali queries, as encode_data's colpali branch runs it
    (main.py:420-425): processor.process_queries(batch) left-pads the batch to its longest
    query (TF:models/gemma/tokenization_gemma.py:55, padding_side left), model(**inputs)
    returns [B, L_b, 128] with the padded rows zeroed; each item's valid rows are its last
    len rows. Returns per item the valid [len, 128] rows."""
    rows = [list(spec.query_tokens(c)) for c in captions]
    L = max(len(r) for r in rows)
    ids = torch.full((len(rows), L), spec.pad_id, dtype=torch.int64)
    mask = torch.zeros((len(rows), L), dtype=torch.int64)
    for i, r in enumerate(rows):
        ids[i, L - len(r):] = torch.tensor(r)
        mask[i, L - len(r):] = 1
    e = forward(spec, sd, ids, mask)
    return [e[i, L - len(r):] for i, r in enumerate(rows)]


@torch.no_grad()
def encode_image(spec, sd: Dict[str, torch.Tensor], image_u8) -> torch.Tensor:
    """One image through processor.process_images + model (main.py:402-405): the PIL-exact
    resize / normalise (oracle/pil_bicubic.py), then [L_img, 128]."""
    from . import pil_bicubic
    ip = spec.image_proc
    pv = torch.from_numpy(pil_bicubic.normalize(pil_bicubic.preprocess_u8(image_u8, ip.size, ip.mode),
                                                ip.mean, ip.std))[None]
    return forward(spec, sd, torch.tensor([spec.image_tokens]), None, pv)[0]


def flops_per_token(spec, L: int) -> float:
    """Algorithmic FLOPs of one decoder token (GEMMs + attention over L keys)."""
    t = spec.text
    d, I, H, hd = t.hidden, t.intermediate, t.heads, t.head_dim
    f = t.layers * (2.0 * d * (H * hd + 2 * hd) + 2.0 * H * hd * d + 2.0 * 3 * d * I + 4.0 * L * H * hd)
    return f + 2.0 * d * spec.dim


def vision_flops(spec) -> float:
    v = spec.vision
    P, d, I = v.num_patches, v.hidden, v.intermediate
    f = 2.0 * P * 3 * v.patch ** 2 * d + v.layers * (2.0 * P * d * (4 * d + 2 * I) + 4.0 * P * P * d)
    return f + 2.0 * P * d * spec.text.hidden
