"""Device-resident weight packs for the encoder towers.

Weights live in HBM in the layout the kernels consume, prepared once at load:
  * q/k/v projections concatenated into one [3d, d] matrix (one GEMM, one
    pass over the activations instead of three);
  * the MLP intermediate width padded to a multiple of 128 with zero rows
    (fc1) / zero columns (fc2) so every GEMM tile is full (gelu(0) = 0);
  * the patch Conv2d weight flattened to [d, 3*p*p] (c, ky, kx order) and
    zero-padded to K % 64 == 0;
  * the SigLIP MAP-head probe query pre-projected (it is input-independent).
Sources: seeded random init (offline default) or an HF state dict /
safetensors file with the transformers parameter names
(TF:models/siglip/modeling_siglip.py, TF:models/clip/modeling_clip.py).
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, List, Optional

import torch

from . import ops
from .config import ModelSpec, TowerConfig

BF16 = torch.bfloat16


@dataclass
class LayerW:
    ln1_g: torch.Tensor
    ln1_b: torch.Tensor
    qkv_w: torch.Tensor   # [3d, d]
    qkv_b: torch.Tensor   # [3d]
    o_w: torch.Tensor     # [d, d]
    o_b: torch.Tensor
    ln2_g: torch.Tensor
    ln2_b: torch.Tensor
    fc1_w: torch.Tensor   # [Ipad, d]
    fc1_b: torch.Tensor   # [Ipad]
    fc2_w: torch.Tensor   # [d, Ipad]
    fc2_b: torch.Tensor
    mx: Optional[object] = None  # mme.mx.LayerMX: fp8 copies of qkv/fc1/fc2 (opt-in precision mode)
    fold: Optional[tuple] = None  # (ops.LNFolded qkv, ops.LNFolded fc1): LayerNorms folded into the weights
    q_prescaled: bool = False  # fold[0]'s Q rows carry the attention's scale * log2(e) (mme_attention_qs)


@dataclass
class MapHeadW:  # SiglipMultiheadAttentionPoolingHead
    q: torch.Tensor       # [d]  = probe @ Wq^T + bq
    kv_w: torch.Tensor    # [2d, d]
    kv_b: torch.Tensor    # [2d]
    out_w: torch.Tensor
    out_b: torch.Tensor
    ln_g: torch.Tensor
    ln_b: torch.Tensor
    fc1_w: torch.Tensor
    fc1_b: torch.Tensor
    fc2_w: torch.Tensor
    fc2_b: torch.Tensor
    # the probe query absorbed into the key projection (mme_map_pool): rows 0..H-1 = bf16(U_h),
    # rows H..2H-1 = bf16(U_h - bf16(U_h)), U_h = W_k,h^T q_h / sqrt(hd) (fp32 at load time)
    u: Optional[torch.Tensor] = None     # [2H, d]
    v_w: Optional[torch.Tensor] = None   # [d, d] = W_v (view of kv_w)
    v_b: Optional[torch.Tensor] = None   # [d]


@dataclass
class VisionW:
    patch_w: torch.Tensor            # [d, kpad]
    patch_b: Optional[torch.Tensor]  # SigLIP conv bias
    pos: torch.Tensor                # [T, d]
    cls: Optional[torch.Tensor]      # CLIP class embedding [d]
    pre_ln_g: Optional[torch.Tensor]
    pre_ln_b: Optional[torch.Tensor]
    layers: List[LayerW]
    post_ln_g: torch.Tensor
    post_ln_b: torch.Tensor
    head: Optional[MapHeadW]         # SigLIP
    proj_w: Optional[torch.Tensor]   # CLIP visual_projection [proj, d]


@dataclass
class TextW:
    tok: torch.Tensor                # [V, d]
    pos: torch.Tensor                # [max_pos, d]
    layers: List[LayerW]
    final_ln_g: torch.Tensor
    final_ln_b: torch.Tensor
    head_w: torch.Tensor             # SigLIP head / CLIP text_projection [proj, d]
    head_b: Optional[torch.Tensor]


@dataclass
class ModelW:
    vision: VisionW
    text: TextW


# ---------------------------------------------------------------- packing helpers
def _pad_rows(w: torch.Tensor, rows: int) -> torch.Tensor:
    if w.shape[0] == rows:
        return w.contiguous()
    out = torch.zeros((rows,) + tuple(w.shape[1:]), dtype=w.dtype, device=w.device)
    out[: w.shape[0]] = w
    return out


def _pad_cols(w: torch.Tensor, cols: int) -> torch.Tensor:
    if w.shape[1] == cols:
        return w.contiguous()
    out = torch.zeros(w.shape[0], cols, dtype=w.dtype, device=w.device)
    out[:, : w.shape[1]] = w
    return out


def pack_layer(cfg: TowerConfig, g: Dict[str, torch.Tensor], device) -> LayerW:
    """g: HF per-layer tensors keyed 'layer_norm1.weight', 'self_attn.q_proj.weight', ..."""
    t = {k: v.to(device=device, dtype=BF16) for k, v in g.items()}
    Ip = cfg.inter_pad
    return LayerW(
        ln1_g=t["layer_norm1.weight"], ln1_b=t["layer_norm1.bias"],
        qkv_w=torch.cat([t["self_attn.q_proj.weight"], t["self_attn.k_proj.weight"], t["self_attn.v_proj.weight"]],
                        0).contiguous(),
        qkv_b=torch.cat([t["self_attn.q_proj.bias"], t["self_attn.k_proj.bias"], t["self_attn.v_proj.bias"]],
                        0).contiguous(),
        o_w=t["self_attn.out_proj.weight"].contiguous(), o_b=t["self_attn.out_proj.bias"],
        ln2_g=t["layer_norm2.weight"], ln2_b=t["layer_norm2.bias"],
        fc1_w=_pad_rows(t["mlp.fc1.weight"], Ip), fc1_b=_pad_rows(t["mlp.fc1.bias"], Ip),
        fc2_w=_pad_cols(t["mlp.fc2.weight"], Ip), fc2_b=t["mlp.fc2.bias"],
    )


def _sub(sd: Dict[str, torch.Tensor], prefix: str) -> Dict[str, torch.Tensor]:
    n = len(prefix)
    return {k[n:]: v for k, v in sd.items() if k.startswith(prefix)}


def from_hf_state_dict(spec: ModelSpec, sd: Dict[str, torch.Tensor], device="cuda") -> ModelW:
    """Pack an HF SiglipModel / CLIPModel state dict (transformers parameter names)."""
    v, tcfg = spec.vision, spec.text
    dev = torch.device(device)

    def b(name):
        return sd[name].to(device=dev, dtype=BF16)

    layers_v = [pack_layer(v, _sub(sd, f"vision_model.encoder.layers.{i}."), dev) for i in range(v.layers)]
    layers_t = [pack_layer(tcfg, _sub(sd, f"text_model.encoder.layers.{i}."), dev) for i in range(tcfg.layers)]
    pw = b("vision_model.embeddings.patch_embedding.weight").reshape(v.hidden, -1)
    patch_w = _pad_cols(pw, v.kpad)
    if spec.family == "siglip":
        d = v.hidden
        in_w, in_b = b("vision_model.head.attention.in_proj_weight"), b("vision_model.head.attention.in_proj_bias")
        probe = b("vision_model.head.probe").reshape(1, d)
        q = ops.gemm(probe.contiguous(), in_w[:d].contiguous(), in_b[:d].contiguous()).reshape(d)
        H, hd = v.heads, v.head_dim
        wk = in_w[d:2 * d].float().reshape(H, hd, d)
        u = torch.einsum("hj,hjc->hc", q.float().reshape(H, hd), wk) * hd ** -0.5  # [H, d] fp32 (load time)
        u_hi = u.to(BF16)
        u2 = torch.cat([u_hi, (u - u_hi.float()).to(BF16)]).contiguous()
        kv_w, kv_b = in_w[d:].contiguous(), in_b[d:].contiguous()
        head = MapHeadW(
            q=q, kv_w=kv_w, kv_b=kv_b, u=u2, v_w=kv_w[d:], v_b=kv_b[d:],
            out_w=b("vision_model.head.attention.out_proj.weight"), out_b=b("vision_model.head.attention.out_proj.bias"),
            ln_g=b("vision_model.head.layernorm.weight"), ln_b=b("vision_model.head.layernorm.bias"),
            fc1_w=_pad_rows(b("vision_model.head.mlp.fc1.weight"), v.inter_pad),
            fc1_b=_pad_rows(b("vision_model.head.mlp.fc1.bias"), v.inter_pad),
            fc2_w=_pad_cols(b("vision_model.head.mlp.fc2.weight"), v.inter_pad),
            fc2_b=b("vision_model.head.mlp.fc2.bias"))
        vision = VisionW(patch_w=patch_w, patch_b=b("vision_model.embeddings.patch_embedding.bias"),
                         pos=b("vision_model.embeddings.position_embedding.weight"), cls=None, pre_ln_g=None,
                         pre_ln_b=None, layers=layers_v, post_ln_g=b("vision_model.post_layernorm.weight"),
                         post_ln_b=b("vision_model.post_layernorm.bias"), head=head, proj_w=None)
        text = TextW(tok=b("text_model.embeddings.token_embedding.weight"),
                     pos=b("text_model.embeddings.position_embedding.weight"), layers=layers_t,
                     final_ln_g=b("text_model.final_layer_norm.weight"),
                     final_ln_b=b("text_model.final_layer_norm.bias"),
                     head_w=b("text_model.head.weight"), head_b=b("text_model.head.bias"))
    else:
        vision = VisionW(patch_w=patch_w, patch_b=None, pos=b("vision_model.embeddings.position_embedding.weight"),
                         cls=b("vision_model.embeddings.class_embedding"),
                         pre_ln_g=b("vision_model.pre_layrnorm.weight"), pre_ln_b=b("vision_model.pre_layrnorm.bias"),
                         layers=layers_v, post_ln_g=b("vision_model.post_layernorm.weight"),
                         post_ln_b=b("vision_model.post_layernorm.bias"), head=None,
                         proj_w=b("visual_projection.weight"))
        text = TextW(tok=b("text_model.embeddings.token_embedding.weight"),
                     pos=b("text_model.embeddings.position_embedding.weight"), layers=layers_t,
                     final_ln_g=b("text_model.final_layer_norm.weight"),
                     final_ln_b=b("text_model.final_layer_norm.bias"),
                     head_w=b("text_projection.weight"), head_b=None)
    return ModelW(vision=vision, text=text)


def random_state_dict(spec: ModelSpec, seed: int = 0, device="cuda") -> Dict[str, torch.Tensor]:
    """Seeded random weights with HF tensor names/shapes (xavier-style Linear init,
    unit LayerNorm, N(0, 1/sqrt(d)) embeddings) — the offline stand-in for
    from_pretrained(hub_id) (main.py:808-820)."""
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

    def emb(name, n, d):
        sd[name] = (torch.randn(n, d, generator=g, device=dev) / math.sqrt(d)).to(BF16)

    def layers(prefix, cfg):
        d, I = cfg.hidden, cfg.intermediate
        for i in range(cfg.layers):
            p = f"{prefix}.encoder.layers.{i}."
            ln(p + "layer_norm1", d)
            ln(p + "layer_norm2", d)
            for n in ("q_proj", "k_proj", "v_proj", "out_proj"):
                lin(p + "self_attn." + n, d, d)
            lin(p + "mlp.fc1", I, d)
            lin(p + "mlp.fc2", d, I)

    v, t = spec.vision, spec.text
    d = v.hidden
    sd["vision_model.embeddings.patch_embedding.weight"] = (
        torch.randn(d, 3, v.patch, v.patch, generator=g, device=dev) / math.sqrt(3 * v.patch * v.patch)).to(BF16)
    T = v.num_patches + (1 if spec.family == "clip" else 0)
    emb("vision_model.embeddings.position_embedding.weight", T, d)
    layers("vision_model", v)
    ln("vision_model.post_layernorm", d)
    emb("text_model.embeddings.token_embedding.weight", t.vocab, t.hidden)
    emb("text_model.embeddings.position_embedding.weight", t.max_pos, t.hidden)
    layers("text_model", t)
    ln("text_model.final_layer_norm", t.hidden)
    if spec.family == "siglip":
        sd["vision_model.embeddings.patch_embedding.bias"] = torch.zeros(d, dtype=BF16, device=dev)
        sd["vision_model.head.probe"] = (torch.randn(1, 1, d, generator=g, device=dev) / math.sqrt(d)).to(BF16)
        a = math.sqrt(6.0 / (4 * d))
        sd["vision_model.head.attention.in_proj_weight"] = (
            (torch.rand(3 * d, d, generator=g, device=dev) * 2 - 1) * a).to(BF16)
        sd["vision_model.head.attention.in_proj_bias"] = torch.zeros(3 * d, dtype=BF16, device=dev)
        lin("vision_model.head.attention.out_proj", d, d)
        ln("vision_model.head.layernorm", d)
        lin("vision_model.head.mlp.fc1", v.intermediate, d)
        lin("vision_model.head.mlp.fc2", d, v.intermediate)
        lin("text_model.head", spec.proj_dim, t.hidden)
    else:
        sd["vision_model.embeddings.class_embedding"] = (torch.randn(d, generator=g, device=dev) /
                                                         math.sqrt(d)).to(BF16)
        ln("vision_model.pre_layrnorm", d)
        lin("visual_projection", spec.proj_dim, d, bias=False)
        lin("text_projection", spec.proj_dim, t.hidden, bias=False)
    return sd


def hf_param_shapes(spec: ModelSpec) -> Dict[str, tuple]:
    """Name -> shape of every learned tensor of the HF SiglipModel / CLIPModel at
    this architecture (the state dict from_hf_state_dict consumes)."""
    sh: Dict[str, tuple] = {}
    v, t = spec.vision, spec.text

    def layers(prefix, cfg):
        d, I = cfg.hidden, cfg.intermediate
        for i in range(cfg.layers):
            p = f"{prefix}.encoder.layers.{i}."
            for n in ("layer_norm1", "layer_norm2"):
                sh[p + n + ".weight"] = (d,)
                sh[p + n + ".bias"] = (d,)
            for n in ("q_proj", "k_proj", "v_proj", "out_proj"):
                sh[p + "self_attn." + n + ".weight"] = (d, d)
                sh[p + "self_attn." + n + ".bias"] = (d,)
            sh[p + "mlp.fc1.weight"], sh[p + "mlp.fc1.bias"] = (I, d), (I,)
            sh[p + "mlp.fc2.weight"], sh[p + "mlp.fc2.bias"] = (d, I), (d,)

    d = v.hidden
    sh["vision_model.embeddings.patch_embedding.weight"] = (d, 3, v.patch, v.patch)
    T = v.num_patches + (1 if spec.family == "clip" else 0)
    sh["vision_model.embeddings.position_embedding.weight"] = (T, d)
    layers("vision_model", v)
    sh["vision_model.post_layernorm.weight"] = sh["vision_model.post_layernorm.bias"] = (d,)
    sh["text_model.embeddings.token_embedding.weight"] = (t.vocab, t.hidden)
    sh["text_model.embeddings.position_embedding.weight"] = (t.max_pos, t.hidden)
    layers("text_model", t)
    sh["text_model.final_layer_norm.weight"] = sh["text_model.final_layer_norm.bias"] = (t.hidden,)
    if spec.family == "siglip":
        sh["vision_model.embeddings.patch_embedding.bias"] = (d,)
        sh["vision_model.head.probe"] = (1, 1, d)
        sh["vision_model.head.attention.in_proj_weight"] = (3 * d, d)
        sh["vision_model.head.attention.in_proj_bias"] = (3 * d,)
        sh["vision_model.head.attention.out_proj.weight"] = (d, d)
        sh["vision_model.head.attention.out_proj.bias"] = (d,)
        sh["vision_model.head.layernorm.weight"] = sh["vision_model.head.layernorm.bias"] = (d,)
        sh["vision_model.head.mlp.fc1.weight"], sh["vision_model.head.mlp.fc1.bias"] = (v.intermediate, d), (v.intermediate,)
        sh["vision_model.head.mlp.fc2.weight"], sh["vision_model.head.mlp.fc2.bias"] = (d, v.intermediate), (d,)
        sh["text_model.head.weight"], sh["text_model.head.bias"] = (spec.proj_dim, t.hidden), (spec.proj_dim,)
    else:
        sh["vision_model.embeddings.class_embedding"] = (d,)
        sh["vision_model.pre_layrnorm.weight"] = sh["vision_model.pre_layrnorm.bias"] = (d,)
        sh["visual_projection.weight"] = (spec.proj_dim, d)
        sh["text_projection.weight"] = (spec.proj_dim, t.hidden)
    return sh


def load_safetensors(path: str) -> Dict[str, torch.Tensor]:
    from safetensors.torch import load_file  # executes nothing from the file
    return load_file(path)


def param_count(sd: Dict[str, torch.Tensor]) -> int:
    return sum(v.numel() for v in sd.values())
