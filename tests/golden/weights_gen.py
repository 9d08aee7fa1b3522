"""Deterministic weights for the tiny parity models (test data generator).

numpy PCG64 (default_rng) is bit-stable across platforms, so the GPU box
regenerates exactly the weights tests/golden/make_goldens.py fed to the
reference here — no weight files need to be committed. Every value is rounded
to bf16 (RNE) and stored as fp32, so the fp32 and bf16 reference runs use the
same numbers. Names/shapes follow transformers' SiglipModel / CLIPModel.
"""
from __future__ import annotations

import math
from typing import Dict

import numpy as np


def bf16_round(a: np.ndarray) -> np.ndarray:
    """Round fp32 to the nearest bf16 (ties to even), returned as fp32."""
    u = np.ascontiguousarray(a, dtype=np.float32).view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    return r.astype(np.uint32).view(np.float32)


def np_state_dict(spec, seed: int = 0) -> Dict[str, np.ndarray]:
    rng = np.random.default_rng(seed)
    sd: Dict[str, np.ndarray] = {}

    def put(name, arr):
        sd[name] = bf16_round(np.asarray(arr, dtype=np.float32))

    def lin(name, out_f, in_f, bias=True):
        a = math.sqrt(6.0 / (in_f + out_f))
        put(name + ".weight", rng.uniform(-a, a, (out_f, in_f)))
        if bias:
            put(name + ".bias", rng.normal(0, 0.02, out_f))

    def ln(name, d):
        put(name + ".weight", 1.0 + rng.normal(0, 0.05, d))
        put(name + ".bias", rng.normal(0, 0.02, d))

    def layers(prefix, cfg):
        d, I = cfg.hidden, cfg.intermediate
        for i in range(cfg.layers):
            p = f"{prefix}.encoder.layers.{i}."
            ln(p + "layer_norm1", d)
            for n in ("q_proj", "k_proj", "v_proj", "out_proj"):
                lin(p + "self_attn." + n, d, d)
            ln(p + "layer_norm2", d)
            lin(p + "mlp.fc1", I, d)
            lin(p + "mlp.fc2", d, I)

    v, t = spec.vision, spec.text
    d = v.hidden
    put("vision_model.embeddings.patch_embedding.weight",
        rng.normal(0, 1 / math.sqrt(3 * v.patch * v.patch), (d, 3, v.patch, v.patch)))
    T = v.num_patches + (1 if spec.family == "clip" else 0)
    put("vision_model.embeddings.position_embedding.weight", rng.normal(0, 1 / math.sqrt(d), (T, d)))
    layers("vision_model", v)
    ln("vision_model.post_layernorm", d)
    put("text_model.embeddings.token_embedding.weight", rng.normal(0, 1 / math.sqrt(t.hidden), (t.vocab, t.hidden)))
    put("text_model.embeddings.position_embedding.weight",
        rng.normal(0, 1 / math.sqrt(t.hidden), (t.max_pos, t.hidden)))
    layers("text_model", t)
    ln("text_model.final_layer_norm", t.hidden)
    if spec.family == "siglip":
        put("vision_model.embeddings.patch_embedding.bias", rng.normal(0, 0.02, d))
        put("vision_model.head.probe", rng.normal(0, 1 / math.sqrt(d), (1, 1, d)))
        a = math.sqrt(6.0 / (4 * d))
        put("vision_model.head.attention.in_proj_weight", rng.uniform(-a, a, (3 * d, d)))
        put("vision_model.head.attention.in_proj_bias", rng.normal(0, 0.02, 3 * d))
        lin("vision_model.head.attention.out_proj", d, d)
        ln("vision_model.head.layernorm", d)
        lin("vision_model.head.mlp.fc1", v.intermediate, d)
        lin("vision_model.head.mlp.fc2", d, v.intermediate)
        lin("text_model.head", spec.proj_dim, t.hidden)
    else:
        put("vision_model.embeddings.class_embedding", rng.normal(0, 1 / math.sqrt(d), d))
        ln("vision_model.pre_layrnorm", d)
        lin("visual_projection", spec.proj_dim, d, bias=False)
        lin("text_projection", spec.proj_dim, t.hidden, bias=False)
    return sd


def np_state_dict_colpali(spec, seed: int = 0) -> Dict[str, np.ndarray]:
    """transformers ColPaliForRetrieval names/shapes (vlm.vision_tower.*, vlm.multi_modal_projector.*,
    vlm.language_model.*, embedding_proj_layer.*) for a ColPaliSpec."""
    rng = np.random.default_rng(seed)
    sd: Dict[str, np.ndarray] = {}

    def put(name, arr):
        sd[name] = bf16_round(np.asarray(arr, dtype=np.float32))

    def lin(name, out_f, in_f, bias=True):
        a = math.sqrt(6.0 / (in_f + out_f))
        put(name + ".weight", rng.uniform(-a, a, (out_f, in_f)))
        if bias:
            put(name + ".bias", rng.normal(0, 0.02, out_f))

    def ln(name, d):
        put(name + ".weight", 1.0 + rng.normal(0, 0.05, d))
        put(name + ".bias", rng.normal(0, 0.02, d))

    v, t = spec.vision, spec.text
    d = v.hidden
    pre = "vlm.vision_tower."
    put(pre + "embeddings.patch_embedding.weight", rng.normal(0, 1 / math.sqrt(3 * v.patch * v.patch),
                                                              (d, 3, v.patch, v.patch)))
    put(pre + "embeddings.patch_embedding.bias", rng.normal(0, 0.02, d))
    put(pre + "embeddings.position_embedding.weight", rng.normal(0, 1 / math.sqrt(d), (v.num_patches, d)))
    for i in range(v.layers):
        p = f"{pre}encoder.layers.{i}."
        ln(p + "layer_norm1", d)
        for n in ("q_proj", "k_proj", "v_proj", "out_proj"):
            lin(p + "self_attn." + n, d, d)
        ln(p + "layer_norm2", d)
        lin(p + "mlp.fc1", v.intermediate, d)
        lin(p + "mlp.fc2", d, v.intermediate)
    ln(pre + "post_layernorm", d)
    lin("vlm.multi_modal_projector.linear", t.hidden, d)
    D, H, hd = t.hidden, t.heads, t.head_dim
    lm = "vlm.language_model."
    put(lm + "embed_tokens.weight", rng.normal(0, 1 / D, (t.vocab, D)))
    for i in range(t.layers):
        p = f"{lm}layers.{i}."
        put(p + "input_layernorm.weight", rng.normal(0, 0.1, D))
        lin(p + "self_attn.q_proj", H * hd, D, bias=False)
        lin(p + "self_attn.k_proj", hd, D, bias=False)
        lin(p + "self_attn.v_proj", hd, D, bias=False)
        lin(p + "self_attn.o_proj", D, H * hd, bias=False)
        put(p + "post_attention_layernorm.weight", rng.normal(0, 0.1, D))
        lin(p + "mlp.gate_proj", t.intermediate, D, bias=False)
        lin(p + "mlp.up_proj", t.intermediate, D, bias=False)
        lin(p + "mlp.down_proj", D, t.intermediate, bias=False)
    put(lm + "norm.weight", rng.normal(0, 0.1, D))
    lin("embedding_proj_layer", spec.dim, D)
    return sd


def bf16_bits_to_f32(b: np.ndarray) -> np.ndarray:
    return (np.asarray(b, np.uint16).astype(np.uint32) << 16).view(np.float32)


def factor_product(a_bits: np.ndarray, b_bits: np.ndarray) -> np.ndarray:
    """W = bf16(A @ B) for bf16 factors A [D, r], B [r, d] (tests/golden/e2e_fitted.npz): float64
    outer products added in a fixed order with numpy's elementwise ufuncs (each op correctly
    rounded, no BLAS), so every box rebuilds the same bits; the fixture stores their SHA-256."""
    a = bf16_bits_to_f32(a_bits).astype(np.float64)
    b = bf16_bits_to_f32(b_bits).astype(np.float64)
    w = np.zeros((a.shape[0], b.shape[1]), np.float64)
    for k in range(a.shape[1]):
        w += np.multiply.outer(a[:, k], b[k])
    return bf16_round(w.astype(np.float32))


def fitted_overrides(spec, fx, key: str) -> Dict[str, np.ndarray]:
    """The fitted projection heads of one model of e2e_fitted.npz, as state-dict entries (fp32 arrays of
    bf16 values). CLIP: visual_projection / text_projection. SigLIP: the MAP head's mlp.fc2 (weight and
    bias: the last factor column) and text_model.head (weight and bias)."""
    import hashlib
    wi = factor_product(fx[f"{key}_img_A"], fx[f"{key}_img_B"])
    wt = factor_product(fx[f"{key}_txt_A"], fx[f"{key}_txt_B"])
    for w, tag in ((wi, "img"), (wt, "txt")):
        sha = hashlib.sha256(w.view(np.uint32).tobytes()).hexdigest()[:32]
        assert sha == str(fx[f"{key}_{tag}_sha"]), f"{key} {tag} head rebuilt differently ({sha})"
    if spec.family == "clip":
        return {"visual_projection.weight": wi, "text_projection.weight": wt}
    return {"vision_model.head.mlp.fc2.weight": np.ascontiguousarray(wi[:, :-1]),
            "vision_model.head.mlp.fc2.bias": np.ascontiguousarray(wi[:, -1]),
            "text_model.head.weight": np.ascontiguousarray(wt[:, :-1]), "text_model.head.bias": np.ascontiguousarray(wt[:, -1])}


def torch_state_dict(spec, seed: int = 0, dtype=None):
    import torch
    dtype = dtype or torch.float32
    gen = np_state_dict_colpali if getattr(spec, "family", "") == "colpali" else np_state_dict
    return {k: torch.from_numpy(v.copy()).to(dtype) for k, v in gen(spec, seed).items()}
