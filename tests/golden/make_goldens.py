"""Generate the golden parity fixtures from the REFERENCE itself (run here only).

This script imports /root/reference/main.py (read-only, never copied) and
drives its own hot-path functions — encode_data (main.py:386-438),
compute_similarity_scores (main.py:440-475), compute_metrics_detailed
(main.py:305-383) — with in-container transformers models / image processors
(transformers 5.15.0, PIL 12.2.0) and deterministic inputs. Only the
resulting input/output arrays are committed (tests/golden/*.npz); the GPU box
never needs /root/reference.

Shims, none of which edits a reference file:
  1. main.DEVICE = 'cpu', main.DTYPE = bf16 (or fp32 for the fp32 oracle run);
  2. a model adapter whose get_*_features return .pooler_output (transformers
     4 semantics);
  3. compute_metrics_detailed is called with the un-transposed I2T matrix
     (the v28 orientation; main.py:622-623's .t() is the KeyError bug §0.1);
  4. identity sample (no bootstrap resampling, §0.5).

Usage: python tests/golden/make_goldens.py   (writes tests/golden/*.npz)
"""
from __future__ import annotations

import os
import sys
import tempfile

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, os.path.join(REPO, "multimodal-embedding_amd"))
sys.path.insert(0, HERE)

from weights_gen import torch_state_dict  # noqa: E402
from mme.config import TINY, OPENAI_CLIP_MEAN, OPENAI_CLIP_STD  # noqa: E402


def import_reference():
    cwd = os.getcwd()
    os.chdir(tempfile.mkdtemp(prefix="mme_ref_"))  # main.py writes benchmark_v29.log into the cwd
    sys.path.insert(0, REF)
    import main  # noqa: E402
    os.chdir(cwd)
    return main


def bf16_bits(t: torch.Tensor) -> np.ndarray:
    return t.to(torch.bfloat16).contiguous().view(torch.int16).numpy().view(np.uint16)


# ------------------------------------------------------------------ preprocess
def make_preprocess():
    from PIL import Image
    from transformers.models.siglip.image_processing_pil_siglip import SiglipImageProcessorPil
    from transformers.models.clip.image_processing_pil_clip import CLIPImageProcessorPil

    rng = np.random.default_rng(0)
    cases = [  # (name, H, W, processor kind, size)
        ("siglip384", 224, 224, "siglip", 384),
        ("clip336", 224, 224, "clip", 336),
        ("dfn378", 224, 224, "clip", 378),
        ("clip336_nonsq", 150, 200, "clip", 336),
        ("vith224_down", 300, 260, "clip", 224),
    ]
    out = {}
    for name, H, W, kind, S in cases:
        img = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
        pil = Image.fromarray(img)
        if kind == "siglip":
            proc = SiglipImageProcessorPil(size={"height": S, "width": S})
            mean, std = (0.5, 0.5, 0.5), (0.5, 0.5, 0.5)
        else:
            proc = CLIPImageProcessorPil(size={"shortest_edge": S}, crop_size={"height": S, "width": S})
            mean, std = OPENAI_CLIP_MEAN, OPENAI_CLIP_STD
        pv = proc(images=[pil], return_tensors="np")["pixel_values"][0].astype(np.float32)  # [3,S,S]
        # the resized + cropped u8 raster, recovered exactly: HF computes
        # float32(float64(u8)/255) then (x - mean)/std in float32; invert by search
        lut = np.empty((3, 256), np.float32)
        for c in range(3):
            r = (np.arange(256, dtype=np.float64) * (1 / 255)).astype(np.float32)
            lut[c] = (r - np.float32(mean[c])) / np.float32(std[c])
        u8 = np.empty((S, S, 3), np.uint8)
        for c in range(3):
            idx = np.searchsorted(lut[c], pv[c])
            idx = np.clip(idx, 0, 255)
            assert np.array_equal(lut[c][idx], pv[c]), f"{name}: pixel_values not on the u8 grid"
            u8[:, :, c] = idx
        out[f"{name}_in"] = img
        out[f"{name}_u8"] = u8
        out[f"{name}_meta"] = np.array([H, W, S, 0 if kind == "siglip" else 1], np.int64)
    np.savez_compressed(os.path.join(HERE, "preprocess.npz"), **out)
    print("preprocess.npz:", {k: v.shape for k, v in out.items()})


# ------------------------------------------------------------------ tiny encoders
class RefAdapter:
    """get_*_features -> .pooler_output (transformers-4 return type)."""

    def __init__(self, hf):
        self.hf = hf

    def get_image_features(self, **kw):
        return self.hf.get_image_features(**kw).pooler_output

    def get_text_features(self, **kw):
        return self.hf.get_text_features(**kw).pooler_output


class RefProcessor:
    """HF PIL image processor + HF-style padding of pre-tokenized id lists."""

    def __init__(self, image_proc, pad_id):
        self.ip, self.pad_id = image_proc, pad_id

    def __call__(self, images=None, text=None, return_tensors="pt", padding=True, truncation=True):
        from transformers import BatchFeature
        if images is not None:
            return self.ip(images=images, return_tensors="pt")
        L = max(len(t) for t in text)
        ids = torch.full((len(text), L), self.pad_id, dtype=torch.int64)
        mask = torch.zeros((len(text), L), dtype=torch.int64)
        for i, t in enumerate(text):
            ids[i, : len(t)] = torch.tensor(t)
            mask[i, : len(t)] = 1
        return BatchFeature({"input_ids": ids, "attention_mask": mask})


def hf_model(spec, dtype, overrides=None):
    from transformers import CLIPConfig, CLIPModel, SiglipConfig, SiglipModel
    v, t = spec.vision, spec.text
    vc = dict(hidden_size=v.hidden, intermediate_size=v.intermediate, num_hidden_layers=v.layers,
              num_attention_heads=v.heads, image_size=v.image_size, patch_size=v.patch, hidden_act=v.act,
              layer_norm_eps=v.eps)
    tc = dict(hidden_size=t.hidden, intermediate_size=t.intermediate, num_hidden_layers=t.layers,
              num_attention_heads=t.heads, vocab_size=t.vocab, max_position_embeddings=t.max_pos, hidden_act=t.act,
              layer_norm_eps=t.eps, eos_token_id=t.eos_id, pad_token_id=t.pad_id)
    if spec.family == "siglip":
        tc["projection_size"] = spec.proj_dim
        cfg = SiglipConfig(text_config=tc, vision_config=vc)
        m = SiglipModel(cfg)
    else:
        tc["bos_token_id"] = t.bos_id
        cfg = CLIPConfig(text_config=tc, vision_config=vc, projection_dim=spec.proj_dim)
        m = CLIPModel(cfg)
    sd = torch_state_dict(spec, seed=0)
    for k, v in (overrides or {}).items():
        assert k in sd and sd[k].shape == v.shape, k
        sd[k] = torch.from_numpy(np.ascontiguousarray(v, np.float32))
    missing, unexpected = m.load_state_dict(sd, strict=False)
    missing = [k for k in missing if not k.endswith(("position_ids", "logit_scale", "logit_bias"))]
    assert not missing and not unexpected, (missing, unexpected)
    return m.to(dtype).eval()


def make_encoders(main):
    from PIL import Image
    from transformers.models.siglip.image_processing_pil_siglip import SiglipImageProcessorPil
    from transformers.models.clip.image_processing_pil_clip import CLIPImageProcessorPil

    for name in ("tiny-siglip", "tiny-clip"):
        spec = TINY[name]
        S = spec.vision.image_size
        rng = np.random.default_rng(7)
        imgs = rng.integers(0, 256, (5, 112, 112, 3), dtype=np.uint8)
        pil = [Image.fromarray(a) for a in imgs]
        t = spec.text
        lens = [t.max_pos, 5, 9, t.max_pos - 3, 3, 7, 11]
        caps = []
        for L in lens:
            if t.bos_id is not None:
                body = rng.integers(1, min(t.bos_id, t.eos_id), L - 2).tolist()
                caps.append([t.bos_id] + body + [t.eos_id])
            else:
                body = rng.integers(2, t.vocab, L - 1).tolist()
                caps.append(body + [t.eos_id])
        if spec.family == "siglip":
            ip = SiglipImageProcessorPil(size={"height": S, "width": S})
        else:
            ip = CLIPImageProcessorPil(size={"shortest_edge": S}, crop_size={"height": S, "width": S})
        proc = RefProcessor(ip, t.pad_id)
        m_info = {"name": name, "type": spec.m_info["type"], "batch_size": spec.batch_size}
        out = {"images": imgs, "lens": np.array(lens, np.int64)}
        Lmax = max(lens)
        ids = np.full((len(caps), Lmax), t.pad_id, np.int64)
        for i, c in enumerate(caps):
            ids[i, : len(c)] = c
        out["ids"] = ids
        for tag, dtype in (("bf16", torch.bfloat16), ("f32", torch.float32)):
            hf = hf_model(spec, dtype)
            main.DEVICE, main.DTYPE = "cpu", dtype
            with torch.no_grad():
                img_e, txt_e = main.encode_data(RefAdapter(hf), proc, m_info, pil, caps)
            if tag == "bf16":
                out["img_bf16"], out["txt_bf16"] = bf16_bits(img_e), bf16_bits(txt_e)
            else:
                out["img_f32"], out["txt_f32"] = img_e.float().numpy(), txt_e.float().numpy()
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **out)
        print(f"{name}.npz:", {k: v.shape for k, v in out.items()})


def make_config0(main):
    """BASELINE configs[0]: OpenAI-CLIP-L (336 px, full architecture, deterministic random weights),
    64 images x 320 captions through the reference's own CPU path: main.encode_data at the default
    --batch-size 32 (main.py:73,131-136) for the images + all captions (main.py:551,557) and for the
    caption-0 T2I queries (main.py:554), then compute_similarity_scores + compute_metrics_detailed.
    Stores the embeddings (bf16 and fp32 runs) and each row's top-11 of the reference's scores."""
    from PIL import Image
    from transformers.models.clip.image_processing_pil_clip import CLIPImageProcessorPil
    from mme.config import get_spec
    from planted import config0_inputs
    spec = get_spec("OpenAI-CLIP-L")
    S = spec.vision.image_size
    imgs, cap_rows = config0_inputs(spec)
    n, caps = imgs.shape[0], len(cap_rows) // imgs.shape[0]
    pil = [Image.fromarray(a) for a in imgs]
    proc = RefProcessor(CLIPImageProcessorPil(size={"shortest_edge": S}, crop_size={"height": S, "width": S}),
                        spec.text.pad_id)
    m_info = {"name": "OpenAI-CLIP-L", "type": "dense", "batch_size": 32}
    out = {"params": np.array([n, caps, 21], np.int64)}
    torch.set_num_threads(os.cpu_count() or 8)
    for tag, dtype in (("bf16", torch.bfloat16), ("f32", torch.float32)):
        hf = RefAdapter(hf_model(spec, dtype))
        main.DEVICE, main.DTYPE = "cpu", dtype
        with torch.no_grad():
            img_e, all_e = main.encode_data(hf, proc, m_info, pil, cap_rows)
            _, t2i_e = main.encode_data(hf, proc, m_info, [], cap_rows[::caps])
        if tag == "bf16":
            out["img_bf16"], out["all_bf16"], out["t2i_bf16"] = bf16_bits(img_e), bf16_bits(all_e), bf16_bits(t2i_e)
            s_t2i = main.compute_similarity_scores(img_e, t2i_e, {"type": "dense"}, None)
            s_i2t = main.compute_similarity_scores(all_e, img_e, {"type": "dense"}, None)
            metrics = main.compute_metrics_detailed(s_t2i, s_i2t, s_t2i.t(), list(range(n)),
                                                    {i: list(range(caps * i, caps * i + caps)) for i in range(n)},
                                                    {i: i for i in range(n)}, [""] * n)
            for key, s in (("t2i", s_t2i), ("i2t", s_i2t), ("sym", s_t2i.t().contiguous())):
                v, ix = torch.topk(s, 11, dim=1)
                out[f"{key}_idx"], out[f"{key}_score"] = ix.numpy().astype(np.int32), v.numpy()
            keys = [k for k in metrics if not k.startswith("_")]
            out["metric_names"] = np.array(keys)
            out["metric_values"] = np.array([metrics[k] for k in keys], np.float64)
        else:
            out["img_f32"], out["all_f32"], out["t2i_f32"] = img_e.numpy(), all_e.numpy(), t2i_e.numpy()
        del hf
    np.savez_compressed(os.path.join(HERE, "config0_clip_l.npz"), **out)
    print("config0_clip_l.npz:", {k: v.shape for k, v in out.items()})


# ------------------------------------------------------------------ end-to-end (encode -> rank) with fitted heads
def _fit_factors(F: np.ndarray, T: np.ndarray):
    """Minimum-norm W [D, d] with F W^T = T (F [m, d] float64 features of rank m <= d), as bf16 factors
    W = A B: B = bf16(V^T) [m, d] from F = U S V^T, then A = ((F B^T)^-1 T)^T [D, m] solved against the
    ROUNDED B (F W^T = (F B^T) A^T = T), so A's own rounding costs one bf16 ulp of the targets (A's column i scales like 1/s_i and
    multiplies back s_i), not the condition number of F."""
    _, _, Vt = np.linalg.svd(F, full_matrices=False)
    B = bf16_bits(torch.from_numpy(Vt.astype(np.float32)))
    Bf = (B.astype(np.uint32) << 16).view(np.float32).astype(np.float64)
    A = np.linalg.solve(F @ Bf.T, T).T
    return bf16_bits(torch.from_numpy(A.astype(np.float32))), B


def make_e2e(main, models=None, fname="e2e_fitted.npz"):
    """End-to-end parity fixture: the reference's own encode_data (main.py:386-438)
    -> compute_similarity_scores (main.py:440-475) -> compute_metrics_detailed (main.py:305-383, v28 I2T
    orientation) on inputs whose ranking is DECIDED beyond bf16 noise.

    With random weights every embedding clusters (pairwise cosine 0.9+), so the top-10 score gaps
    (~1e-4) sit far below the ~1e-3 score noise of any bf16 tower, on the device or on the CPU. Here
    the towers keep their seeded random weights except the last linear map into the joint space,
    which is FITTED in closed form (minimum-norm least squares on the fp32 reference's own pooled
    features) onto graded targets (planted.graded_targets): every T2I / Sym row and the top of every
    I2T row then sees 12 distinct levels 0.038 apart, and recall is not chance (R@1 / R@5 50 %, R@10
    100 %). The fitted maps are the models' weights, used identically by the reference run here and
    by the device on the GPU box: CLIP visual_projection / text_projection; SigLIP the MAP head's
    mlp.fc2 (weight + bias, so image = r + fc2(h) hits the target) and text_model.head. They are
    stored as bf16 factors A [D, m], B [m, d] (weights_gen.factor_product rebuilds W = bf16(A B)
    bit-identically on any box; SHA-256 stored). The inputs are synthetic noise images and ragged
    random-id captions (planted.e2e_inputs), encoded at the reference's --batch-size 32.
    `models` (default planted.E2E_MODELS) / `fname`: the ViT-H towers (planted.E2E_H_MODELS) are written to
    e2e_fitted_h.npz by the same recipe ("e2e_h")."""
    from PIL import Image
    from transformers.models.siglip.image_processing_pil_siglip import SiglipImageProcessorPil
    from transformers.models.clip.image_processing_pil_clip import CLIPImageProcessorPil
    import hashlib
    from mme.config import get_spec
    from planted import E2E_MODELS, e2e_inputs, graded_targets
    from weights_gen import factor_product
    caps, bs = 5, 32
    models = E2E_MODELS if models is None else models
    out = {"models": np.array([m[0] for m in models]), "caps": np.int64(caps), "batch_size": np.int64(bs)}
    torch.set_num_threads(os.cpu_count() or 8)
    for name, n, H in models:
        spec = get_spec(name)
        key = name.replace("-", "_")
        imgs, rows = e2e_inputs(spec, n, H, caps)
        S = spec.vision.image_size
        ip = (SiglipImageProcessorPil(size={"height": S, "width": S}) if spec.family == "siglip" else
              CLIPImageProcessorPil(size={"shortest_edge": S}, crop_size={"height": S, "width": S}))
        proc = RefProcessor(ip, spec.text.pad_id)
        pil = [Image.fromarray(a) for a in imgs]
        # 1. the fp32 reference's pooled features ahead of the fitted maps, batched as encode_data batches
        hf = hf_model(spec, torch.float32)
        fi, fc, ri = [], [], []
        with torch.no_grad():
            for s in range(0, n, bs):
                pv = proc(images=pil[s:s + bs])["pixel_values"]
                if spec.family == "clip":
                    fi.append(hf.vision_model(pixel_values=pv).pooler_output)
                else:
                    head = hf.vision_model.head
                    x = hf.vision_model(pixel_values=pv).last_hidden_state
                    r = head.attention(head.probe.repeat(x.shape[0], 1, 1), x, x)[0]
                    h = head.mlp.activation_fn(head.mlp.fc1(head.layernorm(r)))
                    fi.append(h[:, 0])
                    ri.append(r[:, 0])
            # SigLIP pools the LAST position, a pad token for shorter rows, so a caption's feature depends on
            # its batch's padded length: the T2I encode (main.py:554, its own batches) is fitted too
            t2i_rows = rows[::caps]
            for rr in ((rows,) if spec.family == "clip" else (rows, t2i_rows)):
                for s in range(0, len(rr), bs):
                    b = proc(text=rr[s:s + bs])
                    if spec.family == "clip":
                        fc.append(hf.text_model(**b).pooler_output)
                    else:
                        fc.append(hf.text_model(**b).last_hidden_state[:, -1])
        Fi, Fc = torch.cat(fi).double().numpy(), torch.cat(fc).double().numpy()
        if spec.family != "clip":  # a T2I row padded as in its all-captions batch has the same feature: drop it
            def padded(rr):
                return [max(len(r) for r in rr[s:s + bs]) for s in range(0, len(rr), bs) for _ in rr[s:s + bs]]
            keep = np.array(padded(rows)[::caps]) != np.array(padded(t2i_rows))
            Fc = np.concatenate([Fc[:len(rows)], Fc[len(rows):][keep]])
        D = spec.proj_dim if spec.family == "clip" else spec.vision.hidden
        zi, zc = graded_targets(n, caps, D, seed=0)
        if spec.family == "clip":
            Ti, Tc = zi, zc
        else:  # image = r + fc2(h) + b2 = |r| z  ->  [h, 1] [W2, b2]^T = |r| z - r ; text = head(f) = z
            R = torch.cat(ri).double().numpy()
            Ti = np.median(np.linalg.norm(R, axis=1)) * zi - R
            Tc = np.concatenate([zc, zc[::caps][keep]])
            Fi = np.concatenate([Fi, np.ones((n, 1))], 1)
            Fc = np.concatenate([Fc, np.ones((Fc.shape[0], 1))], 1)
        ov = {}
        for tag, F, T in (("img", Fi, Ti), ("txt", Fc, Tc)):
            A, B = _fit_factors(F, T)
            W = factor_product(A, B)
            out[f"{key}_{tag}_A"], out[f"{key}_{tag}_B"] = A, B
            out[f"{key}_{tag}_sha"] = np.array(hashlib.sha256(W.view(np.uint32).tobytes()).hexdigest()[:32])
            if spec.family == "clip":
                ov["visual_projection.weight" if tag == "img" else "text_projection.weight"] = W
            elif tag == "img":
                ov["vision_model.head.mlp.fc2.weight"], ov["vision_model.head.mlp.fc2.bias"] = W[:, :-1], W[:, -1]
            else:
                ov["text_model.head.weight"], ov["text_model.head.bias"] = W[:, :-1], W[:, -1]
        del hf
        # 2. the reference's chain with the fitted heads, bf16 (the reference's precision) and fp32
        m_info = {"name": name, "type": spec.m_info["type"], "batch_size": bs}
        out[f"{key}_params"] = np.array([n, caps, H, 41], np.int64)
        out[f"{key}_cap_lens"] = np.array([len(r) for r in rows], np.int64)
        out[f"{key}_cap_ids"] = np.concatenate(rows).astype(np.int64)
        for tag, dtype in (("bf16", torch.bfloat16), ("f32", torch.float32)):
            mdl = RefAdapter(hf_model(spec, dtype, overrides=ov))
            main.DEVICE, main.DTYPE = "cpu", dtype
            with torch.no_grad():
                img_e, all_e = main.encode_data(mdl, proc, m_info, pil, rows)
                _, t2i_e = main.encode_data(mdl, proc, m_info, [], rows[::caps])
            if tag == "f32":
                out[f"{key}_img_f32"], out[f"{key}_all_f32"], out[f"{key}_t2i_f32"] = (
                    img_e.numpy(), all_e.numpy(), t2i_e.numpy())
                continue
            out[f"{key}_img_bf16"], out[f"{key}_all_bf16"], out[f"{key}_t2i_bf16"] = (
                bf16_bits(img_e), bf16_bits(all_e), bf16_bits(t2i_e))
            s_t2i = main.compute_similarity_scores(img_e, t2i_e, {"type": "dense"}, None)   # [n, n]  = t2i @ img.T
            s_i2t = main.compute_similarity_scores(all_e, img_e, {"type": "dense"}, None)   # [n, 5n] = img @ all.T
            s_sym = s_t2i.t().contiguous()
            metrics = main.compute_metrics_detailed(s_t2i, s_i2t, s_sym, list(range(n)),
                                                    {i: list(range(caps * i, caps * i + caps)) for i in range(n)},
                                                    {i: i for i in range(n)}, [""] * n)
            for p, s in (("t2i", s_t2i), ("i2t", s_i2t), ("sym", s_sym)):
                v, _ = torch.topk(s, 11, dim=1)
                ix = torch.stack([torch.topk(s[i], 10).indices for i in range(n)])  # compute_metrics_detailed's call
                out[f"{key}_{p}_idx"], out[f"{key}_{p}_score"] = ix.numpy().astype(np.int32), v.numpy()
                gaps = (v[:, :-1] - v[:, 1:]).min(1).values
                print(f"e2e {name} {p}: top-11 min gap median {gaps.median():.3e} min {gaps.min():.3e}", flush=True)
            keys = [k for k in metrics if not k.startswith("_")]
            out["metric_names"] = np.array(keys)
            out[f"{key}_metric_values"] = np.array([metrics[k] for k in keys], np.float64)
            print(f"e2e {name}:", dict(zip(keys, out[f"{key}_metric_values"].round(2))), flush=True)
        e16 = {k: bits_f32(out[f"{key}_{k}_bf16"]) for k in ("img", "all", "t2i")}
        for k in ("img", "all", "t2i"):
            c = (e16[k] * out[f"{key}_{k}_f32"]).sum(1) / np.linalg.norm(e16[k], axis=1)
            print(f"e2e {name} {k}: bf16 vs fp32 reference cos min {c.min():.5f}", flush=True)
    np.savez_compressed(os.path.join(HERE, fname), **out)
    print(f"{fname}:", sum(v.nbytes for v in out.values()) / 1e6, "MB raw")


def bits_f32(b):
    return (np.asarray(b, np.uint16).astype(np.uint32) << 16).view(np.float32)


# ------------------------------------------------------------------ retrieval
def planted(n, caps, D, noise, seed=0):
    """SURVEY.md §8d planted embeddings: img = norm(base + noise*N), cap_{5i+j} = norm(base_i + noise*N)."""
    g = torch.Generator().manual_seed(seed)
    base = torch.randn(n, D, generator=g)
    img = base + noise * torch.randn(n, D, generator=g)
    cap = base.repeat_interleave(caps, 0) + noise * torch.randn(n * caps, D, generator=g)
    img = (img / img.norm(dim=-1, keepdim=True)).to(torch.bfloat16)
    cap = (cap / cap.norm(dim=-1, keepdim=True)).to(torch.bfloat16)
    return img, cap


def make_retrieval(main):
    n, caps, D = 500, 5, 128
    img, all_txt = planted(n, caps, D, noise=1.6)
    t2i = all_txt[::caps].contiguous()
    m_info = {"type": "dense"}
    main.DEVICE = "cpu"
    s_t2i = main.compute_similarity_scores(img, t2i, m_info, None)           # [n, n] = t2i @ img.T
    s_i2t = main.compute_similarity_scores(all_txt, img, m_info, None)       # [n, 5n] = img @ all.T (no .t())
    s_sym = s_t2i.t()
    metrics = main.compute_metrics_detailed(s_t2i, s_i2t, s_sym, list(range(n)),
                                            {i: list(range(caps * i, caps * i + caps)) for i in range(n)},
                                            {i: i for i in range(n)}, [""] * n)
    out = {"img": bf16_bits(img), "all_txt": bf16_bits(all_txt)}
    for tag, s in (("t2i", s_t2i), ("i2t", s_i2t), ("sym", s_sym.contiguous())):
        v, ix = torch.topk(s, 11, dim=1)
        out[f"{tag}_idx"] = ix[:, :10].numpy().astype(np.int32)
        out[f"{tag}_score"] = v[:, :10].numpy()
        out[f"{tag}_margin"] = (v[:, 9] - v[:, 10]).numpy()
    keys = [k for k in metrics if not k.startswith("_")]
    out["metric_names"] = np.array(keys)
    out["metric_values"] = np.array([metrics[k] for k in keys], np.float64)
    np.savez_compressed(os.path.join(HERE, "retrieval.npz"), **out)
    print("retrieval.npz:", dict(zip(keys, out["metric_values"].round(2))))


def make_edge(main):
    """Edge cases of the reference's ranking (main.py:305-383, 440-475) and encode loop (main.py:386-438):
    fewer columns than k (n = 1, 2 and 3 images: torch.topk(k = min(k, ncols))), a ragged last batch,
    and empty inputs (encode_data on [] returns torch.empty(0))."""
    out = {}
    for n, D, noise in ((1, 64, 0.5), (2, 96, 1.0), (3, 128, 1.2), (7, 64, 1.5), (33, 128, 2.0)):
        img, all_txt = planted(n, 5, D, noise=noise, seed=100 + n)
        t2i = all_txt[::5].contiguous()
        main.DEVICE = "cpu"
        s_t2i = main.compute_similarity_scores(img, t2i, {"type": "dense"}, None)
        s_i2t = main.compute_similarity_scores(all_txt, img, {"type": "dense"}, None)
        m = main.compute_metrics_detailed(s_t2i, s_i2t, s_t2i.t(), list(range(n)),
                                          {i: list(range(5 * i, 5 * i + 5)) for i in range(n)},
                                          {i: i for i in range(n)}, [""] * n)
        keys = [k for k in m if not k.startswith("_")]
        out[f"n{n}_img"], out[f"n{n}_all_txt"] = bf16_bits(img), bf16_bits(all_txt)
        out[f"n{n}_metrics"] = np.array([m[k] for k in keys], np.float64)
    out["metric_names"] = np.array(keys)

    class Feed:  # encode_data over empty lists never calls the model
        def get_image_features(self, **_):
            raise AssertionError("called on an empty list")

        get_text_features = get_image_features
    main.DEVICE, main.DTYPE = "cpu", torch.bfloat16
    e_img, e_txt = main.encode_data(Feed(), None, {"type": "dense", "batch_size": 32}, [], [])
    out["empty_shapes"] = np.array([list(e_img.shape), list(e_txt.shape)], np.int64)
    np.savez_compressed(os.path.join(HERE, "edge.npz"), **out)
    print("edge.npz:", {k: v.tolist() for k, v in out.items() if k.endswith("metrics")}, out["empty_shapes"].tolist())


def make_full_retrieval(main):
    """BASELINE configs[1] geometry: n = 5 000 images, m = 25 000 captions, D = 1152,
    planted noise 3.0, ranked by the reference's own compute_similarity_scores +
    compute_metrics_detailed (v28 I2T orientation). Only the seed / checksums, each row's
    top-11 indices and scores, and the 9 metrics are stored; the GPU test regenerates the
    embeddings (tests/golden/planted.py) and checks their checksum first."""
    from planted import bf16_sha, planted_np
    n, caps, D, noise, seed = 5000, 5, 1152, 3.0, 0
    img, all_txt = planted_np(n, caps, D, noise, seed)
    t2i = all_txt[::caps].contiguous()
    m_info = {"type": "dense"}
    main.DEVICE = "cpu"
    s_t2i = main.compute_similarity_scores(img, t2i, m_info, None)           # [n, n]  = t2i @ img.T
    s_i2t = main.compute_similarity_scores(all_txt, img, m_info, None)       # [n, 5n] = img @ all.T (v28)
    s_sym = s_t2i.t()
    metrics = main.compute_metrics_detailed(s_t2i, s_i2t, s_sym, list(range(n)),
                                            {i: list(range(caps * i, caps * i + caps)) for i in range(n)},
                                            {i: i for i in range(n)}, [""] * n)
    out = {"params": np.array([n, caps, D, seed], np.int64), "noise": np.float64(noise),
           "img_sha": np.array(bf16_sha(img)), "txt_sha": np.array(bf16_sha(all_txt))}
    for tag, s in (("t2i", s_t2i), ("i2t", s_i2t), ("sym", s_sym.contiguous())):
        v, ix = torch.topk(s, 11, dim=1)
        out[f"{tag}_idx"] = ix.numpy().astype(np.int32)
        out[f"{tag}_score"] = v.numpy().astype(np.float32)
    keys = [k for k in metrics if not k.startswith("_")]
    out["metric_names"] = np.array(keys)
    out["metric_values"] = np.array([metrics[k] for k in keys], np.float64)
    np.savez_compressed(os.path.join(HERE, "full_retrieval.npz"), **out)
    print("full_retrieval.npz:", dict(zip(keys, out["metric_values"].round(2))))


DENSE_TIE_CASES = (  # (tag, n images, D, noise, seed): both sides of torch.topk's k * 64 <= n switch
    ("wide", 1000, 256, 1.3, 31),    # T2I / Sym 1 000 columns: partial_sort at k = 1, 5, 10
    ("narrow", 300, 256, 1.3, 32),   # 300 columns: partial_sort at k = 1, nth_element at k = 5, 10
    ("tiny", 40, 128, 1.0, 33),      # 40 columns: nth_element at every k; I2T 200: partial_sort at k = 1
)


def make_dense_ties(main):
    """Exact fp32 score ties on the dense path: planted embeddings with exact
    duplicates (tests/golden/planted.py planted_ties: repeated images, caption rows repeated across
    images of one base), scored by the reference's own compute_similarity_scores and ranked by its
    compute_metrics_detailed (main.py:305-383, 440-475; v28 I2T orientation). Stored per case: seed /
    checksums, the duplicate groups, per row the reference's torch.topk(row, 10) indices, top-11 scores
    and the hit flags of compute_metrics_detailed's own per-k calls, and the 9 metrics. The GPU test
    regenerates the embeddings and checks the checksums first."""
    from planted import bf16_sha, planted_ties
    out, caps = {}, 5
    for tag, n, D, noise, seed in DENSE_TIE_CASES:
        img, all_txt, groups = planted_ties(n, caps, D, noise, seed)
        t2i = all_txt[::caps].contiguous()
        m_info = {"type": "dense"}
        main.DEVICE = "cpu"
        s_t2i = main.compute_similarity_scores(img, t2i, m_info, None)           # [n, n]  = t2i @ img.T
        s_i2t = main.compute_similarity_scores(all_txt, img, m_info, None)       # [n, 5n] = img @ all.T (v28)
        s_sym = s_t2i.t().contiguous()
        metrics = main.compute_metrics_detailed(s_t2i, s_i2t, s_sym, list(range(n)),
                                                {i: list(range(caps * i, caps * i + caps)) for i in range(n)},
                                                {i: i for i in range(n)}, [""] * n)
        hits = np.zeros((3, n, 3), bool)
        tied = np.zeros((3, n), bool)
        for p, (ptag, s, tgt) in enumerate((("t2i", s_t2i, lambda i: [i]),
                                            ("i2t", s_i2t, lambda i: range(caps * i, caps * i + caps)),
                                            ("sym", s_sym, lambda i: [i]))):
            for i in range(n):
                for j, k in enumerate((1, 5, 10)):
                    top = torch.topk(s[i], k=min(k, s.shape[1])).indices.tolist()
                    hits[p, i, j] = any(c in top for c in tgt(i))
            kk = min(11, s.shape[1])
            v11, _ = torch.topk(s, kk, dim=1)
            k10 = min(10, s.shape[1])
            ix10 = torch.stack([torch.topk(s[i], k10).indices for i in range(n)])
            tied[p] = (v11[:, 1:] == v11[:, :-1]).any(1).numpy()
            cols = np.broadcast_to(np.arange(s.shape[1]), s.shape)
            lex = np.lexsort((cols, -s.numpy()), axis=1)[:, :k10]
            out[f"{tag}_{ptag}_idx"] = ix10.numpy().astype(np.int32)
            out[f"{tag}_{ptag}_score"] = v11.numpy().astype(np.float32)
            print(f"dense_ties {tag} {ptag}: {int(tied[p].sum())}/{n} rows with an exact tie in the top {kk}; "
                  f"torch order != (score desc, column asc) on {int((lex != ix10.numpy()).any(1).sum())} rows")
        keys = [k for k in metrics if not k.startswith("_")]
        vals = np.array([metrics[k] for k in keys], np.float64)
        assert np.allclose(vals.reshape(3, 3), 100.0 * hits.sum(1) / n)
        # the duplicated columns score exactly equal in the reference's own fp32 matmul
        for mode, size, *mem in groups.tolist():
            mem = mem[:size]
            if mode in (0, 3):
                assert (s_t2i[:, mem] == s_t2i[:, mem[:1]]).all()
        out.update({f"{tag}_params": np.array([n, caps, D, seed], np.int64), f"{tag}_noise": np.float64(noise),
                    f"{tag}_img_sha": np.array(bf16_sha(img)), f"{tag}_txt_sha": np.array(bf16_sha(all_txt)),
                    f"{tag}_groups": groups, f"{tag}_hits": hits, f"{tag}_tied": tied,
                    f"{tag}_metric_values": vals})
        out["metric_names"] = np.array(keys)
        print(f"dense_ties {tag}:", dict(zip(keys, vals.round(2))))
    out["cases"] = np.array([c[0] for c in DENSE_TIE_CASES])
    np.savez_compressed(os.path.join(HERE, "dense_ties.npz"), **out)


# ------------------------------------------------------------------ maxsim + l2norm
def make_maxsim(main):
    from transformers.models.colpali.processing_colpali import ColPaliProcessor

    class Scorer:
        def score(self, qs, ps):
            return ColPaliProcessor.score_retrieval(None, qs, ps, output_dtype=torch.float32)

    out = {}
    rng = torch.Generator().manual_seed(3)
    for case, (nq, nd, qr, dr) in {"ragged": (23, 27, (5, 31), (20, 71)), "fixed": (12, 14, (26, 27), (64, 65))}.items():
        def mk(n, lo, hi):
            vs = []
            for _ in range(n):
                T = int(torch.randint(lo, hi, (1,), generator=rng))
                v = torch.randn(T, 128, generator=rng)
                vs.append((v / v.norm(dim=-1, keepdim=True)).to(torch.bfloat16))
            return vs
        qs, ds = mk(nq, *qr), mk(nd, *dr)
        main.DEVICE = "cpu"
        # the reference's own 10 x 10 chunk loop (main.py:451-470)
        s = main.compute_similarity_scores(ds, qs, {"type": "colpali"}, Scorer())
        out[f"{case}_q"] = np.concatenate([bf16_bits(v) for v in qs])
        out[f"{case}_qlen"] = np.array([v.shape[0] for v in qs], np.int32)
        out[f"{case}_d"] = np.concatenate([bf16_bits(v) for v in ds])
        out[f"{case}_dlen"] = np.array([v.shape[0] for v in ds], np.int32)
        out[f"{case}_score"] = s.numpy().astype(np.float32)
    np.savez_compressed(os.path.join(HERE, "maxsim.npz"), **out)
    print("maxsim.npz:", {k: v.shape for k, v in out.items()})


def make_colpali_recall(main):
    """ColPali recall at a non-trivial size (SURVEY §8d config 4 geometry, n scaled to 64):
    64 images x 1 030 planted doc tokens, 320 captions of 8..20 tokens left-padded per batch
    of 4 (tests/golden/planted.py), scored by the reference's own colpali branch of
    compute_similarity_scores (10 x 10 chunk loop, main.py:451-470; processor.score =
    transformers' ColPaliProcessor.score_retrieval, the in-container colpali_engine stand-in)
    and ranked by compute_metrics_detailed (main.py:305-383, per-row torch.topk for k = 1, 5, 10,
    v28 I2T orientation). Stores both score matrices and the reference's per-row hit flags."""
    from planted import bf16_sha, left_padded_items, planted_multivec
    from transformers.models.colpali.processing_colpali import ColPaliProcessor

    class Scorer:
        def score(self, qs, ps):
            return ColPaliProcessor.score_retrieval(None, qs, ps, output_dtype=torch.float32)

    n, caps, Ld, qlens, noise, seed = 64, 5, 1030, (8, 21), 7.0, 0
    img, cap, lens, pad = planted_multivec(n, caps, Ld, qlens, noise, seed=seed)
    imgs = [img[i] for i in range(n)]
    cap_items = left_padded_items(cap, lens, pad)
    # T2I queries are caption 0 of each image, encoded in their own batches of 4 (main.py:554)
    t2i_lens = lens[::caps].clone()
    t2i_pad = torch.tensor([int(t2i_lens[s:s + 4].max()) for s in range(0, n, 4) for _ in range(min(4, n - s))],
                           dtype=torch.int32)
    t2i_items = left_padded_items(cap[::caps].contiguous(), t2i_lens, t2i_pad)
    main.DEVICE = "cpu"
    m_info = {"type": "colpali"}
    s_t2i = main.compute_similarity_scores(imgs, t2i_items, m_info, Scorer())       # [n, n]
    s_i2t = main.compute_similarity_scores(cap_items, imgs, m_info, Scorer())       # [n, 5n] (v28 orientation)
    s_sym = s_t2i.t().contiguous()
    metrics = main.compute_metrics_detailed(s_t2i, s_i2t, s_sym, list(range(n)),
                                            {i: list(range(caps * i, caps * i + caps)) for i in range(n)},
                                            {i: i for i in range(n)}, [""] * n)
    hits = np.zeros((3, n, 3), bool)  # the reference's own per-row outcome (same torch.topk calls)
    for p, (s, tgt) in enumerate(((s_t2i, lambda i: [i]), (s_i2t, lambda i: range(caps * i, caps * i + caps)),
                                  (s_sym, lambda i: [i]))):
        for i in range(n):
            for j, k in enumerate((1, 5, 10)):
                top = torch.topk(s[i], k=min(k, s.shape[1])).indices.tolist()
                hits[p, i, j] = any(c in top for c in tgt(i))
    keys = [k for k in metrics if not k.startswith("_")]
    vals = np.array([metrics[k] for k in keys], np.float64)
    assert np.allclose(vals.reshape(3, 3), 100.0 * hits.sum(1) / n)
    out = {"params": np.array([n, caps, Ld, qlens[0], qlens[1], seed], np.int64), "noise": np.float64(noise),
           "img_sha": np.array(bf16_sha(img)), "cap_sha": np.array(bf16_sha(cap)),
           "t2i_score": s_t2i.numpy().astype(np.float32), "i2t_score": s_i2t.numpy().astype(np.float32),
           "hits": hits, "metric_names": np.array(keys), "metric_values": vals}
    np.savez_compressed(os.path.join(HERE, "colpali_recall.npz"), **out)
    print("colpali_recall.npz:", dict(zip(keys, vals.round(2))))


_CPF = {}  # worker state of make_colpali_full (spawned processes, one torch thread each)


def _colpali_full_init(tmp):
    torch.set_num_threads(1)
    from planted import left_padded_items
    from transformers.models.colpali.processing_colpali import ColPaliProcessor
    img = torch.from_numpy(np.load(os.path.join(tmp, "img.npy"))).view(torch.bfloat16)
    cap = torch.from_numpy(np.load(os.path.join(tmp, "cap.npy"))).view(torch.bfloat16)
    lens, pad = (torch.from_numpy(np.load(os.path.join(tmp, f"{k}.npy"))) for k in ("lens", "pad"))
    t2i_pad = torch.from_numpy(np.load(os.path.join(tmp, "t2i_pad.npy")))
    caps = int(np.load(os.path.join(tmp, "caps.npy")))

    class Scorer:
        def score(self, qs, ps):
            return ColPaliProcessor.score_retrieval(None, qs, ps, output_dtype=torch.float32)
    _CPF.update(main=import_reference(), scorer=Scorer(), imgs=[img[i] for i in range(img.shape[0])],
                t2i=left_padded_items(cap[::caps].contiguous(), lens[::caps].clone(), t2i_pad),
                caps=left_padded_items(cap, lens, pad))
    _CPF["main"].DEVICE = "cpu"


def _colpali_full_rows(task):
    """Rows [lo, hi) (a multiple of the reference's chunk of 10) of one score matrix, computed
    by the reference's own compute_similarity_scores colpali branch: every 10 x 10 chunk call
    of the full loop over these query rows, in the same order."""
    which, lo, hi = task
    m = _CPF["main"]
    if which == "t2i":   # queries = caption-0 items, docs = images
        s = m.compute_similarity_scores(_CPF["imgs"], _CPF["t2i"][lo:hi], {"type": "colpali"}, _CPF["scorer"])
    else:                # I2T (v28 orientation): queries = images, docs = all caption items
        s = m.compute_similarity_scores(_CPF["caps"], _CPF["imgs"][lo:hi], {"type": "colpali"}, _CPF["scorer"])
    return which, lo, s.numpy()


def make_colpali_full(main, workers: int = 7):
    """BASELINE configs[3] at its full geometry: 1 000 images x 1 030 planted doc tokens and
    5 000 captions of 23..29 tokens (Tq ~ 26) left-padded per batch of 4
    (tests/golden/planted.py, noise 7.0: T2I R@1 ~ 34 %). Scored by the reference's own colpali
    branch of compute_similarity_scores (10 x 10 chunk loop, main.py:451-470; processor.score =
    transformers' ColPaliProcessor.score_retrieval) and ranked by compute_metrics_detailed
    (main.py:305-383, v28 I2T orientation). The 60 000 chunk calls run in `workers` spawned
    processes with one torch thread each (the per-call scores are bit-identical to the
    multi-threaded ones and 4x faster); each worker takes whole chunk rows of 10 queries, so
    every call sees exactly the chunks of the full loop. Stored: seed / checksums, per row the
    reference's own torch.topk(row, 10) indices and its top-11 scores, the per-row hit flags of
    compute_metrics_detailed's calls, a sample of whole score rows, and the 9 metrics."""
    import multiprocessing as mp
    from planted import bf16_sha, planted_multivec
    n, caps, Ld, qlens, noise, seed = 1000, 5, 1030, (23, 30), 7.0, 0
    img, cap, lens, pad = planted_multivec(n, caps, Ld, qlens, noise, seed=seed)
    t2i_lens = lens[::caps].clone()
    t2i_pad = torch.tensor([int(t2i_lens[s:s + 4].max()) for s in range(0, n, 4) for _ in range(min(4, n - s))],
                           dtype=torch.int32)
    tmp = tempfile.mkdtemp(prefix="mme_cpf_")
    np.save(os.path.join(tmp, "img.npy"), img.view(torch.int16).numpy())
    np.save(os.path.join(tmp, "cap.npy"), cap.view(torch.int16).numpy())
    for k, v in (("lens", lens), ("pad", pad), ("t2i_pad", t2i_pad)):
        np.save(os.path.join(tmp, f"{k}.npy"), v.numpy())
    np.save(os.path.join(tmp, "caps.npy"), np.int64(caps))
    tasks = [("i2t", lo, min(lo + 20, n)) for lo in range(0, n, 20)] + \
            [("t2i", lo, min(lo + 50, n)) for lo in range(0, n, 50)]
    S = {"t2i": torch.empty(n, n), "i2t": torch.empty(n, caps * n)}
    with mp.get_context("spawn").Pool(workers, initializer=_colpali_full_init, initargs=(tmp,)) as pool:
        for done, (which, lo, s) in enumerate(pool.imap_unordered(_colpali_full_rows, tasks)):
            S[which][lo:lo + s.shape[0]] = torch.from_numpy(s)
            print(f"colpali_full: {done + 1}/{len(tasks)} row blocks", flush=True)
    s_t2i, s_i2t = S["t2i"], S["i2t"]
    s_sym = s_t2i.t().contiguous()
    metrics = main.compute_metrics_detailed(s_t2i, s_i2t, s_sym, list(range(n)),
                                            {i: list(range(caps * i, caps * i + caps)) for i in range(n)},
                                            {i: i for i in range(n)}, [""] * n)
    hits = np.zeros((3, n, 3), bool)  # the reference's own per-row outcome (the same torch.topk calls)
    out = {"params": np.array([n, caps, Ld, qlens[0], qlens[1], seed], np.int64), "noise": np.float64(noise),
           "img_sha": np.array(bf16_sha(img)), "cap_sha": np.array(bf16_sha(cap))}
    lowest = np.zeros((3, n), bool)  # torch.topk(row, 10) == the (score desc, column asc) order
    for p, (tag, s, tgt) in enumerate((("t2i", s_t2i, lambda i: [i]),
                                       ("i2t", s_i2t, lambda i: range(caps * i, caps * i + caps)),
                                       ("sym", s_sym, lambda i: [i]))):
        for i in range(n):
            for j, k in enumerate((1, 5, 10)):
                top = torch.topk(s[i], k=min(k, s.shape[1])).indices.tolist()
                hits[p, i, j] = any(c in top for c in tgt(i))
        v11, _ = torch.topk(s, 11, dim=1)
        ix10 = torch.stack([torch.topk(s[i], 10).indices for i in range(n)])
        cols = np.broadcast_to(np.arange(s.shape[1]), s.shape)
        lex = np.lexsort((cols, -s.numpy()), axis=1)[:, :10]
        lowest[p] = (lex == ix10.numpy()).all(1)
        out[f"{tag}_idx"] = ix10.numpy().astype(np.int32)
        out[f"{tag}_score"] = v11.numpy().astype(np.float32)
        print(f"colpali_full {tag}: torch.topk order == (score desc, column asc) on {int(lowest[p].sum())}/{n} rows")
    keys = [k for k in metrics if not k.startswith("_")]
    vals = np.array([metrics[k] for k in keys], np.float64)
    assert np.allclose(vals.reshape(3, 3), 100.0 * hits.sum(1) / n)
    sample = np.array([0, 1, 2, 3, 250, 499, 500, 777, 996, 997, 998, 999], np.int64)
    out.update(hits=hits, lowest_index_rows=lowest, metric_names=np.array(keys), metric_values=vals,
               sample_rows=sample, t2i_rows=s_t2i[sample].numpy(), i2t_rows=s_i2t[sample].numpy())
    np.savez_compressed(os.path.join(HERE, "colpali_full.npz"), **out)
    print("colpali_full.npz:", dict(zip(keys, vals.round(2))))


def make_torch_topk():
    """torch.topk's own CPU outputs on tie-heavy rows (the selection main.py:335,365,375 runs per row):
    integer-level scores (2, 5 or 50 levels) so exact ties decide most rows, at widths on both sides of
    torch's partial_sort / nth_element switch (k * 64 <= n) and k = 1, 5, 10. Pins oracle/torch_topk.cpp
    and the device's mme_topk_rows_torch."""
    rng = np.random.default_rng(11)
    out, cases = {}, []
    for n in (7, 10, 64, 100, 320, 639, 640, 1000, 5000):
        for k in (1, 5, 10):
            if k > n:
                continue
            for levels in (2, 5, 50):
                s = rng.integers(0, levels, (6, n)).astype(np.float32) * np.float32(0.25)
                v, i = torch.topk(torch.from_numpy(s), k, dim=1)
                tag = f"n{n}_k{k}_l{levels}"
                out[f"{tag}_s"] = (s * 4).astype(np.uint8)
                out[f"{tag}_idx"] = i.numpy().astype(np.int32)
                cases.append(tag)
    out["cases"] = np.array(cases)
    np.savez_compressed(os.path.join(HERE, "torch_topk.npz"), **out)
    print("torch_topk.npz:", len(cases), "cases")


def make_l2norm(main):
    """main.py:414 `out / out.norm(dim=-1, keepdim=True)` on bf16 model outputs."""
    g = torch.Generator().manual_seed(5)
    x = (torch.randn(96, 1152, generator=g) * torch.rand(96, 1, generator=g) * 4).to(torch.bfloat16)

    class Feed:
        def get_image_features(self, pixel_values):
            return x[pixel_values[:, 0].long()]

    class P:
        def __call__(self, images=None, **_):
            from transformers import BatchFeature
            return BatchFeature({"pixel_values": torch.tensor(images, dtype=torch.float32)[:, None]})

    main.DEVICE, main.DTYPE = "cpu", torch.bfloat16
    y, _ = main.encode_data(Feed(), P(), {"type": "dense", "batch_size": 32}, list(range(96)), [])
    np.savez_compressed(os.path.join(HERE, "l2norm.npz"), x=bf16_bits(x), y=bf16_bits(y))
    print("l2norm.npz", y.shape)


# ------------------------------------------------------------------ ColPali encoder
class ColPaliRefModel:
    """model(**inputs) -> embeddings tensor [B, L, 128] (colpali_engine's ColPali returns the
    tensor; transformers' ColPaliForRetrieval wraps it in .embeddings)."""

    def __init__(self, hf):
        self.hf = hf

    def __call__(self, **kw):
        return self.hf(**kw).embeddings


class ColPaliRefProcessor:
    """process_images / process_queries with the ColPaliProcessor layout
    (TF:models/colpali/processing_colpali.py:113-142) over pre-tokenized ids:
    images [<image>]*P + [bos] + prompt + [\\n]; queries [bos] + prefix + ids + [pad]*10 + [\\n],
    left-padded (Gemma tokenizer padding_side='left'), token_type_ids all 0."""

    def __init__(self, spec, image_proc):
        self.spec, self.ip = spec, image_proc

    def _batch(self, rows):
        from transformers import BatchFeature
        L = max(len(r) for r in rows)
        ids = torch.full((len(rows), L), self.spec.pad_id, dtype=torch.int64)
        mask = torch.zeros((len(rows), L), dtype=torch.int64)
        for i, r in enumerate(rows):
            ids[i, L - len(r):] = torch.tensor(r)
            mask[i, L - len(r):] = 1
        return BatchFeature({"input_ids": ids, "attention_mask": mask, "token_type_ids": torch.zeros_like(ids)})

    def process_images(self, images):
        b = self._batch([list(self.spec.image_tokens)] * len(images))
        b["pixel_values"] = self.ip(images=images, return_tensors="pt")["pixel_values"]
        return b

    def process_queries(self, queries):
        return self._batch([list(self.spec.query_tokens(q)) for q in queries])


def hf_colpali(spec, dtype):
    from transformers import ColPaliConfig, ColPaliForRetrieval
    v, t = spec.vision, spec.text
    vc = dict(model_type="siglip_vision_model", hidden_size=v.hidden, intermediate_size=v.intermediate,
              num_hidden_layers=v.layers, num_attention_heads=v.heads, image_size=v.image_size, patch_size=v.patch,
              hidden_act=v.act, layer_norm_eps=v.eps, vision_use_head=False)
    tc = dict(model_type="gemma", hidden_size=t.hidden, intermediate_size=t.intermediate, num_hidden_layers=t.layers,
              num_attention_heads=t.heads, num_key_value_heads=1, head_dim=t.head_dim, vocab_size=t.vocab,
              rms_norm_eps=t.eps, hidden_act="gelu_pytorch_tanh", pad_token_id=spec.pad_id, bos_token_id=spec.bos_id,
              eos_token_id=spec.eos_id)
    cfg = ColPaliConfig(vlm_config=dict(model_type="paligemma", vision_config=vc, text_config=tc,
                                        image_token_index=spec.image_token_id, vocab_size=t.vocab,
                                        projection_dim=t.hidden, hidden_size=t.hidden), embedding_dim=spec.dim)
    m = ColPaliForRetrieval(cfg)
    sd = torch_state_dict(spec, seed=0)
    missing, unexpected = m.load_state_dict(sd, strict=False)
    assert not missing and not unexpected, (missing, unexpected)
    return m.to(dtype).eval()


def make_colpali(main):
    from PIL import Image
    from transformers.models.siglip.image_processing_pil_siglip import SiglipImageProcessorPil
    from mme.config import COLPALI

    spec = COLPALI["tiny-colpali"]
    S = spec.vision.image_size
    rng = np.random.default_rng(11)
    imgs = rng.integers(0, 256, (5, 96, 80, 3), dtype=np.uint8)
    pil = [Image.fromarray(a) for a in imgs]
    lens = [7, 3, 12, 5, 9, 4, 10]
    caps = [rng.integers(3, 990, L).tolist() for L in lens]
    proc = ColPaliRefProcessor(spec, SiglipImageProcessorPil(size={"height": S, "width": S}))
    m_info = {"name": "tiny-colpali", "type": "colpali", "batch_size": spec.batch_size}
    out = {"images": imgs, "cap_lens": np.array(lens, np.int64), "cap_ids": np.concatenate(caps).astype(np.int64)}
    for tag, dtype in (("bf16", torch.bfloat16), ("f32", torch.float32)):
        model = ColPaliRefModel(hf_colpali(spec, dtype))
        main.DEVICE, main.DTYPE = "cpu", dtype
        with torch.no_grad():
            # encode_data concatenates the per-item [T, 128] outputs along rows (main.py:416,436;
            # the flattening defect of SURVEY §0.2): the row counts below split them again
            cat_i, cat_t = main.encode_data(model, proc, m_info, pil, caps)
        bs = spec.batch_size
        img_rows = [len(spec.image_tokens)] * len(pil)
        txt_rows = []
        for s in range(0, len(caps), bs):
            Lb = max(len(spec.query_tokens(c)) for c in caps[s:s + bs])
            txt_rows += [Lb] * len(caps[s:s + bs])
        assert cat_i.shape[0] == sum(img_rows) and cat_t.shape[0] == sum(txt_rows)
        out["img_rows"], out["txt_rows"] = np.array(img_rows, np.int64), np.array(txt_rows, np.int64)
        if tag == "bf16":
            out["img_bf16"], out["txt_bf16"] = bf16_bits(cat_i), bf16_bits(cat_t)

            class Scorer:  # colpali_engine score -> transformers' score_retrieval stand-in
                def score(self, qs, ps):
                    from transformers.models.colpali.processing_colpali import ColPaliProcessor
                    return ColPaliProcessor.score_retrieval(None, qs, ps, output_dtype=torch.float32)

            # T2I orientation of run_bootstrap_benchmark with per-item lists kept intact
            # (the mme semantics): queries = captions, docs = images
            img_l, txt_l = list(cat_i.split(img_rows)), list(cat_t.split(txt_rows))
            out["t2i_score"] = main.compute_similarity_scores(img_l, txt_l, {"type": "colpali"}, Scorer()).numpy()
        else:
            out["img_f32"], out["txt_f32"] = cat_i.numpy(), cat_t.numpy()
    np.savez_compressed(os.path.join(HERE, "tiny-colpali.npz"), **out)
    print("tiny-colpali.npz:", {k: v.shape for k, v in out.items()})


# ------------------------------------------------------------------ Winoground
def make_winoground():
    """The reference's own run_winoground (run_benchmark_grand_slam_v28_publication_ready.py:413-461)
    over the tiny models, with its load_dataset patched to return synthetic examples."""
    from PIL import Image
    from transformers.models.siglip.image_processing_pil_siglip import SiglipImageProcessorPil
    from transformers.models.clip.image_processing_pil_clip import CLIPImageProcessorPil
    cwd = os.getcwd()
    os.chdir(tempfile.mkdtemp(prefix="mme_ref_"))
    sys.path.insert(0, REF)
    import run_benchmark_grand_slam_v28_publication_ready as v28  # noqa: E402
    os.chdir(cwd)
    sys.path.insert(0, os.path.join(REPO, "multimodal-embedding_amd"))
    from mme.winoground import synthetic_examples
    out = {}
    for name in ("tiny-siglip", "tiny-clip"):
        spec = TINY[name]
        t = spec.text
        lo, hi = (1, min(t.bos_id, t.eos_id)) if t.bos_id is not None else (2, t.vocab)
        exs = synthetic_examples(40, seed=3, size=72, vocab=(lo, hi), lens=(3, t.max_pos - 2))
        for ex in exs:  # the tokenizer's special tokens, as the reference's processor would add them
            for j in (0, 1):
                c = ex[f"caption_{j}"]
                ex[f"caption_{j}"] = ([t.bos_id] + c + [t.eos_id]) if t.bos_id is not None else (c + [t.eos_id])
        S = spec.vision.image_size
        ip = (SiglipImageProcessorPil(size={"height": S, "width": S}) if spec.family == "siglip" else
              CLIPImageProcessorPil(size={"shortest_edge": S}, crop_size={"height": S, "width": S}))
        proc = RefProcessor(ip, t.pad_id)
        hf = RefAdapter(hf_model(spec, torch.bfloat16))
        ds = [{"image_0": Image.fromarray(e["image_0"]), "image_1": Image.fromarray(e["image_1"]),
               "caption_0": e["caption_0"], "caption_1": e["caption_1"]} for e in exs]
        v28.DEVICE, v28.DTYPE = "cpu", torch.bfloat16
        v28.load_dataset = lambda *a, **k: ds
        m = v28.run_winoground(hf, proc, {"type": spec.m_info["type"]})
        assert m, "run_winoground returned no metrics"
        key = name.replace("-", "_")
        # per-example 2x2 scores through the same modules (run_winoground's dense steps,
        # restated) so tests can tell decisive decisions from bf16 near-ties
        sc = []
        with torch.no_grad():
            for e in ds:
                ie = hf.get_image_features(**proc(images=[e["image_0"], e["image_1"]]))
                te = hf.get_text_features(**proc(text=[e["caption_0"], e["caption_1"]]))
                ie, te = ie / ie.norm(dim=-1, keepdim=True), te / te.norm(dim=-1, keepdim=True)
                sc.append(torch.matmul(te.to(torch.bfloat16), ie.to(torch.bfloat16).t()).float().reshape(4).numpy())
        sc = np.stack(sc)
        tx = (sc[:, 0] > sc[:, 1]) & (sc[:, 3] > sc[:, 2])
        im = (sc[:, 0] > sc[:, 2]) & (sc[:, 3] > sc[:, 1])
        n = len(ds)
        assert [100.0 * tx.sum() / n, 100.0 * im.sum() / n, 100.0 * (tx & im).sum() / n] == \
            [m["Wino Text"], m["Wino Image"], m["Wino Group"]], "restated scores disagree with run_winoground"
        out[f"{key}_scores"] = sc.astype(np.float32)
        out[f"{key}_metrics"] = np.array([m["Wino Text"], m["Wino Image"], m["Wino Group"]], np.float64)
        out[f"{key}_images"] = np.stack([np.stack([e["image_0"], e["image_1"]]) for e in exs])
        caps = [e[f"caption_{j}"] for e in exs for j in (0, 1)]
        out[f"{key}_cap_lens"] = np.array([len(c) for c in caps], np.int64)
        out[f"{key}_cap_ids"] = np.concatenate(caps).astype(np.int64)
    np.savez_compressed(os.path.join(HERE, "winoground.npz"), **out)
    print("winoground.npz:", {k: v.tolist() for k, v in out.items() if k.endswith("metrics")})


# ------------------------------------------------------------------ bootstrap
def make_bootstrap(main):
    """The reference's own resampled scoring + compute_metrics_detailed (main.py:586-634) on planted
    embeddings, with seeded sample indices (the reference's np.random.choice is unseeded, §0.5)."""
    n, caps, D, iters = 120, 5, 64, 25
    img, all_txt = planted(n, caps, D, noise=1.2, seed=4)
    t2i = all_txt[::caps].contiguous()
    rng = np.random.default_rng(11)
    samples = rng.integers(0, n, (iters, n)).astype(np.int32)
    main.DEVICE = "cpu"
    m_info = {"type": "dense"}
    vals = []
    for smp in samples:
        si, st = img[smp], t2i[smp]
        capidx = [c for i in smp for c in range(caps * int(i), caps * int(i) + caps)]
        s_t2i = main.compute_similarity_scores(si, st, m_info, None)
        s_i2t = main.compute_similarity_scores(all_txt[capidx], si, m_info, None)  # v28 orientation (no .t())
        m = main.compute_metrics_detailed(s_t2i, s_i2t, s_t2i.t(), list(range(n)),
                                          {i: list(range(caps * i, caps * i + caps)) for i in range(n)},
                                          {i: i for i in range(n)}, [""] * n)
        vals.append([m[f"{p}_R@{k}"] for p in ("T2I", "I2T", "I2T_Sym") for k in (1, 5, 10)])
    np.savez_compressed(os.path.join(HERE, "bootstrap.npz"), img=bf16_bits(img), all_txt=bf16_bits(all_txt),
                        samples=samples, metrics=np.array(vals, np.float64))
    print("bootstrap.npz:", np.array(vals).mean(0).round(2))


if __name__ == "__main__":
    torch.manual_seed(0)
    main = import_reference()
    from planted import E2E_H_MODELS
    only = sys.argv[1:]
    steps = {"preprocess": make_preprocess, "l2norm": lambda: make_l2norm(main),
             "retrieval": lambda: make_retrieval(main), "full_retrieval": lambda: make_full_retrieval(main),
             "maxsim": lambda: make_maxsim(main), "colpali_recall": lambda: make_colpali_recall(main),
             "encoders": lambda: make_encoders(main), "colpali": lambda: make_colpali(main),
             "config0": lambda: make_config0(main), "edge": lambda: make_edge(main),
             "winoground": make_winoground, "bootstrap": lambda: make_bootstrap(main),
             "colpali_full": lambda: make_colpali_full(main), "torch_topk": make_torch_topk,
             "dense_ties": lambda: make_dense_ties(main), "e2e": lambda: make_e2e(main),
             "e2e_h": lambda: make_e2e(main, E2E_H_MODELS, "e2e_fitted_h.npz")}
    for name, fn in steps.items():
        if not only or name in only:
            fn()
