"""Encoder towers on the MI355X vs the reference's encode_data outputs.

Tiny configs (head dims 72 / 80 / 64, ragged captions, padded MLP widths) are
pinned by tests/golden/tiny-*.npz, produced by main.encode_data over the HF
modules (make_goldens.py). Full-size towers (random weights at the exact
architecture) are checked against the fp32 CPU oracle on a few inputs.
Tolerance: the oracle is fp32, the device path bf16 with fp32 accumulation —
per-row cosine >= 0.999 (SURVEY.md §8d parity criteria).
"""
import numpy as np
import pytest
import torch

from helpers import bits_to_f32, row_cos
from mme import encode, get_spec
from mme.models import CLIPModel, SiglipModel
from mme.processor import Processor
from weights_gen import torch_state_dict

pytestmark = pytest.mark.gpu

COS_MIN = 0.999


def _model(spec):
    sd = torch_state_dict(spec, 0, torch.bfloat16)
    cls = SiglipModel if spec.family == "siglip" else CLIPModel
    return cls.from_spec(spec, device="cuda", state_dict=sd)


def _inputs(g):
    caps = [g["ids"][i, :l].tolist() for i, l in enumerate(g["lens"])]
    return list(g["images"]), caps


@pytest.mark.parametrize("name", ["tiny-siglip", "tiny-clip"])
def test_encode_data_hf_surface(cuda, golden, name):
    """mme.encode.encode_data (main.py:386-438 restated) through the processor/model duck type."""
    spec = get_spec(name)
    g = golden(name)
    model, proc = _model(spec), Processor(spec)
    imgs, caps = _inputs(g)
    ie, te = encode.encode_data(model, proc, spec.m_info, imgs, caps)
    for got, key in ((ie, "img"), (te, "txt")):
        ref32 = torch.from_numpy(g[key + "_f32"])
        ref16 = torch.from_numpy(bits_to_f32(g[key + "_bf16"]))
        assert got.dtype == torch.bfloat16 and got.device.type == "cpu"
        assert row_cos(got, ref32).min() >= COS_MIN, f"{name} {key} vs fp32 reference"
        assert row_cos(got, ref16).min() >= COS_MIN, f"{name} {key} vs bf16 reference"
        assert (got.float() - ref32).abs().max() < 1.5e-2


@pytest.mark.parametrize("name", ["tiny-siglip", "tiny-clip"])
def test_fast_paths_match_surface(cuda, golden, name):
    """encode_images(u8) / encode_texts(ids, lens) == the HF-surface path (same kernels, fused preprocessing)."""
    spec = get_spec(name)
    g = golden(name)
    model, proc = _model(spec), Processor(spec)
    imgs, caps = _inputs(g)
    ie, te = encode.encode_data(model, proc, spec.m_info, imgs, caps)
    fi = model.encode_images(torch.from_numpy(g["images"]).cuda(), batch=2).cpu()
    ids = torch.from_numpy(g["ids"]).cuda()
    lens = torch.from_numpy(g["lens"])
    ft = model.encode_texts(ids, lens, ref_batch=spec.batch_size, exec_batch=3).cpu()
    assert torch.equal(fi, ie)
    assert torch.equal(ft, te)


def production_batches(spec, n_img: int = 5000, caps: int = 5):
    """The execution batches bench.py's 5k x 25k job runs (tail_aware_batch over 256 CUs of
    mme.config.exec_batches): SigLIP-400M 417 images / 5 000 captions."""
    from mme.config import exec_batches
    from mme.models import tail_aware_batch
    v = spec.vision
    T = v.num_patches + (0 if spec.family == "siglip" else 1)
    ib, tb = exec_batches(spec)
    return (tail_aware_batch(n_img, ib, T, v, 256),
            tail_aware_batch(caps * n_img, tb, spec.text.max_pos, spec.text, 256))


@pytest.mark.slow
@pytest.mark.parametrize("name,n_img,n_cap", [("SigLIP-400M", 2, 3), ("OpenAI-CLIP-L", 1, 2), ("LAION-CLIP-H", 1, 2),
                                              ("MetaCLIP-H14", 1, 2)])
def test_full_size_towers_vs_oracle(cuda, monkeypatch, name, n_img, n_cap):
    """Full-size towers (random weights at the exact architecture) vs the fp32 oracle, at two launch
    geometries: the items alone, and the same items at the first / last rows of ONE production
    execution batch (SigLIP: 417 images = 303 993 GEMM rows, 5 000 captions; the other rows are
    other synthetic inputs). Both must reach cos >= 0.999; the production-batch embeddings of
    the oracle items are compared with the small-batch ones (bit-identical or cos >= 0.9999:
    small shapes run the generic GEMM kernel, production shapes the pipelined one, so the fp32
    summation order may differ)."""
    from oracle import encoders as oracle_enc
    from mme.processor import synthetic_caption_ids, synthetic_images
    from mme.weights import random_state_dict
    spec = get_spec(name)
    sd = random_state_dict(spec, seed=0, device="cuda")
    cls = SiglipModel if spec.family == "siglip" else CLIPModel
    model = cls.from_spec(spec, device="cuda", state_dict=sd)
    imgs = synthetic_images(n_img)
    ids = synthetic_caption_ids(spec, n_cap)
    gi = model.encode_images(torch.from_numpy(imgs).cuda()).cpu()
    gt = model.encode_texts(torch.from_numpy(ids).cuda()).cpu()
    # production geometry: one execution batch of the bench's size, oracle items at both ends
    bi, bt = production_batches(spec)
    monkeypatch.setenv("MME_TAIL_AWARE_BATCH", "0")  # exactly one execution batch of bi / bt rows
    big_imgs = torch.from_numpy(synthetic_images(bi, seed=9)).cuda()
    img_pos = [0, bi - 1][:n_img] if n_img <= 2 else list(range(n_img))
    for p, j in zip(img_pos, range(n_img)):
        big_imgs[p] = torch.from_numpy(imgs[j])
    big_ids = torch.from_numpy(synthetic_caption_ids(spec, bt, seed=9)).cuda()
    cap_pos = [0, bt // 2, bt - 1][:n_cap]
    for p, j in zip(cap_pos, range(n_cap)):
        big_ids[p] = torch.from_numpy(ids[j])
    pi = model.encode_images(big_imgs, batch=bi)[img_pos].cpu()
    pt = model.encode_texts(big_ids, exec_batch=bt)[cap_pos].cpu()
    for small, prod, what in ((gi, pi, "images"), (gt, pt, "captions")):
        same = torch.equal(small, prod)
        print(f"{name} {what}: production batch ({bi if what == 'images' else bt}) bit-identical to the "
              f"small batch: {same}; cos {row_cos(small, prod).min().item():.6f}")
        assert same or row_cos(small, prod).min() >= 0.9999
    sd_cpu = {k: v.float().cpu() for k, v in sd.items()}
    del sd
    torch.set_num_threads(16)
    oi, ot = oracle_enc.encode_data(spec, sd_cpu, list(imgs), ids.tolist(), bs=n_img, out_dtype=torch.float32)
    for got in (gi, pi):
        assert row_cos(got, oi).min() >= COS_MIN
    for got in (gt, pt):
        assert row_cos(got, ot).min() >= COS_MIN


@pytest.mark.parametrize("name", ["tiny-siglip", "tiny-clip"])
def test_host_streamed_images_vs_reference(cuda, golden, name):
    """SURVEY §8f-2 pinned to the reference: u8 images in HOST memory, streamed H2D in batches of 2
    (pinned staging, side-stream copies) -> the reference's encode_data outputs (tiny-*.npz)."""
    spec = get_spec(name)
    g = golden(name)
    model = _model(spec)
    host = torch.from_numpy(np.ascontiguousarray(g["images"]))
    assert not host.is_cuda
    got = model.encode_images(host, batch=2).cpu()
    ref32 = torch.from_numpy(g["img_f32"])
    ref16 = torch.from_numpy(bits_to_f32(g["img_bf16"]))
    assert row_cos(got, ref32).min() >= COS_MIN and row_cos(got, ref16).min() >= COS_MIN
    assert (got.float() - ref32).abs().max() < 1.5e-2


def test_encode_images_from_host_memory(cuda, golden):
    """host-resident u8 images streamed H2D (double-buffered side-stream copies)
    give the same embeddings as device-resident ones."""
    spec = get_spec("tiny-siglip")
    model = _model(spec)
    rng = np.random.default_rng(3)
    imgs = torch.from_numpy(rng.integers(0, 256, (11, 80, 96, 3), dtype=np.uint8))
    dev = model.encode_images(imgs.cuda(), batch=4).cpu()
    host = model.encode_images(imgs, batch=4).cpu()
    assert torch.equal(dev, host)


@pytest.mark.slow
def test_fused_statistics_at_production_geometry(cuda, monkeypatch):
    """The residual-GEMM LayerNorm statistics (mme_gemm_res_stats: split grid, tail tiles, the stats
    hand-off between layers) against the separate mme_rowstats pass, at the bench's execution batches
    (SigLIP-400M: 417 images = 303 993 rows, 5 000 captions): same embeddings within fp32 summation
    noise (the statistics differ only in summation order)."""
    from mme import models
    from mme.processor import synthetic_caption_ids, synthetic_images
    from mme.weights import random_state_dict
    spec = get_spec("SigLIP-400M")
    model = SiglipModel.from_spec(spec, device="cuda", state_dict=random_state_dict(spec, seed=0, device="cuda"))
    bi, bt = production_batches(spec)
    monkeypatch.setenv("MME_TAIL_AWARE_BATCH", "0")
    imgs = torch.from_numpy(synthetic_images(bi, seed=4)).cuda()
    ids = torch.from_numpy(synthetic_caption_ids(spec, bt, seed=4)).cuda()
    out = {}
    for fused in (True, False):
        monkeypatch.setattr(models, "FUSED_STATS", fused)
        out[fused] = (model.encode_images(imgs, batch=bi).cpu(), model.encode_texts(ids, exec_batch=bt).cpu())
    for k, what in ((0, "images"), (1, "captions")):
        c = row_cos(out[True][k], out[False][k])
        print(f"{what}: fused vs separate statistics cos min {c.min().item():.6f}, "
              f"{torch.equal(out[True][k], out[False][k])=}")
        assert c.min() >= 0.9999


@pytest.mark.slow
@pytest.mark.parametrize("name", ["SigLIP-400M", "OpenAI-CLIP-L"])
def test_pruned_last_layer_at_production_geometry(cuda, monkeypatch, name):
    """The last encoder layer's row-wise half (o_proj, layer_norm2, MLP) on the pooled rows only
    (models.PRUNE_LAST: CLIP CLS / EOS rows, SigLIP text last token) against the same layer on
    every row, at the bench's execution batches: the pooled rows' arithmetic is unchanged, so the
    embeddings agree bit for bit where both forms run the same GEMM kernel (M·N >= 2^20 on both
    sides) and within fp32 summation noise where the pruned M drops to the generic kernel."""
    from mme import models
    from mme.processor import synthetic_caption_ids, synthetic_images
    from mme.weights import random_state_dict
    spec = get_spec(name)
    cls = SiglipModel if spec.family == "siglip" else CLIPModel
    model = cls.from_spec(spec, device="cuda", state_dict=random_state_dict(spec, seed=0, device="cuda"))
    bi, bt = production_batches(spec)
    monkeypatch.setenv("MME_TAIL_AWARE_BATCH", "0")
    imgs = torch.from_numpy(synthetic_images(bi, seed=5)).cuda()
    ids = torch.from_numpy(synthetic_caption_ids(spec, bt, seed=5)).cuda()
    out = {}
    for prune in (True, False):
        monkeypatch.setattr(models, "PRUNE_LAST", prune)
        out[prune] = (model.encode_images(imgs, batch=bi).cpu(), model.encode_texts(ids, exec_batch=bt).cpu())
    for k, what in ((0, "images"), (1, "captions")):
        same = torch.equal(out[True][k], out[False][k])
        c = row_cos(out[True][k], out[False][k])
        print(f"{name} {what}: pruned vs full last layer cos min {c.min().item():.7f}, bit-identical {same}")
        assert same or c.min() >= 0.99999
    # SigLIP's captions: o_proj / fc1 / fc2 at M = 5 000 run the same pipelined kernel as at 320 000 rows
    if spec.family == "siglip":
        assert torch.equal(out[True][1], out[False][1])


@pytest.mark.slow
def test_map_head_absorbed_at_production_geometry(cuda, monkeypatch):
    """SigLIP's MAP head with the probe query absorbed into the key projection (models.MAP_ABSORB:
    score GEMM x . [U_hi; U_lo]^T, mme_map_pool, W_v on the B*H pooled rows) against the K / V
    projection + mme_probe_attention form, at the bench's execution batch (417 images): the two
    differ only in where bf16 rounding falls (K / V rows vs the pooled rows)."""
    from mme import models
    from mme.processor import synthetic_images
    from mme.weights import random_state_dict
    spec = get_spec("SigLIP-400M")
    model = SiglipModel.from_spec(spec, device="cuda", state_dict=random_state_dict(spec, seed=0, device="cuda"))
    bi, _ = production_batches(spec)
    monkeypatch.setenv("MME_TAIL_AWARE_BATCH", "0")
    imgs = torch.from_numpy(synthetic_images(bi, seed=6)).cuda()
    out = {}
    for absorb in (True, False):
        monkeypatch.setattr(models, "MAP_ABSORB", absorb)
        out[absorb] = model.encode_images(imgs, batch=bi).cpu()
    c = row_cos(out[True], out[False])
    print(f"MAP head absorbed vs K / V projection: cos min {c.min().item():.7f} mean {c.mean().item():.7f}")
    assert c.min() >= 0.9999
