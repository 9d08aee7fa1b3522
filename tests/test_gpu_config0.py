"""BASELINE configs[0] on the MI355X: OpenAI-CLIP-L (336 px, full architecture), 64 images x 320
captions, against the reference's own CPU path (tests/golden/config0_clip_l.npz: main.encode_data
at --batch-size 32, then compute_similarity_scores + compute_metrics_detailed; make_goldens.py).

Embeddings: per-row cosine >= 0.999 against the reference's fp32 run through the
drop-in surface (processor + get_*_features, mme.encode.encode_data) and the fast paths.
Retrieval: the reference's own embeddings ranked on the device must reproduce its top-10 order and
R@k (fp32 near-tie rule). The ranking of the device's OWN embeddings against the reference's chain is
tests/test_gpu_e2e.py: with these random weights every embedding clusters and no row's top-11 gap
exceeds the bf16 score noise (round 5's test here asserted on 0 decided rows), so that test fits the
towers' last linear maps onto graded targets at this same geometry (OpenAI-CLIP-L, 64 x 320) and
requires >= 80 % decided rows, all identical, and identical R@k."""
import numpy as np
import pytest
import torch

from helpers import bits_to_f32, row_cos
from planted import config0_inputs
from mme import encode, get_spec, ops
from mme.models import CLIPModel
from mme.processor import Processor
from weights_gen import torch_state_dict

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def clip_l(cuda):
    spec = get_spec("OpenAI-CLIP-L")
    model = CLIPModel.from_spec(spec, device="cuda", state_dict=torch_state_dict(spec, 0, torch.bfloat16))
    return spec, model


def test_config0_embeddings_vs_reference(clip_l, golden):
    spec, model = clip_l
    g = golden("config0_clip_l")
    imgs, rows = config0_inputs(spec)
    n, caps = imgs.shape[0], len(rows) // imgs.shape[0]
    ie, ae = encode.encode_data(model, Processor(spec), {"type": "dense", "batch_size": 32}, list(imgs), rows)
    _, te = encode.encode_data(model, Processor(spec), {"type": "dense", "batch_size": 32}, [], rows[::caps])
    for got, key in ((ie, "img"), (ae, "all"), (te, "t2i")):
        c32 = row_cos(got, torch.from_numpy(g[key + "_f32"]))
        c16 = row_cos(got, torch.from_numpy(bits_to_f32(g[key + "_bf16"])))
        print(f"{key}: cos vs reference fp32 min {c32.min():.5f}, vs reference bf16 min {c16.min():.5f}")
        assert c32.min() >= 0.999 and c16.min() >= 0.999
    # fast paths (u8 images resident, id tables + lengths) give the surface's bytes
    fi = model.encode_images(torch.from_numpy(imgs).cuda()).cpu()
    L = max(len(r) for r in rows)
    ids = torch.full((len(rows), L), spec.text.pad_id, dtype=torch.int64)
    for i, r in enumerate(rows):
        ids[i, : len(r)] = torch.tensor(r)
    lens = torch.tensor([len(r) for r in rows])
    fa = model.encode_texts(ids.cuda(), lens, ref_batch=32).cpu()
    assert row_cos(fi, ie).min() >= 0.9999 and row_cos(fa, ae).min() >= 0.9999


def test_config0_retrieval_vs_reference(cuda, golden):
    """The retrieval stage at configs[0] geometry: the reference's own bf16 embeddings ranked on the
    device (mme_sim_topk, recall counters) == its compute_similarity_scores + torch.topk (top-10 in
    order, fp32 near-tie rule of oracle.retrieval.compare_topk) and its compute_metrics_detailed."""
    from oracle import retrieval as R
    from mme import retrieval
    g = golden("config0_clip_l")
    emb = {k: torch.from_numpy(bits_to_f32(g[k + "_bf16"])).to(torch.bfloat16).cuda() for k in ("img", "all", "t2i")}
    for tag, qk, dk in (("t2i", "t2i", "img"), ("i2t", "img", "all"), ("sym", "img", "t2i")):
        idx, sc = ops.sim_topk(emb[qk], emb[dk], 10)
        same, near = R.compare_topk(idx.cpu().numpy(), g[tag + "_idx"], g[tag + "_score"])
        print(f"{tag}: {int(same.sum())}/{len(same)} rows identical, {int(near.sum())} fp32 near-tie rows")
        assert (same | near).all()
        assert np.abs(sc.cpu().numpy() - g[tag + "_score"][:, :10]).max() < 1e-5
    got = retrieval.compute_metrics(emb["img"], emb["t2i"], emb["all"])
    assert got == dict(zip([str(k) for k in g["metric_names"]], g["metric_values"]))
