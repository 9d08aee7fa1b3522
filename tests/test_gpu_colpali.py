"""ColPali encoder on the MI355X: Gemma kernels vs fp32 references,
the tiny model vs the reference's encode_data outputs (tests/golden/tiny-colpali.npz),
fast paths vs the HF surface, and the full-size ColPali-v1.3 towers vs the CPU oracle.

Tolerances: kernels whose rounding steps are restated exactly (RMSNorm, RoPE,
embedding assembly, masked L2) are compared bit-exactly against a torch
restatement of the same bf16 ops, or within one bf16 ulp where fp32 reduction
order differs; MFMA paths (attention, GeGLU GEMM) against fp32 within bf16
output rounding; whole towers by per-token cosine >= 0.999.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from helpers import bits_to_f32, row_cos
from mme import ops
from mme._lib import ACT_GEGLU_TANH
from mme.colpali_encoder import ColPaliModel, ColPaliProcessor, interleave_gate_up
from mme.config import COLPALI
from weights_gen import torch_state_dict

pytestmark = pytest.mark.gpu
BF = torch.bfloat16
SPEC = COLPALI["tiny-colpali"]


def _ulps(a, b):
    ai = a.to(BF).view(torch.int16).int()
    bi = b.to(BF).view(torch.int16).int()
    return (ai - bi).abs().max().item()


def test_rmsnorm_matches_gemma_module(cuda):
    g = torch.Generator().manual_seed(0)
    x = (torch.randn(333, 2048, generator=g) * 3).to(BF)
    w = (torch.randn(2048, generator=g) * 0.3).to(BF)
    xf = x.float()
    ref = ((xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + 1e-6)) * (1.0 + w.float())).to(BF)
    got = ops.rmsnorm(x.cuda(), w.cuda(), 1e-6).cpu()
    assert _ulps(got, ref) <= 1


def test_rope_matches_oracle(cuda):
    from oracle.colpali_encoder import _rope
    g = torch.Generator().manual_seed(1)
    B, T, H, hd = 3, 77, 8, 256
    qkv = torch.randn(B * T, (H + 2) * hd, generator=g).to(BF)
    got = ops.rope_(qkv.clone().cuda(), T, H + 1, hd, 1, 10000.0).cpu()
    pos = torch.arange(T, dtype=torch.float) + 1
    x = qkv.view(B, T, H + 2, hd)[:, :, : H + 1].transpose(1, 2)  # [B, H+1, T, hd]
    ref = _rope(x, pos, 10000.0).transpose(1, 2).reshape(B * T, (H + 1) * hd)
    assert _ulps(got[:, : (H + 1) * hd], ref) <= 1
    frac = (got[:, : (H + 1) * hd].view(torch.int16) == ref.view(torch.int16)).float().mean().item()
    assert frac > 0.999
    assert torch.equal(got[:, (H + 1) * hd:], qkv[:, (H + 1) * hd:])  # V untouched


@pytest.mark.parametrize("B,T,Hq,left", [(2, 1030, 8, False), (3, 45, 8, True), (5, 33, 2, True), (1, 7, 4, False)])
def test_attention_mqa_vs_fp32(cuda, B, T, Hq, left):
    g = torch.Generator().manual_seed(T)
    hd = 256
    qkv = (torch.randn(B * T, (Hq + 2) * hd, generator=g) * 0.5).to(BF)
    lens = torch.randint(max(1, T // 3), T + 1, (B,), generator=g)
    lens[0] = T
    ks = (T - lens) if left else torch.zeros(B, dtype=torch.long)
    ke = ks + lens
    got = ops.attention_mqa(qkv.cuda(), B, T, Hq, hd, kstart=ks.int().cuda(), kend=ke.int().cuda()).cpu().float()
    x = qkv.float().view(B, T, Hq + 2, hd)
    q, k, v = x[:, :, :Hq].transpose(1, 2), x[:, :, Hq:Hq + 1].transpose(1, 2), x[:, :, Hq + 1:].transpose(1, 2)
    s = q @ k.transpose(-1, -2) * hd ** -0.5
    keys = torch.arange(T)
    valid = (keys[None, :] >= ks[:, None]) & (keys[None, :] < ke[:, None])
    s = s.masked_fill(~valid[:, None, None, :], float("-inf"))
    ref = (torch.softmax(s, -1) @ v).transpose(1, 2).reshape(B * T, Hq * hd)
    err = (got - ref).abs().max().item()
    assert err < 2e-2, err
    assert row_cos(got, ref).min() > 0.9995


def test_geglu_gemm_vs_fp32(cuda):
    g = torch.Generator().manual_seed(3)
    M, K, I = 700, 512, 1024
    a = (torch.randn(M, K, generator=g)).to(BF)
    gate = (torch.randn(I, K, generator=g) / K ** 0.5).to(BF)
    up = (torch.randn(I, K, generator=g) / K ** 0.5).to(BF)
    got = ops.gemm(a.cuda(), interleave_gate_up(gate, up).cuda(), act=ACT_GEGLU_TANH).cpu()
    assert got.shape == (M, I)
    gb = (a.float() @ gate.float().T).to(BF)
    ub = (a.float() @ up.float().T).to(BF)
    ref = (F.gelu(gb.float(), approximate="tanh").to(BF).float() * ub.float()).to(BF)
    # fp32 accumulation order may flip the bf16 rounding of gate / up (then propagated): allow
    # 2 bf16 ulps of the product, and require most outputs to be bit-identical
    err = (got.float() - ref.float()).abs()
    bound = 2 * 2.0 ** -7 * ref.float().abs() + 1e-3
    assert bool((err <= bound).all()), float((err - bound).max())
    assert (got.view(torch.int16) == ref.view(torch.int16)).float().mean().item() > 0.95


def test_gemma_embed_and_masked_l2(cuda):
    g = torch.Generator().manual_seed(4)
    B, L, P, d, V = 3, 20, 6, 512, 1000
    tok = torch.randn(V, d, generator=g).to(BF)
    ids = torch.randint(0, V, (B, L), generator=g)
    img = torch.randn(B * P, d, generator=g).to(BF)
    scale = float(torch.tensor(d ** 0.5).to(BF))
    got = ops.gemma_embed(ids.cuda(), tok.cuda(), scale, img=img.cuda(), img_prefix=P).cpu().view(B, L, d)
    ref = tok[ids] * torch.tensor(scale).to(BF)
    ref[:, :P] = img.view(B, P, d)
    assert torch.equal(got, ref)
    x = (torch.randn(B * L, 128, generator=g) * 2).to(BF)
    mask = torch.randint(0, 2, (B * L,), generator=g)
    y = ops.l2norm_masked(x.cuda(), mask.cuda()).cpu()
    ref = (x / x.norm(dim=-1, keepdim=True)) * mask[:, None]
    assert torch.equal(y.view(torch.int16), ref.view(torch.int16))


def _tiny_model():
    return ColPaliModel.from_spec(SPEC, device="cuda", state_dict=torch_state_dict(SPEC, 0, BF))


def _captions(g):
    return [c.tolist() for c in np.split(g["cap_ids"], np.cumsum(g["cap_lens"])[:-1])]


def test_tiny_colpali_vs_reference(cuda, golden):
    """mme.encode.encode_data's colpali branch over the processor / model duck type vs main.encode_data."""
    from mme import encode
    g = golden("tiny-colpali")
    model, proc = _tiny_model(), ColPaliProcessor(SPEC)
    ie, te = encode.encode_data(model, proc, SPEC.m_info, list(g["images"]), _captions(g))
    gi, gt = torch.cat(ie), torch.cat(te)
    assert [e.shape[0] for e in ie] == g["img_rows"].tolist() and [e.shape[0] for e in te] == g["txt_rows"].tolist()
    for got, key in ((gi, "img"), (gt, "txt")):
        r32 = torch.from_numpy(g[key + "_f32"])
        r16 = torch.from_numpy(bits_to_f32(g[key + "_bf16"]))
        keep = r32.abs().sum(1) > 0
        assert torch.equal(got.float().abs().sum(1) > 0, keep), f"{key}: zero (padding) rows differ"
        assert row_cos(got[keep], r32[keep]).min() >= 0.999, key
        assert row_cos(got[keep], r16[keep]).min() >= 0.999, key


def test_tiny_fast_paths_and_scores(cuda, golden):
    """encode_images(u8) / encode_queries(ids) == the HF surface rows; MaxSim over them vs the
    reference chunk loop on the reference's own embeddings (T2I)."""
    from mme import encode
    from mme.colpali import maxsim_scores, pack_multivectors
    g = golden("tiny-colpali")
    model, proc = _tiny_model(), ColPaliProcessor(SPEC)
    caps = _captions(g)
    ie, te = encode.encode_data(model, proc, SPEC.m_info, list(g["images"]), caps)
    fi = model.encode_images(torch.from_numpy(g["images"]).cuda(), batch=2).cpu()
    assert torch.equal(fi, torch.stack(ie))
    Q, ql, qpad = model.encode_queries(caps, exec_batch=2)
    for i, e in enumerate(te):
        n = int(ql[i])
        assert torch.equal(Q[i, :n].cpu(), e[e.shape[0] - n:]), i
    assert qpad.cpu().tolist() == g["txt_rows"].tolist()
    D, dl = pack_multivectors(list(fi), device="cuda")  # zero-padded to a multiple of 16 tokens
    s = maxsim_scores(Q, ql, D, dl, doc_chunk=10).cpu().numpy()
    ref = g["t2i_score"]
    assert np.abs(s - ref).max() <= 0.05 + 0.01 * np.abs(ref).max()
    assert np.array_equal(s.argmax(1), ref.argmax(1))


@pytest.mark.slow
def test_full_size_colpali_vs_oracle_at_production_geometry(cuda):
    """ColPali-v1.3 at full size (PaliGemma-3B) against the fp32 oracle (oracle/colpali_encoder.py,
    the transformers ColPaliForRetrieval port pinned to tiny-colpali.npz) at the bench's launch
    geometry: the first and last images of one 32-image execution batch, and the first and last
    queries of one query execution batch (each with its reference batch of 4 left-padded like
    process_queries, main.py:420-425). Per token: cosine >= 0.995 minimum, >= 0.999 mean."""
    from oracle import colpali_encoder as oc
    from mme.colpali_encoder import random_state_dict
    from mme.processor import synthetic_images
    import bench
    spec = COLPALI["ColPali-v1.3"]
    sd = random_state_dict(spec, seed=0, device="cuda")
    model = ColPaliModel.from_spec(spec, device="cuda", state_dict=sd)
    imgs = synthetic_images(32)
    caps = bench.colpali_captions(64, 1)
    gi = model.encode_images(torch.from_numpy(imgs).cuda(), batch=32).cpu()
    Q, ql, qpad = model.encode_queries(caps, exec_batch=64)
    Q, ql = Q.cpu(), ql.cpu()
    sd_cpu = {k: v.float().cpu() for k, v in sd.items()}
    del sd, model
    torch.cuda.empty_cache()
    torch.set_num_threads(16)
    cos = []
    for i in (0, 31):
        c = row_cos(gi[i], oc.encode_image(spec, sd_cpu, imgs[i]))
        print(f"image {i}: token cosine min {c.min().item():.5f} mean {c.mean().item():.6f}")
        cos.append(c)
    for i in (0, 63):
        lo = i // 4 * 4
        ref = oc.encode_query_batch(spec, sd_cpu, caps[lo:lo + 4])[i - lo]
        n = int(ql[i])
        assert ref.shape[0] == n
        c = row_cos(Q[i, :n], ref)
        print(f"query {i}: token cosine min {c.min().item():.5f} mean {c.mean().item():.6f}")
        cos.append(c)
    c = torch.cat(cos)
    assert c.min() >= 0.995 and c.mean() >= 0.999, (c.min().item(), c.mean().item())


def test_colpali_recall_vs_oracle(cuda):
    """Fast-path encode -> MaxSim (T2I, I2T incl. each caption doc's own left padding) ->
    device top-k -> hit counters, vs the reference chunk loop (oracle/maxsim.py) over the
    same per-item embedding lists (left-padded [L_b, 128] caption tensors, as encode_data
    returns them) and the oracle's top-k / recall."""
    from mme.colpali import colpali_recall, pack_multivectors
    from oracle import maxsim as om
    from oracle import torch_topk as TT
    rng = np.random.default_rng(5)
    n, caps = 6, 5
    model = _tiny_model()
    imgs = rng.integers(0, 256, (n, 64, 64, 3), dtype=np.uint8)
    all_caps = [rng.integers(3, 990, int(rng.integers(2, 12))).tolist() for _ in range(n * caps)]
    t2i_caps = all_caps[::caps]
    fi = model.encode_images(torch.from_numpy(imgs).cuda())
    D, dl = pack_multivectors(list(fi), device="cuda")
    Qt, qtl, _ = model.encode_queries(t2i_caps)
    Qa, qal, qap = model.encode_queries(all_caps)
    counts, sc = colpali_recall(D, dl, Qt, qtl, Qa, qal, qap, caps_per_image=caps)

    def items(Q, ql, qp):  # per-caption [L_b, 128] with its zero (left) padding rows, as the reference holds it
        out = []
        for i in range(Q.shape[0]):
            e = torch.zeros(int(qp[i]), 128, dtype=BF)
            e[int(qp[i]) - int(ql[i]):] = Q[i, : int(ql[i])].cpu()
            out.append(e)
        return out
    imgs_l = [e.cpu() for e in fi]
    t2i_l, all_l = items(Qt, qtl, model.encode_queries(t2i_caps)[2]), items(Qa, qal, qap)
    ref_t2i = om.score_reference_chunks(t2i_l, imgs_l).numpy()
    ref_i2t = om.score_reference_chunks(imgs_l, all_l).numpy()
    for got, ref in ((sc["t2i"].cpu().numpy(), ref_t2i), (sc["i2t"].cpu().numpy(), ref_i2t)):
        assert np.abs(got - ref).max() <= 2.0 ** -7 * np.abs(ref).max() + 1e-3
    ks = (1, 5, 10)
    for name, s, tc in (("T2I", sc["t2i"], 1), ("I2T", sc["i2t"], caps), ("I2T_Sym", sc["t2i"].t(), 1)):
        ref = TT.hits(s.cpu().numpy(), tc, ks).sum(0)  # torch.topk per row and k (main.py:331-378)
        assert [counts[f"{name}_R@{x}"] for x in ks] == [100.0 * r / n for r in ref], name


def test_colpali_recall_vs_reference_scores(cuda, golden):
    """ColPali recall pinned to the reference's OWN scores (tests/golden/colpali_recall.npz: 64 images
    x 1 030 planted doc tokens, 320 left-padded captions, scored by main.compute_similarity_scores'
    colpali chunk loop and ranked by compute_metrics_detailed's per-row torch.topk).

    Scores: device MaxSim vs the reference matrices, bit-identical (0 ulp: processor.score rounds
    every dot product to bf16, and the device reproduces the rounding and the summation order).
    Recall: the device ranks every row in torch.topk's CPU order (mme_topk_rows_torch: the
    reference's libstdc++ partial_sort / nth_element replayed, ties included), one selection per
    k as compute_metrics_detailed calls it, so every row's hit / miss equals the reference's own
    outcome -- no tie exemption."""
    from planted import bf16_sha, planted_multivec
    from mme.colpali import colpali_recall, pack_multivectors
    g = golden("colpali_recall")
    n, caps, Ld, q0, q1, seed = (int(x) for x in g["params"])
    img, cap, lens, pad = planted_multivec(n, caps, Ld, (q0, q1), float(g["noise"]), seed=seed)
    assert bf16_sha(img) == str(g["img_sha"]) and bf16_sha(cap) == str(g["cap_sha"])
    D, dl = pack_multivectors([img[i] for i in range(n)], device="cuda")
    Lq = -(-cap.shape[1] // 16) * 16
    Qa = torch.zeros(n * caps, Lq, 128, dtype=BF)
    Qa[:, : cap.shape[1]] = cap
    t2i_lens = lens[::caps].clone()
    counts, sc = colpali_recall(D, dl, Qa[::caps].contiguous().cuda(), t2i_lens.cuda(), Qa.cuda(), lens.cuda(),
                                pad.cuda(), caps_per_image=caps)
    got = {"t2i": sc["t2i"].cpu().numpy(), "i2t": sc["i2t"].cpu().numpy()}
    ref = {"t2i": g["t2i_score"], "i2t": g["i2t_score"]}
    for tag in ("t2i", "i2t"):
        a = torch.from_numpy(got[tag]).to(BF).view(torch.int16).int()
        b = torch.from_numpy(ref[tag]).to(BF).view(torch.int16).int()
        assert np.array_equal(torch.from_numpy(got[tag]).to(BF).float().numpy(), got[tag])  # bf16-quantised
        ulp = (a - b).abs()
        print(f"{tag}: {(ulp == 0).float().mean().item():.5f} of scores bit-identical, max {ulp.max().item()} ulp")
        assert ulp.max().item() == 0, f"{tag}: MaxSim scores differ from the reference's"
    ks = (1, 5, 10)
    protos = (("T2I", "t2i", False, 1), ("I2T", "i2t", False, caps), ("I2T_Sym", "t2i", True, 1))
    for p, (name, tag, transpose, tc) in enumerate(protos):
        s_dev = sc[tag].t().contiguous() if transpose else sc[tag]
        dev_rows = np.stack([(ops.topk_rows_torch(s_dev, min(k, s_dev.shape[1]))[0].cpu().numpy() // tc
                              == np.arange(n)[:, None]).any(1) for k in ks], 1)
        ref_rows = g["hits"][p]
        print(f"{name}: {int((dev_rows != ref_rows).any(1).sum())} rows differ from the reference's own outcome; "
              f"reference R@k {[round(100.0 * c / n, 2) for c in ref_rows.sum(0)]}, device "
              f"{[counts[f'{name}_R@{k}'] for k in ks]}")
        assert np.array_equal(dev_rows, ref_rows), f"{name}: rows {np.nonzero((dev_rows != ref_rows).any(1))[0]}"
        assert [counts[f"{name}_R@{k}"] for k in ks] == [100.0 * c / n for c in ref_rows.sum(0)]


@pytest.mark.slow
def test_colpali_full_geometry_vs_reference(cuda, golden):
    """BASELINE configs[3] at its full geometry (tests/golden/colpali_full.npz: 1 000 images x 1 030
    planted doc tokens, 5 000 captions of 23..29 tokens left-padded per batch of 4), pinned to the
    reference's own colpali chunk loop (main.py:451-470) and compute_metrics_detailed
    (main.py:305-383) with its per-row torch.topk:
      * scores: processor.score rounds every 128-term dot product to bf16; the CPU's bf16 GEMM and
        the MFMA sum those 128 products in different fp32 orders, so a dot product that lands on a
        bf16 rounding boundary can round the other way: on the sampled whole rows at most 1 bf16
        ulp apart and >= 99.9 % bit-identical;
      * every row whose top-11 score values are bit-identical to the reference's has the
        reference's torch.topk(row, 10) indices in torch's order (exact ties included:
        mme_topk_rows_torch replays torch's libstdc++ selection) and its hit / miss at k = 1, 5, 10;
        rows whose top-11 differ (by <= 1 ulp each) are the only exemption, and are counted;
      * Recall@{1,5,10} of all three protocols identical to the reference's."""
    from planted import bf16_sha, planted_multivec
    from mme.colpali import colpali_recall
    g = golden("colpali_full")
    n, caps, Ld, q0, q1, seed = (int(x) for x in g["params"])
    img, cap, lens, pad = planted_multivec(n, caps, Ld, (q0, q1), float(g["noise"]), seed=seed)
    assert bf16_sha(img) == str(g["img_sha"]) and bf16_sha(cap) == str(g["cap_sha"])
    Lp = -(-Ld // 16) * 16
    D = torch.zeros(n, Lp, 128, dtype=BF, device="cuda")
    D[:, :Ld] = img.cuda()
    dl = torch.full((n,), Ld, dtype=torch.int32, device="cuda")
    del img
    Lq = -(-cap.shape[1] // 16) * 16
    Qa = torch.zeros(n * caps, Lq, 128, dtype=BF, device="cuda")
    Qa[:, : cap.shape[1]] = cap.cuda()
    lens_d = lens.cuda()
    counts, sc = colpali_recall(D, dl, Qa[::caps].contiguous(), lens_d[::caps].contiguous(), Qa, lens_d,
                                pad.cuda(), caps_per_image=caps)
    got = {"t2i": sc["t2i"].cpu().numpy(), "i2t": sc["i2t"].cpu().numpy()}
    rows = g["sample_rows"]

    def ulps(x, y):
        a = torch.from_numpy(np.ascontiguousarray(x)).to(BF).view(torch.int16).int()
        b = torch.from_numpy(np.ascontiguousarray(y)).to(BF).view(torch.int16).int()
        return (a - b).abs().numpy()
    for tag in ("t2i", "i2t"):
        u = ulps(got[tag][rows], g[f"{tag}_rows"])
        print(f"{tag}: sampled rows, {int((u > 0).sum())} of {u.size} scores differ, max {int(u.max())} ulp")
        assert u.max() <= 1 and (u == 0).mean() >= 0.999, tag
    ks = (1, 5, 10)
    names = {"t2i": "T2I", "i2t": "I2T", "sym": "I2T_Sym"}
    for p, (tag, tc) in enumerate((("t2i", 1), ("i2t", caps), ("sym", 1))):
        s_dev = sc["t2i"].t().contiguous() if tag == "sym" else sc[tag]
        s = s_dev.cpu().numpy()
        sco = -np.sort(-s, 1)[:, :11]
        u11 = ulps(sco, g[f"{tag}_score"])
        same_sc = (u11 == 0).all(1)
        idx10 = ops.topk_rows_torch(s_dev, 10)[0].cpu().numpy()
        same_idx = (idx10 == g[f"{tag}_idx"]).all(1)
        dev_rows = np.stack([(ops.topk_rows_torch(s_dev, k)[0].cpu().numpy() // tc == np.arange(n)[:, None]).any(1)
                             for k in ks], 1)
        same_hits = (dev_rows == g["hits"][p]).all(1)
        name = names[tag]
        print(f"{name}: top-11 scores identical {int(same_sc.sum())}/{n} (others <= {int(u11.max())} ulp), top-10 "
              f"indices identical in torch's order {int(same_idx.sum())}/{n}, hit rows identical "
              f"{int(same_hits.sum())}/{n}; device R@k {[counts[f'{name}_R@{k}'] for k in ks]}")
        assert u11.max() <= 1, name
        assert (same_idx | ~same_sc).all() and (same_hits | ~same_sc).all(), name
        assert [counts[f"{name}_R@{k}"] for k in ks] == [100.0 * c / n for c in dev_rows.sum(0)]
    ref = dict(zip([str(k) for k in g["metric_names"]], g["metric_values"]))
    for k, v in ref.items():
        assert counts[k] == pytest.approx(v, abs=1e-9), k


def test_topk_rows_torch_vs_torch_golden(cuda, golden):
    """mme_topk_rows_torch against torch.topk's own outputs on tie-heavy rows (tests/golden/torch_topk.npz),
    on both sides of torch's partial_sort / nth_element switch; plus a column offset and a strided row."""
    g = golden("torch_topk")
    for tag in g["cases"]:
        tag = str(tag)
        s = torch.from_numpy(g[f"{tag}_s"].astype(np.float32) * np.float32(0.25)).cuda()
        ref = g[f"{tag}_idx"]
        k = ref.shape[1]
        idx, val = ops.topk_rows_torch(s, k)
        assert np.array_equal(idx.cpu().numpy(), ref), tag
        assert torch.equal(val, torch.gather(s, 1, idx.long())), tag
    wide = torch.zeros(5, 700, device="cuda")
    wide[:, :640] = torch.from_numpy(g["n640_k10_l5_s"][:5].astype(np.float32) * np.float32(0.25)).cuda()
    idx, _ = ops.topk_rows_torch(wide[:, :640], 10, col_offset=7)
    assert np.array_equal(idx.cpu().numpy() - 7, g["n640_k10_l5_idx"][:5])
