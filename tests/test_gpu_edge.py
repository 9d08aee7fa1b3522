"""Edge cases of the hot path on the MI355X against the reference (tests/golden/edge.npz,
dense_ties.npz): fewer candidates than k, ragged / tiny job sizes, empty inputs, exact score ties."""
import numpy as np
import pytest
import torch

from helpers import bits_to_bf16
from mme import encode, get_spec, ops, retrieval
from mme.models import SiglipModel
from mme.processor import Processor
from weights_gen import torch_state_dict

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n", [1, 2, 3, 7, 33])
def test_small_jobs_recall_equals_reference(cuda, golden, n):
    """n images < k = 10 (T2I and Sym rank n < 10 columns: k = min(k, ncols)), 5n captions."""
    g = golden("edge")
    img = bits_to_bf16(g[f"n{n}_img"]).cuda()
    allt = bits_to_bf16(g[f"n{n}_all_txt"]).cuda()
    got = retrieval.compute_metrics(img, allt[::5].contiguous(), allt)
    assert list(got.values()) == list(g[f"n{n}_metrics"])


def test_empty_inputs_match_reference(cuda, golden):
    """encode_data on empty image / caption lists returns torch.empty(0) (main.py:416,436) and never
    calls the model; one side empty leaves the other intact."""
    g = golden("edge")
    spec = get_spec("tiny-siglip")
    model = SiglipModel.from_spec(spec, device="cuda", state_dict=torch_state_dict(spec, 0, torch.bfloat16))
    ie, te = encode.encode_data(model, Processor(spec), spec.m_info, [], [])
    assert [list(ie.shape), list(te.shape)] == g["empty_shapes"].tolist()
    rng = np.random.default_rng(0)
    imgs = list(rng.integers(0, 256, (3, 64, 64, 3), dtype=np.uint8))
    ie, te = encode.encode_data(model, Processor(spec), spec.m_info, imgs, [])
    assert ie.shape == (3, spec.proj_dim) and te.numel() == 0
    _, te2 = encode.encode_data(model, Processor(spec), spec.m_info, [], [[5, 6, 7, 1]])
    assert te2.shape == (1, spec.proj_dim)
    # the fast paths take zero-row inputs too
    assert model.encode_texts(torch.zeros(0, 16, dtype=torch.int64, device="cuda")).shape == (0, spec.proj_dim)


def test_exact_ties_kernel_order_and_torch_order(cuda):
    """Duplicated documents give exactly equal scores. The fused kernels' own table is ordered (score
    desc, column asc) (mme_sim_topk, mme_topk_rows); the ranking the job uses (retrieval.rank_rows)
    flags exactly tied rows and re-selects them in torch.topk's CPU order, which must equal the
    oracle's torch-order selection (oracle/torch_topk.cpp, pinned to torch.topk itself)."""
    from oracle import retrieval as R
    g = torch.Generator().manual_seed(3)
    base = torch.nn.functional.normalize(torch.randn(40, 128, generator=g), dim=-1).to(torch.bfloat16)
    docs = base.repeat(3, 1)[torch.randperm(120, generator=g)]      # every document three times
    q = torch.nn.functional.normalize(torch.randn(25, 128, generator=g), dim=-1).to(torch.bfloat16)
    s = R.scores(q.float().numpy(), docs.float().numpy())
    idx, sc = ops.sim_topk(q.cuda(), docs.cuda(), 10)
    lidx, _ = R._lex_topk(s, 10)
    assert np.array_equal(idx.cpu().numpy(), lidx)
    idx2, _ = ops.topk_rows(torch.from_numpy(s).cuda(), 10)
    assert np.array_equal(idx2.cpu().numpy(), lidx)
    ranked = retrieval.rank_rows(q.cuda(), docs.cuda(), 3)
    tidx, _ = R.topk(s, 10)
    assert ranked.tie_rows.numel() == 25                            # every row's top 11 holds a tie
    assert np.array_equal(ranked.idx.cpu().numpy(), tidx)
    assert not np.array_equal(tidx, lidx)                           # torch's order is not column order here
    assert ranked.hits.tolist() == R.hits(s, 3).sum(0).tolist()


@pytest.mark.parametrize("nd", [3, 5, 7])
def test_exact_ties_fewer_columns_than_k(cuda, nd):
    """nd < 10 columns, every one an exact duplicate: k = min(k, nd) repeats (e.g. [1, 5, 5] at nd 5), so
    rank_rows must keep ONE torch-order selection per distinct k (tie_idx[k] lines up with tie_rows)
    while counting hits for every requested k; hits and order equal the oracle's torch.topk replay."""
    from oracle import retrieval as R
    g = torch.Generator().manual_seed(nd)
    doc = torch.nn.functional.normalize(torch.randn(1, 64, generator=g), dim=-1).to(torch.bfloat16)
    docs = doc.repeat(nd, 1)
    q = torch.nn.functional.normalize(torch.randn(6, 64, generator=g), dim=-1).to(torch.bfloat16)
    s = R.scores(q.float().numpy(), docs.float().numpy())
    ranked = retrieval.rank_rows(q.cuda(), docs.cuda(), 1)
    assert ranked.tie_rows.numel() == 6
    for k in {min(x, nd) for x in (1, 5, 10)}:
        assert ranked.tie_idx[k].shape == (ranked.tie_rows.numel(), k)
    tidx, _ = R.topk(s, nd)
    assert np.array_equal(ranked.idx.cpu().numpy(), tidx)
    assert ranked.hits.tolist() == R.hits(s, 1).sum(0).tolist()


def _device_hit_flags(ranked, tgt_count, n_cols, row_offset=0, ks=(1, 5, 10)):
    """[rows, len(ks)] bool from rank_rows' tables: rows without a tie from the torch-order top-10
    table, re-selected rows from their per-k selections."""
    idx = ranked.idx.cpu().numpy()
    rows = np.arange(idx.shape[0]) + row_offset
    out = np.stack([((idx[:, :min(k, n_cols)] // tgt_count) == rows[:, None]).any(1) for k in ks], 1)
    tie = ranked.tie_rows.cpu().numpy()
    for j, k in enumerate(ks):
        if tie.size:
            ik = ranked.tie_idx[min(k, n_cols)].cpu().numpy()
            out[tie, j] = ((ik // tgt_count) == rows[tie, None]).any(1)
    return out


@pytest.mark.parametrize("case", ["wide", "narrow", "tiny"])
def test_dense_exact_ties_vs_reference(cuda, golden, case):
    """Exact fp32 ties on the dense path, pinned to the reference (dense_ties.npz: duplicated images /
    captions scored by main.compute_similarity_scores, ranked by compute_metrics_detailed's per-k
    torch.topk calls; T2I / Sym at 1 000, 300 and 40 columns cover both of torch's branches). Device:
    every row's hit / miss at k = 1, 5, 10 and its top-10 IN torch.topk's ORDER identical to the
    reference's (fp32 near-ties between unequal scores excepted and counted), the 9 metrics identical."""
    from planted import bf16_sha, planted_ties
    from oracle import retrieval as R
    g = golden("dense_ties")
    n, caps, D, seed = (int(x) for x in g[case + "_params"])
    img_b, allt_b, _ = planted_ties(n, caps, D, float(g[case + "_noise"]), seed)
    assert bf16_sha(img_b) == str(g[case + "_img_sha"]) and bf16_sha(allt_b) == str(g[case + "_txt_sha"])
    img, allt = img_b.cuda(), allt_b.cuda()
    t2i = allt[::caps].contiguous()
    for p, (tag, q, d, tc) in enumerate((("t2i", t2i, img, 1), ("i2t", img, allt, caps), ("sym", img, t2i, 1))):
        ranked = retrieval.rank_rows(q, d, tc)
        same, near = R.compare_topk(ranked.idx.cpu().numpy(), g[f"{case}_{tag}_idx"], g[f"{case}_{tag}_score"])
        flags = _device_hit_flags(ranked, tc, d.shape[0])
        hit_same = (flags == g[case + "_hits"][p]).all(1)
        tied = g[case + "_tied"][p]
        dev_tied = np.zeros(n, bool)
        dev_tied[ranked.tie_rows.cpu().numpy()] = True
        print(f"{case} {tag}: {int(tied.sum())} reference rows with an exact tie in the top 11, "
              f"{int(dev_tied.sum())} re-ranked on the device; top-10 identical {int(same.sum())}/{n}, "
              f"hit rows identical {int(hit_same.sum())}/{n}, near-tie rows {int(near.sum())}")
        assert (same | near).all(), f"{tag}: top-10 differs on decisive rows {np.nonzero(~same & ~near)[0][:5]}"
        assert (hit_same | near).all(), f"{tag}: hit flags differ on rows {np.nonzero(~hit_same & ~near)[0][:5]}"
        assert ((dev_tied == tied) | near).all()
        assert tied.sum() > 0
    got = retrieval.compute_metrics(img, t2i, allt)
    assert list(got.values()) == list(g[case + "_metric_values"])


@pytest.mark.parametrize("D", [8, 96, 200])
def test_embedding_widths_off_the_tile_grid(cuda, D):
    """Embedding widths that are not multiples of the 64-deep K step (zero-padded on the host)."""
    from oracle import retrieval as R
    g = torch.Generator().manual_seed(D)
    q = torch.nn.functional.normalize(torch.randn(37, D, generator=g), dim=-1).to(torch.bfloat16)
    d = torch.nn.functional.normalize(torch.randn(301, D, generator=g), dim=-1).to(torch.bfloat16)
    idx, sc = ops.sim_topk(q.cuda(), d.cuda(), 10)
    ridx, rsc = R.topk(R.scores(q.float().numpy(), d.float().numpy()), 11)
    same, near = R.compare_topk(idx.cpu().numpy(), ridx, rsc)
    assert (same | near).all()
    s = retrieval.compute_similarity_scores(d.cuda(), q.cuda())
    torch.testing.assert_close(s.cpu(), q.float() @ d.float().T, atol=1e-5, rtol=1e-5)
