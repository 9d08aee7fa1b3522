"""Fused similarity + top-k + recall vs the reference (tests/golden/retrieval.npz)."""
import numpy as np
import pytest
import torch

from helpers import bits_to_bf16
from mme import ops, retrieval

pytestmark = pytest.mark.gpu


def _emb(g):
    img = bits_to_bf16(g["img"]).cuda()
    allt = bits_to_bf16(g["all_txt"]).cuda()
    return img, allt[::5].contiguous(), allt


@pytest.mark.parametrize("tag", ["t2i", "i2t", "sym"])
def test_topk_indices_match_reference(cuda, golden, tag):
    g = golden("retrieval")
    img, t2i, allt = _emb(g)
    q, d = {"t2i": (t2i, img), "i2t": (img, allt), "sym": (img, t2i)}[tag]
    idx, sc = ops.sim_topk(q, d, 10)
    idx, sc = idx.cpu().numpy(), sc.cpu().numpy()
    # bf16 x bf16 products are exact in fp32; only the summation order differs from
    # the CPU matmul, so scores agree to ~1e-6 and indices must be identical.
    assert np.abs(sc - g[f"{tag}_score"]).max() < 1e-3
    assert np.array_equal(idx, g[f"{tag}_idx"])


def test_recall_metrics_identical(cuda, golden):
    g = golden("retrieval")
    img, t2i, allt = _emb(g)
    got = retrieval.compute_metrics(img, t2i, allt)
    ref = dict(zip([str(k) for k in g["metric_names"]], g["metric_values"]))
    assert got == ref


def test_similarity_matrix(cuda, golden):
    g = golden("retrieval")
    img, t2i, _ = _emb(g)
    s = retrieval.compute_similarity_scores(img, t2i)
    ref = t2i.float() @ img.float().T
    torch.testing.assert_close(s, ref, atol=1e-5, rtol=1e-5)


def test_topk_merge_and_offsets(cuda):
    gen = torch.Generator(device="cuda").manual_seed(4)
    q = torch.randn(300, 256, device="cuda", generator=gen).to(torch.bfloat16)
    d = torch.randn(3000, 256, device="cuda", generator=gen).to(torch.bfloat16)
    full_i, full_s = ops.sim_topk(q, d, 10)
    parts = [ops.sim_topk(q, d[i * 1000:(i + 1) * 1000], 10, col_offset=i * 1000) for i in range(3)]
    mi, ms = ops.topk_merge(torch.cat([p[0] for p in parts], 1), torch.cat([p[1] for p in parts], 1), 3, 10)
    assert torch.equal(mi, full_i)
    assert torch.equal(ms, full_s)


@pytest.mark.slow
def test_full_size_topk_vs_torch(cuda):
    """BASELINE size (5 000 x 25 000, D = 1152): indices vs a torch fp32 matmul + topk,
    checked on every row whose 10th/11th score margin exceeds the fp32 reordering noise."""
    gen = torch.Generator(device="cuda").manual_seed(0)
    n, D = 5000, 1152
    base = torch.randn(n, D, device="cuda", generator=gen)
    img = torch.nn.functional.normalize(base + 3 * torch.randn(n, D, device="cuda", generator=gen)).to(torch.bfloat16)
    cap = torch.nn.functional.normalize(base.repeat_interleave(5, 0) + 3 * torch.randn(5 * n, D, device="cuda",
                                                                                   generator=gen)).to(torch.bfloat16)
    idx, sc = ops.sim_topk(img, cap, 10)
    s = img.float() @ cap.float().T
    v, ix = torch.topk(s, 11, dim=1)
    ok = (v[:, 9] - v[:, 10]) > 1e-5
    assert ok.float().mean() > 0.95  # rows whose top-10 boundary is not an fp32-noise near-tie
    torch.testing.assert_close(sc, v[:, :10], atol=1e-4, rtol=0)
    # identical index SETS on rows with a clear top-10 boundary
    a = idx.sort(1).values[ok]
    b = ix[:, :10].int().sort(1).values[ok]
    assert torch.equal(a, b)
