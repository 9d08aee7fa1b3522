"""Edge cases of the hot path on the MI355X against the reference (tests/golden/edge.npz):
fewer candidates than k, ragged / tiny job sizes, empty inputs, exact score ties."""
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


def test_exact_ties_break_by_lowest_column(cuda):
    """Duplicated documents give exactly equal scores; the device order is (score desc, column asc),
    the rule oracle/retrieval.py states (torch.topk's CPU order on exact ties is implementation
    defined), for the fused sim/top-k and the row top-k of a score matrix alike."""
    from oracle import retrieval as R
    g = torch.Generator().manual_seed(3)
    base = torch.nn.functional.normalize(torch.randn(40, 128, generator=g), dim=-1).to(torch.bfloat16)
    docs = base.repeat(3, 1)[torch.randperm(120, generator=g)]      # every document three times
    q = torch.nn.functional.normalize(torch.randn(25, 128, generator=g), dim=-1).to(torch.bfloat16)
    idx, sc = ops.sim_topk(q.cuda(), docs.cuda(), 10)
    ridx, rsc = R.topk(R.scores(q.float().numpy(), docs.float().numpy()), 10)
    assert np.array_equal(idx.cpu().numpy(), ridx)
    s = (q.float() @ docs.float().T).cuda()
    idx2, _ = ops.topk_rows(s.contiguous(), 10)
    assert np.array_equal(idx2.cpu().numpy(), ridx)


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
