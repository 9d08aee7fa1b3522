"""ColPali MaxSim vs the reference's chunked processor.score (tests/golden/maxsim.npz)."""
import numpy as np
import pytest
import torch

from mme import colpali
from oracle import maxsim as oracle_maxsim

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("case", ["ragged", "fixed"])
def test_maxsim_matches_reference(cuda, golden, case):
    g = golden("maxsim")
    qs = oracle_maxsim.split(g[case + "_q"], g[case + "_qlen"])
    ds = oracle_maxsim.split(g[case + "_d"], g[case + "_dlen"])
    got = colpali.ColPaliScorer().score_chunked(qs, ds, chunk=10).cpu().numpy()
    ref = g[case + "_score"]
    # sums of bf16-rounded maxima, rounded to bf16: equal up to one bf16 ulp where
    # an fp32 accumulation-order difference flips a rounding
    ulp = np.abs(ref) * 2.0 ** -7 + 1e-6
    assert np.all(np.abs(got - ref) <= ulp)
    assert np.mean(got == ref) > 0.95


def test_maxsim_single_call_semantics(cuda, golden):
    g = golden("maxsim")
    qs = oracle_maxsim.split(g["ragged_q"], g["ragged_qlen"])[:10]
    ds = oracle_maxsim.split(g["ragged_d"], g["ragged_dlen"])[:10]
    got = colpali.ColPaliScorer().score(qs, ds).numpy()
    ref = oracle_maxsim.score_chunk(qs, ds).numpy()
    assert np.all(np.abs(got - ref) <= np.abs(ref) * 2.0 ** -7 + 1e-6)


def test_maxsim_ranks_vs_torch_fp32(cuda):
    gen = torch.Generator(device="cuda").manual_seed(1)
    Q = torch.nn.functional.normalize(torch.randn(40, 32, 128, device="cuda", generator=gen), dim=-1)
    D = torch.nn.functional.normalize(torch.randn(50, 1040, 128, device="cuda", generator=gen), dim=-1)
    ql = torch.full((40,), 26, dtype=torch.int32, device="cuda")
    dl = torch.full((50,), 1030, dtype=torch.int32, device="cuda")
    Qb, Db = Q.to(torch.bfloat16), D.to(torch.bfloat16)
    got = colpali.maxsim_scores(Qb, ql, Db, dl)
    s = torch.einsum("qnd,csd->qcns", Qb[:, :26].float(), Db[:, :1030].float()).max(-1).values
    ref = s.to(torch.bfloat16).float().sum(-1).to(torch.bfloat16).float()
    torch.testing.assert_close(got, ref, atol=0.05, rtol=2 ** -7)
