"""Bootstrap resampling vs the reference's own resampled scoring +
compute_metrics_detailed (tests/golden/bootstrap.npz, seeded sample indices).

CPU: the oracle (full matrices + index gathers, every row ranked in torch.topk's own CPU
order -- oracle/torch_topk.cpp) gives the reference's per-iteration metrics exactly,
including the rows where a duplicated image ties its copy at the k-th place.
GPU: the device path (mme_gather_scores + mme_topk_rows_torch + mme_recall_hits_groups)
equals the oracle bit-exactly on the same score matrices, and so the reference."""
import numpy as np
import pytest
import torch

from helpers import bits_to_f32


def _tables(g):
    img = bits_to_f32(g["img"])
    allt = bits_to_f32(g["all_txt"])
    return img, allt[::5].copy(), allt


def test_oracle_vs_reference_bootstrap(golden):
    from oracle import bootstrap as ob
    g = golden("bootstrap")
    img, t2i, allt = _tables(g)
    n = img.shape[0]
    s_t2i = (torch.from_numpy(t2i) @ torch.from_numpy(img).T).numpy()
    s_i2t = (torch.from_numpy(img) @ torch.from_numpy(allt).T).numpy()
    ambiguous = 0
    for smp, ref in zip(g["samples"], g["metrics"]):
        hits, amb = ob.resample_hits(s_t2i, s_i2t, smp)
        assert np.array_equal(100.0 * hits / n, ref), (100.0 * hits / n, ref)
        ambiguous += int(amb.sum())
    # a duplicated top-1 image is tied with its copy in ~40 % of rows: a column-order rule
    # would have had to guess on these; torch.topk's own order settles every one of them
    assert ambiguous > 0


@pytest.mark.gpu
def test_device_bootstrap_equals_oracle(cuda, golden):
    from mme import bootstrap as mb
    from oracle import bootstrap as ob
    g = golden("bootstrap")
    img, t2i, allt = (torch.from_numpy(x).to("cuda", torch.bfloat16) for x in _tables(g))
    s_t2i, s_i2t = mb.full_scores(img, t2i, allt)
    samples = torch.from_numpy(g["samples"]).cuda()
    hits = mb.bootstrap_hits(s_t2i, s_i2t, samples, batch=7).cpu().numpy()
    a, b = s_t2i.cpu().numpy(), s_i2t.cpu().numpy()
    for it, smp in enumerate(g["samples"]):
        ref, _ = ob.resample_hits(a, b, smp)
        assert np.array_equal(hits[it], ref), it
    n = img.shape[0]
    row = mb.bootstrap_row(torch.from_numpy(hits), n)
    assert list(row)[:4] == ["T2I_R@1_mean", "T2I_R@1_lower", "T2I_R@1_upper", "T2I_R@1_std"]
    assert row["T2I_R@1_lower"] <= row["T2I_R@1_mean"] <= row["T2I_R@1_upper"]
    # and so the reference's own per-iteration values, exactly
    assert np.array_equal(100.0 * hits / n, g["metrics"])


@pytest.mark.gpu
def test_device_bootstrap_large(cuda):
    """n = 5 000, 40 resamples: the device path runs at the headline size (hits vs oracle on 2)."""
    from mme import bootstrap as mb
    from oracle import bootstrap as ob
    gen = torch.Generator(device="cuda").manual_seed(0)
    n, D = 5000, 256
    base = torch.randn(n, D, device="cuda", generator=gen)
    nrm = lambda x: (x / x.norm(dim=-1, keepdim=True)).to(torch.bfloat16)
    img = nrm(base + 1.5 * torch.randn(n, D, device="cuda", generator=gen))
    allt = nrm(base.repeat_interleave(5, 0) + 1.5 * torch.randn(5 * n, D, device="cuda", generator=gen))
    s_t2i, s_i2t = mb.full_scores(img, allt[::5].contiguous(), allt)
    samples = mb.sample_indices(n, 40, seed=1)
    hits = mb.bootstrap_hits(s_t2i, s_i2t, samples).cpu().numpy()
    a, b = s_t2i.cpu().numpy(), s_i2t.cpu().numpy()
    for it in (0, 39):
        ref, _ = ob.resample_hits(a, b, samples[it].cpu().numpy())
        assert np.array_equal(hits[it], ref), it


@pytest.mark.gpu
def test_harness_bootstrap_row(cuda, tmp_path):
    """run_benchmark(n_iterations>0) -> the reference's CSV row with bootstrap mean / CI / std."""
    from mme import get_spec
    from mme.harness import METRIC_KEYS, run_benchmark, write_csv
    from mme.models import SiglipModel
    from weights_gen import torch_state_dict
    spec = get_spec("tiny-siglip")
    model = SiglipModel.from_spec(spec, device="cuda", state_dict=torch_state_dict(spec, 0, torch.bfloat16))
    rng = np.random.default_rng(0)
    imgs = torch.from_numpy(rng.integers(0, 256, (12, 64, 64, 3), dtype=np.uint8)).cuda()
    ids = torch.from_numpy(np.concatenate([rng.integers(2, 1000, (60, 15)), np.ones((60, 1), np.int64)], 1)).cuda()
    row = run_benchmark(model, imgs, ids, n_iterations=20)
    cols = [f"{k}_{s}" for k in METRIC_KEYS for s in ("mean", "lower", "upper", "std")]
    assert list(row)[1:1 + len(cols)] == cols
    assert all(row[f"{k}_lower"] <= row[f"{k}_mean"] + 1e-9 <= row[f"{k}_upper"] + 2e-9 for k in METRIC_KEYS)
    write_csv([row], str(tmp_path / "r.csv"))
    assert (tmp_path / "r.csv").read_text().splitlines()[0].startswith(",Model,T2I_R@1_mean")
