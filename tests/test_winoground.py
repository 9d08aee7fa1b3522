"""Winoground 2x2 scorer vs the reference's own run_winoground
(tests/golden/winoground.npz: run_benchmark_grand_slam_v28_publication_ready.py:413-461
over the tiny models with load_dataset patched to synthetic examples, plus the
per-example 2x2 scores of the same modules).

The decision rule is exact; the embeddings are bf16 unit vectors whose rounding
differs between implementations (|delta s| up to ~1.5e-3 observed), so a comparison
whose two reference scores lie within 3e-3 + 2^-7 |s| (a near-tie: the tiny random
models score everything near 0) may flip. Every DECISIVE comparison must match, and the metrics
must equal the reference's up to the near-tie examples.
CPU: the oracle (bf16 encoders + decision rule). GPU: the device path (batched
encode + mme_winoground)."""
import numpy as np
import pytest
import torch

from mme import get_spec

NAMES = ["tiny-siglip", "tiny-clip"]
PAIRS = {"text": ((0, 1), (3, 2)), "image": ((0, 2), (3, 1))}  # a > b comparisons on s00,s01,s10,s11


def _examples(g, key):
    imgs = g[f"{key}_images"]
    caps = np.split(g[f"{key}_cap_ids"], np.cumsum(g[f"{key}_cap_lens"])[:-1])
    return [{"image_0": imgs[i, 0], "image_1": imgs[i, 1], "caption_0": caps[2 * i].tolist(),
             "caption_1": caps[2 * i + 1].tolist()} for i in range(imgs.shape[0])]


def _check(got_scores, g, key):
    ref = g[f"{key}_scores"]
    got = np.asarray(got_scores, np.float32).reshape(-1, 4)
    near = np.zeros(len(ref), bool)
    for kind, pairs in PAIRS.items():
        for a, b in pairs:
            tol = 2.0 ** -7 * np.maximum(np.abs(ref[:, a]), np.abs(ref[:, b])) + 3e-3
            decisive = np.abs(ref[:, a] - ref[:, b]) > tol
            near |= ~decisive
            assert np.array_equal((got[:, a] > got[:, b])[decisive], (ref[:, a] > ref[:, b])[decisive]), (kind, a, b)
    from oracle import winoground as ow
    m, r = ow.metrics(got), g[f"{key}_metrics"]
    slack = 100.0 * near.sum() / len(ref)
    for j, k in enumerate(("Wino Text", "Wino Image", "Wino Group")):
        assert abs(m[k] - r[j]) <= slack + 1e-9, (k, m[k], r[j], slack)
    return m


@pytest.mark.parametrize("name", NAMES)
def test_golden_scores_reproduce_reference_metrics(golden, name):
    from oracle import winoground as ow
    g = golden("winoground")
    key = name.replace("-", "_")
    m = ow.metrics(g[f"{key}_scores"])
    assert [m["Wino Text"], m["Wino Image"], m["Wino Group"]] == g[f"{key}_metrics"].tolist()


@pytest.mark.parametrize("name", NAMES)
def test_oracle_vs_reference(golden, name):
    from oracle import encoders as oe
    from oracle import winoground as ow
    from weights_gen import torch_state_dict
    g = golden("winoground")
    key = name.replace("-", "_")
    spec = get_spec(name)
    exs = _examples(g, key)
    sd = torch_state_dict(spec, 0, torch.bfloat16)
    ie, te = oe.encode_data(spec, sd, [ex[f"image_{j}"] for ex in exs for j in (0, 1)],
                            [ex[f"caption_{j}"] for ex in exs for j in (0, 1)], bs=2)
    _check([ow.scores(te[2 * i:2 * i + 2], ie[2 * i:2 * i + 2]).numpy() for i in range(len(exs))], g, key)


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_device_winoground_vs_reference(cuda, golden, name):
    from mme.models import CLIPModel, SiglipModel
    from mme.processor import Processor
    from mme.winoground import run_winoground, winoground_scores
    from oracle import winoground as ow
    from weights_gen import torch_state_dict
    g = golden("winoground")
    key = name.replace("-", "_")
    spec = get_spec(name)
    cls = SiglipModel if spec.family == "siglip" else CLIPModel
    model = cls.from_spec(spec, device="cuda", state_dict=torch_state_dict(spec, 0, torch.bfloat16))
    proc = Processor(spec)
    exs = _examples(g, key)
    scores, counts = winoground_scores(model, proc, exs)
    m = _check(scores.cpu().numpy(), g, key)
    assert run_winoground(model, proc, spec.m_info, exs) == m  # the kernel's counters == the rule on its scores
    c = counts.cpu().tolist()
    assert [100.0 * x / len(exs) for x in c] == [m["Wino Text"], m["Wino Image"], m["Wino Group"]]
