"""oracle/torch_topk.cpp (torch.topk's CPU selection: libstdc++ partial_sort / nth_element, the
algorithm behind main.py:335,365,375's per-row torch.topk) against torch.topk's own outputs
(tests/golden/torch_topk.npz, written by tests/golden/make_goldens.py) and against the
reference's own top-10 of the configs[3]-geometry ColPali fixture."""
import numpy as np
import torch

from oracle import torch_topk as TT


def test_oracle_matches_torch_golden(golden):
    g = golden("torch_topk")
    for tag in g["cases"]:
        tag = str(tag)
        s = g[f"{tag}_s"].astype(np.float32) * np.float32(0.25)
        k = g[f"{tag}_idx"].shape[1]
        idx, val = TT.topk(s, k)
        assert np.array_equal(idx, g[f"{tag}_idx"]), tag
        assert np.array_equal(val, np.take_along_axis(s, idx, 1)), tag


def test_oracle_matches_live_torch_topk():
    """The same, live, on fresh tie-heavy rows (this container's torch.topk)."""
    rng = np.random.default_rng(5)
    for n in (3, 17, 64, 65, 129, 640, 641, 2000):
        for k in (1, 2, 5, 10, 16):
            if k > n:
                continue
            s = rng.integers(0, 4, (8, n)).astype(np.float32)
            ref = torch.topk(torch.from_numpy(s), k, dim=1).indices.numpy()
            assert np.array_equal(TT.topk(s, k)[0], ref), (n, k)


def test_oracle_reproduces_reference_colpali_ranking(golden):
    """Sampled whole score rows of colpali_full.npz (the reference's own scores): the oracle
    gives the reference's own torch.topk(row, 10) and hit flags."""
    g = golden("colpali_full")
    rows = g["sample_rows"]
    caps = int(g["params"][1])
    for p, (tag, tc) in enumerate((("t2i", 1), ("i2t", caps))):
        S = g[f"{tag}_rows"]
        idx, _ = TT.topk(S, 10)
        assert np.array_equal(idx, g[f"{tag}_idx"][rows])
        hh = np.stack([((TT.topk(S, k)[0] // tc) == rows[:, None]).any(1) for k in (1, 5, 10)], 1)
        assert np.array_equal(hh, g["hits"][p][rows])


def test_tie_order_is_not_column_order(golden):
    """Why the oracle exists: on bf16-quantised MaxSim rows torch.topk's tie order is not the
    column order (the reference's top-10 differs from a (score desc, column asc) sort on most rows)."""
    g = golden("colpali_full")
    assert (~g["lowest_index_rows"]).sum() > 1000
