"""Host-side logic of the mme package (no GPU): geometry, tokenization/padding,
text batch planning, ColPali chunk flags, harness CSV, model registry."""
import csv
import math

import numpy as np
import pytest
import torch

from mme import REGISTRY, TINY, get_spec
from mme.colpali import chunk_zero_flags
from mme.config import image_flops, text_flops
from mme.harness import METRIC_KEYS, write_csv
from mme.models import _gemm_tiles, _seq_lens, balanced, plan_text_batches, tail_aware_batch
from mme.processor import Processor, image_geometry, synthetic_caption_ids
from oracle import pil_bicubic


@pytest.mark.parametrize("H,W", [(224, 224), (150, 200), (300, 260), (480, 640), (640, 427)])
@pytest.mark.parametrize("name", ["SigLIP-400M", "OpenAI-CLIP-L", "LAION-CLIP-H", "Apple-DFN5B-H"])
def test_image_geometry_matches_oracle(name, H, W):
    ip = get_spec(name).image_proc
    assert image_geometry(H, W, ip) == pil_bicubic.geometry(H, W, ip.size, ip.mode)


def test_processor_text_padding_and_truncation():
    spec = get_spec("tiny-clip")
    proc = Processor(spec, device="cpu")
    bf = proc(text=["a photo of a cat", "dog"], padding=True, truncation=True)
    ids, mask = bf["input_ids"], bf["attention_mask"]
    assert ids.shape == mask.shape and ids.dtype == torch.int64
    assert ids[0, 0] == spec.text.bos_id and ids[0, int(mask[0].sum()) - 1] == spec.text.eos_id
    assert ids[1, int(mask[1].sum()):].eq(spec.text.pad_id).all()
    long = proc(text=[" ".join(["w"] * 100)])["input_ids"]
    assert long.shape[1] == spec.text.max_pos and long[0, -1] == spec.text.eos_id
    pre = proc(text=[[998, 5, 6, 999], [998, 999]])
    assert pre["input_ids"].tolist() == [[998, 5, 6, 999], [998, 999, 999, 999]]
    assert pre["attention_mask"].tolist() == [[1, 1, 1, 1], [1, 1, 0, 0]]


def test_seq_lens_requires_right_padding():
    m = torch.tensor([[1, 1, 0], [1, 1, 1]])
    assert _seq_lens(m, 2, 3, "cpu").tolist() == [2, 3]
    assert _seq_lens(torch.ones(2, 3, dtype=torch.int64), 2, 3, "cpu") is None
    with pytest.raises(ValueError):
        _seq_lens(torch.tensor([[0, 1, 1]]), 1, 3, "cpu")


def test_plan_text_batches_preserves_reference_padding():
    lens = [8, 2, 3, 1, 5, 5, 5, 5, 8, 1]
    plan = list(plan_text_batches(10, 8, lens, 4, 3))
    seen = sorted(i for _, rows in plan for i in rows)
    assert seen == list(range(10))
    # every caption runs at the padded length of ITS reference batch of 4
    for Lb, rows in plan:
        for i in rows:
            s = (i // 4) * 4
            assert Lb == max(lens[s:s + 4])
        assert len(rows) <= 3


def test_chunk_zero_flags():
    d = torch.tensor([30, 30, 20, 25, 25, 25, 10], dtype=torch.int32)
    assert chunk_zero_flags(d, 3).tolist() == [0, 0, 1, 0, 0, 0, 0]
    assert chunk_zero_flags(d, 10).tolist() == [0, 0, 1, 1, 1, 1, 1]


def test_write_csv_columns(tmp_path):
    row = {"Model": "x"}
    for k in METRIC_KEYS:
        for suf in ("_mean", "_lower", "_upper", "_std"):
            row[k + suf] = 1.0
    row.update({"Time": 1.0, "QPS": 2.0, "Encoding_Time": 0.5, "Img_per_sec": 4.0, "_failure_analysis": {}})
    p = tmp_path / "r.csv"
    write_csv([row], str(p))
    hdr = next(csv.reader(open(p)))
    # main.py:642-665 column order (pandas index column first)
    assert hdr[:2] == ["", "Model"] and hdr[2] == "T2I_R@1_mean" and hdr[-5:] == [
        "Time", "QPS", "Encoding_Time", "Img_per_sec", "_failure_analysis"]


def test_registry_flops_match_survey():
    # per-image GFLOP (vision tower) and per-caption GFLOP
    assert image_flops(REGISTRY["SigLIP-400M"]) / 1e9 == pytest.approx(670.3, rel=0.01)
    assert image_flops(REGISTRY["OpenAI-CLIP-L"]) / 1e9 == pytest.approx(381.9, rel=0.01)
    assert image_flops(REGISTRY["LAION-CLIP-H"]) / 1e9 == pytest.approx(334.6, rel=0.01)
    assert image_flops(REGISTRY["Apple-DFN5B-H"]) / 1e9 == pytest.approx(1007.0, rel=0.01)
    assert text_flops(REGISTRY["SigLIP-400M"], 64) / 1e9 == pytest.approx(53.13, rel=0.01)
    assert text_flops(REGISTRY["OpenAI-CLIP-L"], 77) / 1e9 == pytest.approx(13.30, rel=0.02)


def test_registry_param_counts_match_hf():
    # SURVEY.md §6 [probe]: SigLIP 878.0 M, CLIP-L-336 427.9 M, ViT-H 986.1 M, DFN5B-H 986.7 M
    from weights_gen import np_state_dict  # noqa: F401  (shape source shared with the goldens)
    from mme.weights import hf_param_shapes
    count = lambda n: sum(math.prod(s) for s in hf_param_shapes(get_spec(n)).values()) / 1e6
    assert count("SigLIP-400M") == pytest.approx(878.0, abs=0.6)
    assert count("OpenAI-CLIP-L") == pytest.approx(427.9, abs=0.6)
    assert count("LAION-CLIP-H") == pytest.approx(986.1, abs=0.6)
    assert count("Apple-DFN5B-H") == pytest.approx(986.7, abs=0.6)


def test_synthetic_captions_shape():
    s = get_spec("SigLIP-400M")
    ids = synthetic_caption_ids(s, 10)
    assert ids.shape == (10, 64) and (ids[:, -1] == s.text.eos_id).all() and ids[:, :-1].min() >= 2
    c = get_spec("OpenAI-CLIP-L")
    ids = synthetic_caption_ids(c, 10)
    assert ids.shape == (10, 77) and (ids[:, 0] == 49406).all() and (ids[:, -1] == 49407).all()


@pytest.mark.parametrize("name", ["tiny-siglip", "tiny-clip"])
def test_random_init_matches_hf_shapes(name):
    from mme.weights import hf_param_shapes, random_state_dict
    from weights_gen import np_state_dict
    spec = get_spec(name)
    shapes = hf_param_shapes(spec)
    sd = random_state_dict(spec, seed=0, device="cpu")
    assert {k: tuple(v.shape) for k, v in sd.items()} == shapes
    assert {k: v.shape for k, v in np_state_dict(spec).items()} == shapes


def test_layernorm_fold_algebra():
    """ops.LNFolded (mme_gemm_lnfold's weights): rstd * (x . w'^T - mean * cs) + b' equals
    LayerNorm(x) . w^T + b up to the bf16 rounding of w' = w * gamma (host-side check of the
    identity the GPU epilogue evaluates; the kernel itself is tested in test_gpu_kernels)."""
    from mme import ops
    g = torch.Generator().manual_seed(0)
    M, K, N = 64, 256, 96
    x = (torch.randn(M, K, generator=g) * 3 + 1.5).bfloat16().float()
    gamma = (1 + 0.2 * torch.randn(K, generator=g)).bfloat16()
    beta = (0.1 * torch.randn(K, generator=g)).bfloat16()
    w = (torch.randn(N, K, generator=g) / K ** 0.5).bfloat16()
    b = (0.1 * torch.randn(N, generator=g)).bfloat16()
    fold = ops.LNFolded(w, b, gamma, beta)
    mean = x.mean(dim=1, keepdim=True)
    rstd = torch.rsqrt(x.var(dim=1, unbiased=False, keepdim=True) + 1e-6)
    out = rstd * (x @ fold.w.float().T - mean * fold.cs) + fold.b
    ref = torch.nn.functional.layer_norm(x, (K,), gamma.float(), beta.float(), 1e-6) @ w.float().T + b.float()
    torch.testing.assert_close(out, ref, atol=2e-2, rtol=2e-2)
    assert fold.w.dtype == torch.bfloat16 and fold.cs.dtype == torch.float32 and fold.b.dtype == torch.float32


def test_gemm_tiles_matches_dispatch():
    # 256 x 256 tiles; N = 256 k + 128 -> the last 128 columns as 512 x 128 tiles (gemm.hip split grid)
    assert _gemm_tiles(256 * 10, 1024) == 40
    assert _gemm_tiles(256 * 10 + 1, 1024) == 44
    assert _gemm_tiles(256 * 10, 1152) == 40 + 5
    assert _gemm_tiles(256 * 9, 1152) == 36 + 5
    assert _gemm_tiles(256 * 4, 1100) == 4 * 5


@pytest.mark.parametrize("name", ["SigLIP-400M", "LAION-CLIP-H", "Apple-DFN5B-H", "OpenAI-CLIP-L"])
@pytest.mark.parametrize("n", [1, 7, 625, 1250, 5000, 25000])
def test_tail_aware_batch(name, n):
    spec = get_spec(name)
    for cfg, rows, batch in ((spec.vision, spec.vision.num_patches + 1, 256), (spec.text, spec.text.max_pos, 2048)):
        b = tail_aware_batch(n, batch, rows, cfg)
        assert 1 <= b <= batch
        nb = -(-n // b)
        assert -(-n // balanced(n, batch)) <= nb <= -(-n // batch) + 3  # equal split, at most 3 extra batches
        assert -(-n // nb) == b  # batches as equal as they can be
    assert tail_aware_batch(n, 256, 729, None) == balanced(n, 256)


def test_tail_aware_batch_siglip_shapes():
    spec = get_spec("SigLIP-400M")
    assert tail_aware_batch(5000, 256, 729, spec.vision) == 239  # o_proj / fc2: 12.0 waves of 256 tiles
    assert tail_aware_batch(25000, 2048, 64, spec.text) == 1563


def test_exec_batches_per_family():
    """bench.py's default execution batches (mme.config.exec_batches): the 8192-caption cap is SigLIP's
    only (profiles/r03_v28_*, r03_v29_*); the tail-aware split of the 5k x 25k job follows."""
    from mme.config import REGISTRY, exec_batches
    from mme.models import tail_aware_batch
    sig = REGISTRY["SigLIP-400M"]
    assert exec_batches(sig) == (512, 8192)
    assert tail_aware_batch(25000, 8192, sig.text.max_pos, sig.text) == 5000
    assert tail_aware_batch(5000, 512, sig.vision.num_patches, sig.vision) == 417
    for name in ("OpenAI-CLIP-L", "LAION-CLIP-H", "Apple-DFN5B-H"):
        assert exec_batches(REGISTRY[name]) == (512, 4096)


@pytest.mark.parametrize("n", [7711, 8192, 16384, 40000])
def test_exec_batch_keeps_gemm_operands_under_4gib(n):
    """A SigLIP caption batch whose fc2 operand ([rows, max(3d, I_pad)] bf16) would reach 4 GiB is split
    (pipe9 addresses operands with 32-bit offsets, so 8 192 captions at L = 64 would drop
    fc2 to the generic kernel); the vision towers' 512-image batches stay under it too."""
    from mme.config import REGISTRY, exec_batches
    sig = REGISTRY["SigLIP-400M"]
    t = sig.text
    widest = t.max_pos * max(3 * t.hidden, t.inter_pad) * 2
    b = tail_aware_batch(n, exec_batches(sig)[1], t.max_pos, t)
    assert b * widest < 1 << 32 and b <= 7710
    for name in ("SigLIP-400M", "LAION-CLIP-H", "Apple-DFN5B-H", "OpenAI-CLIP-L"):
        v = REGISTRY[name].vision
        rows = v.num_patches + 1
        bv = tail_aware_batch(5000, exec_batches(REGISTRY[name])[0], rows, v)
        assert bv * rows * max(3 * v.hidden, v.inter_pad) * 2 < 1 << 32
