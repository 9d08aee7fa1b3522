"""The ColPali encoder oracle (oracle/colpali_encoder.py) against the reference's own
encode_data run over transformers' ColPaliForRetrieval (tests/golden/tiny-colpali.npz,
make_goldens.py make_colpali). CPU only."""
import numpy as np
import torch

from helpers import bits_to_f32, row_cos
from mme.config import COLPALI
from oracle import colpali_encoder as oc
from oracle import pil_bicubic
from weights_gen import torch_state_dict

SPEC = COLPALI["tiny-colpali"]


def left_pad(rows, pad):
    L = max(len(r) for r in rows)
    ids = torch.full((len(rows), L), pad, dtype=torch.int64)
    mask = torch.zeros((len(rows), L), dtype=torch.int64)
    for i, r in enumerate(rows):
        ids[i, L - len(r):] = torch.tensor(r)
        mask[i, L - len(r):] = 1
    return ids, mask


def oracle_encode(g, dtype):
    """encode_data's colpali branch (main.py:400-436) over the oracle, lists kept per item."""
    sd = torch_state_dict(SPEC, 0, dtype)
    ip = SPEC.image_proc
    bs = SPEC.batch_size
    imgs, caps = list(g["images"]), np.split(g["cap_ids"], np.cumsum(g["cap_lens"])[:-1])
    out_i, out_t = [], []
    for s in range(0, len(imgs), bs):
        chunk = imgs[s:s + bs]
        pv = torch.from_numpy(np.stack([pil_bicubic.normalize(pil_bicubic.preprocess_u8(a, ip.size, ip.mode),
                                                              ip.mean, ip.std) for a in chunk]))
        ids, mask = left_pad([list(SPEC.image_tokens)] * len(chunk), SPEC.pad_id)
        out_i += list(oc.forward(SPEC, sd, ids, mask, pv))
    for s in range(0, len(caps), bs):
        ids, mask = left_pad([list(SPEC.query_tokens(c)) for c in caps[s:s + bs]], SPEC.pad_id)
        out_t += list(oc.forward(SPEC, sd, ids, mask))
    return torch.cat(out_i), torch.cat(out_t)


def test_oracle_matches_reference_fp32(golden):
    g = golden("tiny-colpali")
    oi, ot = oracle_encode(g, torch.float32)
    assert oi.shape == g["img_f32"].shape and ot.shape == g["txt_f32"].shape
    np.testing.assert_allclose(oi.numpy(), g["img_f32"], atol=2e-5)
    np.testing.assert_allclose(ot.numpy(), g["txt_f32"], atol=2e-5)


def test_oracle_matches_reference_bf16(golden):
    g = golden("tiny-colpali")
    oi, ot = oracle_encode(g, torch.bfloat16)
    ri, rt = bits_to_f32(g["img_bf16"]), bits_to_f32(g["txt_bf16"])
    keep = np.abs(rt).sum(1) > 0  # zero (padding) rows
    assert np.array_equal(np.abs(ot.float().numpy()).sum(1) > 0, keep)
    assert row_cos(oi, ri).min() > 0.999
    assert row_cos(ot[keep], rt[keep]).min() > 0.999


def test_padding_rows_are_zero_and_left(golden):
    g = golden("tiny-colpali")
    rows = np.split(g["txt_f32"], np.cumsum(g["txt_rows"])[:-1])
    for r, L in zip(rows, g["cap_lens"]):
        n = len(SPEC.query_tokens([0] * int(L)))
        assert np.all(r[: len(r) - n] == 0) and np.all(np.abs(r[len(r) - n:]).sum(1) > 0)
