#!/usr/bin/env python3
"""ColPali MaxSim benchmark at BASELINE config 4 (1 000 images x 5 000 captions):
T2I = 1 000 caption queries [26 tok] x 1 000 image docs [1030 tok],
I2T = 1 000 image queries [1030 tok] x 5 000 caption docs [26 tok], dim 128, bf16."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-embedding_amd"))
import torch  # noqa: E402
from mme import colpali  # noqa: E402

n_img, n_cap, Li, Lc = int(os.environ.get("N_IMG", 1000)), int(os.environ.get("N_CAP", 5000)), 1030, 26
g = torch.Generator(device="cuda").manual_seed(0)
img = torch.nn.functional.normalize(torch.randn(n_img, 1040, 128, device="cuda", generator=g), dim=-1).to(torch.bfloat16)
img[:, Li:] = 0
cap = torch.nn.functional.normalize(torch.randn(n_cap, 32, 128, device="cuda", generator=g), dim=-1).to(torch.bfloat16)
cap[:, Lc:] = 0
il = torch.full((n_img,), Li, dtype=torch.int32, device="cuda")
cl = torch.full((n_cap,), Lc, dtype=torch.int32, device="cuda")
t2i_q = cap[::5].contiguous()
t2i_ql = cl[::5].contiguous()
for name, Q, ql, D, dl in (("T2I", t2i_q, t2i_ql, img, il), ("I2T", img, il, cap, cl)):
    colpali.maxsim_scores(Q, ql, D, dl)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    out = colpali.maxsim_scores(Q, ql, D, dl)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e)
    fl = 2.0 * Q.shape[0] * D.shape[0] * int(ql[0]) * int(dl[0]) * 128
    print(f"MaxSim {name}: {Q.shape[0]}x{D.shape[0]} q_len {int(ql[0])} d_len {int(dl[0])}: {ms:.2f} ms, "
          f"{fl / ms / 1e9:.1f} TFLOP/s algorithmic", flush=True)
