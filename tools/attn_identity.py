#!/usr/bin/env python3
"""SHA-256 of the production attention outputs on fixed seeded inputs (plain and Q-pre-scaled entries):
run once per library (MME_LIB=...) and compare the digests to show a change is bit-identical.

    python tools/attn_identity.py > a.txt; MME_LIB=old.so python tools/attn_identity.py > b.txt; diff a.txt b.txt
"""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-embedding_amd"))
import torch  # noqa: E402
from mme import ops  # noqa: E402

CASES = [  # B, T, H, hd, causal, lens
    (9, 729, 16, 72, False, None), (5, 730, 16, 80, False, None), (6, 257, 16, 80, False, None),
    (64, 77, 16, 64, True, None), (33, 77, 12, 64, True, "ragged"), (7, 577, 16, 64, False, None),
    (40, 64, 16, 72, False, "ragged"), (3, 200, 4, 72, True, None), (3, 300, 3, 64, True, "ragged"),
    (2, 1024, 16, 72, False, None), (4, 100, 5, 80, True, None),
]
for B, T, H, hd, causal, lens in CASES:
    g = torch.Generator(device="cuda").manual_seed(B * T + hd)
    qkv = (torch.randn(B * T, 3 * H * hd, device="cuda", generator=g) * 1.5).to(torch.bfloat16)
    sl = None
    if lens == "ragged":
        sl = torch.randint(1, T + 1, (B,), device="cuda", generator=g, dtype=torch.int32)
    for qs in (False, True):
        out = ops.attention(qkv, B, T, H, hd, seq_lens=sl, causal=causal, q_prescaled=qs)
        torch.cuda.synchronize()
        h = hashlib.sha256(out.view(torch.int16).cpu().numpy().tobytes()).hexdigest()[:24]
        print(f"B {B} T {T} H {H} hd {hd} causal {int(causal)} lens {lens} qs {int(qs)}: {h}", flush=True)
