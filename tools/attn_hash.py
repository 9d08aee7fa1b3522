#!/usr/bin/env python3
"""SHA-256 of ops.attention's output on seeded SigLIP-text-like inputs (B x 64 tokens, 16 heads x 72, with and
without a padding mask): run under two libraries (MME_LIB=...) to check that a kernel change is bit-identical."""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-embedding_amd"))
import torch  # noqa: E402
from mme import ops  # noqa: E402

g = torch.Generator(device="cuda").manual_seed(5)
h = hashlib.sha256()
for B, T, H, hd, lens in ((333, 64, 16, 72, None), (257, 64, 16, 72, "rand"), (3, 64, 3, 72, None)):
    qkv = (torch.randn(B * T, 3 * H * hd, device="cuda", generator=g) * 2).to(torch.bfloat16)
    sl = None if lens is None else torch.randint(1, T + 1, (B,), device="cuda", generator=g).to(torch.int32)
    o = ops.attention(qkv, B, T, H, hd, seq_lens=sl)
    torch.cuda.synchronize()
    h.update(o.view(torch.int16).cpu().numpy().tobytes())
print(os.path.basename(os.environ.get("MME_LIB", "libmme.so")), h.hexdigest())
