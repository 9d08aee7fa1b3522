#!/usr/bin/env python3
"""Error of attention kernel forms against an fp32 (fp64-accumulated) reference on the SigLIP vision
geometry (hd 72, T 729): max / mean |diff| and the 99.99th percentile, per form. Needs MME_DEV=1 for
development kinds. Usage: attn_err.py --variants 0,113 [--batch 16] [--scale 1.5]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-embedding_amd"))
import torch  # noqa: E402
from mme import ops  # noqa: E402

VARIANTS = [int(v) for v in sys.argv[sys.argv.index("--variants") + 1].split(",")]
B = int(sys.argv[sys.argv.index("--batch") + 1]) if "--batch" in sys.argv else 16
SCALE = float(sys.argv[sys.argv.index("--scale") + 1]) if "--scale" in sys.argv else 1.5
T, H, HD = 729, 16, 72
g = torch.Generator(device="cuda").manual_seed(7)
qkv = (torch.randn(B * T, 3 * H * HD, device="cuda", generator=g) * SCALE).to(torch.bfloat16)
q, k, v = qkv.double().view(B, T, 3, H, HD).permute(2, 0, 3, 1, 4)
ref = (torch.softmax((q @ k.transpose(-1, -2)) * HD ** -0.5, -1) @ v).transpose(1, 2).reshape(B * T, H * HD)
for var in VARIANTS:
    with ops.kernel_forms(**({"attention": var} if var else {})):
        out = ops.attention(qkv, B, T, H, HD)
    torch.cuda.synchronize()
    d = (out.double() - ref).abs().flatten()
    q9 = torch.quantile(d[torch.randperm(d.numel(), device="cuda")[:1 << 22]], 0.9999).item()
    print(f"v{var} B={B} scale={SCALE}: max {d.max().item():.4g} mean {d.mean().item():.4g} p99.99 {q9:.4g}", flush=True)
