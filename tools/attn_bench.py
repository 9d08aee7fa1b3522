#!/usr/bin/env python3
"""Attention microbenchmark on encoder shapes (HIP-event timed)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-embedding_amd"))
import torch  # noqa: E402
from mme import ops  # noqa: E402

CASES = [  # name, B, T, H, hd, causal
    ("siglip_vision", 256, 729, 16, 72, False),
    ("siglip_text", 1024, 64, 16, 72, False),
    ("clipL_vision", 256, 577, 16, 64, False),
    ("vitH_vision", 256, 257, 16, 80, False),
    ("clip_text_causal", 1024, 77, 16, 64, True),
]
for name, B, T, H, hd, causal in CASES:
    qkv = torch.randn(B * T, 3 * H * hd, device="cuda").to(torch.bfloat16)
    out = torch.empty(B * T, H * hd, device="cuda", dtype=torch.bfloat16)
    ops.attention(qkv, B, T, H, hd, causal=causal, out=out)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    it = 5
    s.record()
    for _ in range(it):
        ops.attention(qkv, B, T, H, hd, causal=causal, out=out)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / it
    fl = 4.0 * B * H * T * T * hd * (0.5 if causal else 1.0)
    print(f"{name:18s} B={B} T={T} H={H} hd={hd}: {ms:7.3f} ms {fl / ms / 1e9:7.1f} TFLOP/s", flush=True)
