#!/usr/bin/env python3
"""LayerNorm / LayerNorm -> mx8 timing at the encoder geometries (HIP events, best of 3 x 10 launches):
algorithmic bytes (bf16 row in + gamma/beta + bf16 out, or + mx8 out with its scales) / time."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-embedding_amd"))
import torch  # noqa: E402
from mme import mx, ops  # noqa: E402

CASES = [("dfn5b_vision_417", 417 * 730, 1280), ("siglip_vision_417", 417 * 729, 1152), ("clip_text_4096", 4096 * 77, 1024)]
for name, rows, d in CASES:
    torch.manual_seed(0)
    x = torch.randn(rows, d, device="cuda").to(torch.bfloat16)
    g = torch.randn(d, device="cuda").to(torch.bfloat16)
    b = torch.randn(d, device="cuda").to(torch.bfloat16)
    out = mx.MXTensor.empty(rows, d, "cuda")
    for kind in ("bf16", "mx8"):
        run = (lambda: ops.layernorm(x, g, b, 1e-5)) if kind == "bf16" else (lambda: mx.layernorm(x, g, b, 1e-5, out))
        for _ in range(3):
            run()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ms = 1e30
        for _ in range(3):
            s.record()
            for _ in range(10):
                run()
            e.record()
            torch.cuda.synchronize()
            ms = min(ms, s.elapsed_time(e) / 10)
        byts = rows * d * 2 + (rows * d * 2 if kind == "bf16" else rows * d + rows * d // 32)
        print(f"{name:18s} {kind}: {ms * 1e3:8.1f} us  {byts / ms / 1e9:7.2f} TB/s", flush=True)
