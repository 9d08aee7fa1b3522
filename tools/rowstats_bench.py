#!/usr/bin/env python3
"""Dev: HBM rate of mme_rowstats and mme_layernorm on the SigLIP residual stream."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-embedding_amd"))
import torch  # noqa: E402
from mme import ops  # noqa: E402

for rows in (256 * 729, 2048 * 64):
    x = torch.randn(rows, 1152, device="cuda").bfloat16()
    g = torch.ones(1152, device="cuda").bfloat16()
    st = torch.empty(rows, 2, device="cuda")
    h = torch.empty_like(x)
    for name, fn, nbytes in (("rowstats", lambda: ops.rowstats(x, 1e-6, out=st), x.numel() * 2),
                             ("layernorm", lambda: ops.layernorm(x, g, g, 1e-6, out=h), x.numel() * 4)):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(20):
            fn()
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / 20
        print(f"{name:9s} rows={rows}: {ms * 1e3:7.1f} us  {nbytes / ms / 1e9:6.2f} TB/s", flush=True)
