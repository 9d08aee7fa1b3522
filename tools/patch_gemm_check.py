#!/usr/bin/env python3
"""Dev: time the SigLIP patch-embedding GEMM (K = 640 padded, position-table residual with
res_period = 729) against the same product without / with a full residual."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-embedding_amd"))
import torch  # noqa: E402
from mme import ops  # noqa: E402

M, N, K = 256 * 729, 1152, int(sys.argv[1]) if len(sys.argv) > 1 else 640
g = torch.Generator(device="cuda").manual_seed(0)
A = torch.randn(M, K, device="cuda", generator=g).bfloat16()
W = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
b = torch.randn(N, device="cuda", generator=g).bfloat16()
pos = torch.randn(729, N, device="cuda", generator=g).bfloat16()
R = torch.randn(M, N, device="cuda", generator=g).bfloat16()
C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
cases = {"plain": dict(), "bias": dict(bias=b), "bias+pos(period 729)": dict(bias=b, residual=pos, res_period=729),
         "bias+full residual": dict(bias=b, residual=R)}
for name, kw in cases.items():
    for _ in range(3):
        ops.gemm(A, W, out=C, **kw)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(10):
        ops.gemm(A, W, out=C, **kw)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / 10
    print(f"{name:24s} K={K}: {ms:.3f} ms  {2 * M * N * K / ms / 1e9:.1f} TF/s", flush=True)
