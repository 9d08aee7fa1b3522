#!/usr/bin/env python3
"""Dev: compare a GEMM variant against the production kernel on small shapes and
print where the outputs differ (row/col blocks)."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-embedding_amd"))
import torch  # noqa: E402
from mme import _lib, ops  # noqa: E402

lib = _lib.load()
lib.mme_gemm_variant.argtypes = [ctypes.c_int]
var = int(sys.argv[1]) if len(sys.argv) > 1 else 50
g = torch.Generator(device="cuda").manual_seed(0)
for (M, N, K) in [(256, 256, 64), (256, 256, 128), (256, 256, 256), (512, 512, 1152), (186624 // 8, 1152, 1152)]:
    A = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    W = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
    ref = (A.float() @ W.float().t())
    lib.mme_gemm_variant(var)
    C = ops.gemm(A, W)
    torch.cuda.synchronize()
    lib.mme_gemm_variant(-1)
    d = (C.float() - ref).abs()
    bad = d > 0.05
    print(f"M={M} N={N} K={K}: max err {d.max().item():.4f}, bad {bad.sum().item()} / {bad.numel()}", flush=True)
    if bad.any():
        t = bad[:256, :256].reshape(16, 16, 16, 16).any(dim=3).any(dim=1)  # 16x16 blocks of the first tile
        for r in range(16):
            print("   ", "".join("X" if t[r, c] else "." for c in range(16)))
        rows = bad.any(dim=1).nonzero().flatten()
        print("    bad rows (first tile mod 256):", sorted(set((rows % 256).tolist()))[:40])
