#!/usr/bin/env python3
"""Dev: compare a GEMM variant against the fp32 product and against the production
kernel (bit-exact expected when only the tiling differs) on small / odd shapes,
for every epilogue; prints where the outputs differ."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-embedding_amd"))
import torch  # noqa: E402
from mme import _lib, ops  # noqa: E402

lib = _lib.load()
lib.mme_gemm_variant.argtypes = [ctypes.c_int]
var = int(sys.argv[1]) if len(sys.argv) > 1 else 50
g = torch.Generator(device="cuda").manual_seed(0)
fails = 0
for (M, N, K) in [(256, 256, 64), (1000, 1152, 1152), (700, 3456, 1152), (2304, 1152, 4352), (186624 // 8, 1152, 1152)]:
    A = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    W = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
    bias = (torch.randn(N, device="cuda", generator=g) * 0.1).bfloat16()
    R = torch.randn(M, N, device="cuda", generator=g).bfloat16()
    ref = (A.float() @ W.float().t())
    for epi, kw in [("none", {}), ("bias+gelu", {"bias": bias, "act": _lib.ACT_GELU_TANH}),
                    ("bias+res", {"bias": bias, "residual": R})]:
        lib.mme_gemm_variant(-1)
        C0 = ops.gemm(A, W, **kw)
        lib.mme_gemm_variant(var)
        C = ops.gemm(A, W, **kw)
        torch.cuda.synchronize()
        lib.mme_gemm_variant(-1)
        same = torch.equal(C, C0)
        msg = f"M={M} N={N} K={K} {epi:9s}: bit-identical to production: {same}"
        if epi == "none":
            d = (C.float() - ref).abs()
            msg += f", max err vs fp32 {d.max().item():.4f}"
        print(msg, flush=True)
        if not same:
            fails += 1
            bad = (C.float() - C0.float()).abs() > 0.05
            rows = bad.any(dim=1).nonzero().flatten()
            cols = bad.any(dim=0).nonzero().flatten()
            print("    bad rows", rows[:8].tolist(), "... n", len(rows), " bad cols", cols[:8].tolist(), "... n", len(cols))
print("FAILS", fails)
