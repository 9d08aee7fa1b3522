#!/usr/bin/env python3
"""LayerNorm-folded GEMM microbenchmark (mme_gemm_lnfold) on the SigLIP-400M vision
shapes: QKV (no activation) and fc1 (gelu_tanh), M = 256 images x 729 tokens.
HIP-event timed, best of 3 groups. Select the library with MME_LIB to A/B two builds;
prints one JSON line with ms / TFLOP/s per shape and a checksum of the outputs.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-embedding_amd"))
import torch  # noqa: E402
from mme import _lib, ops  # noqa: E402

M, D = 256 * 729, 1152
SHAPES = {"qkv": (3456, _lib.ACT_NONE, 3456), "fc1": (4352, _lib.ACT_GELU_TANH, 4304)}


def main():
    g = torch.Generator(device="cuda").manual_seed(0)
    x = (torch.randn(M, D, device="cuda", generator=g) + 0.3).to(torch.bfloat16)
    st = ops.rowstats(x, 1e-6, d=D)
    res = {"lib": os.path.basename(_lib.LIB_PATH)}
    for name, (N, act, n_real) in SHAPES.items():
        w = (torch.randn(N, D, device="cuda", generator=g) / D ** 0.5).to(torch.bfloat16)
        b = (torch.randn(N, device="cuda", generator=g) * 0.1).to(torch.bfloat16)
        gam = (1 + 0.1 * torch.randn(D, device="cuda", generator=g)).to(torch.bfloat16)
        bet = (0.1 * torch.randn(D, device="cuda", generator=g)).to(torch.bfloat16)
        f = ops.LNFolded(w, b, gam, bet)
        out = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
        for _ in range(3):
            ops.gemm_lnfold(x, f, st, act=act, out=out)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        best = 1e30
        for _ in range(3):
            s.record()
            for _ in range(10):
                ops.gemm_lnfold(x, f, st, act=act, out=out)
            e.record()
            torch.cuda.synchronize()
            best = min(best, s.elapsed_time(e) / 10)
        fl = 2.0 * M * n_real * D
        res[name] = {"ms": round(best, 4), "tflops": round(fl / best / 1e9, 1),
                     "checksum": float(out.float().abs().sum().item())}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
