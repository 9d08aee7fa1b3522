#!/usr/bin/env python3
"""Localise differences between the mx9 fp8 GEMM and the 64-deep half-line kernel.

For one shape, A is quantised with only one 32-wide K block non-zero at a time; for
each block the two kernels' bf16 outputs are compared and the wrong rows / columns
are summarised (tile row band, wave row, 32-row fragment; wave column, fragment).
Also runs the all-blocks case and a constant-scale case (every block amax equal).
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-embedding_amd"))
import torch  # noqa: E402
from mme import _lib, mx  # noqa: E402


def summary(d):
    rows = torch.nonzero(d.any(1)).flatten().tolist()
    cols = torch.nonzero(d.any(0)).flatten().tolist()
    if not rows:
        return "ok"
    f = lambda xs, m: sorted({x % m for x in xs})
    return (f"{int(d.sum())} wrong; rows {len(rows)} (first {rows[:6]}, row%256 wave rows {sorted({(r % 256) // 128 for r in rows})}, "
            f"r%32 {f(rows, 32)[:8]}); cols {len(cols)} (first {cols[:6]}, (c%256)//64 {sorted({(c % 256) // 64 for c in cols})}, "
            f"c%64//32 {sorted({(c % 64) // 32 for c in cols})})")


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--shape", default="256,256,256")
    a = p.parse_args()
    M, N, K = map(int, a.shape.split(","))
    lib = _lib.load()
    lib.mme_gemm_mx_variant.argtypes = [ctypes.c_int]
    g = torch.Generator(device="cuda").manual_seed(0)
    A = torch.randn(M, K, device="cuda", generator=g)
    W = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5)
    wq = mx.quantize(W.to(torch.bfloat16))

    def both(aq, wq_):
        lib.mme_gemm_mx_variant(0)
        old = mx.gemm(aq, wq_)
        lib.mme_gemm_mx_variant(-1)
        new = mx.gemm(aq, wq_)
        torch.cuda.synchronize()
        return old, new

    old, new = both(mx.quantize(A.to(torch.bfloat16)), wq)
    print("all blocks:", summary(old != new), "max|diff|", (old.float() - new.float()).abs().max().item(), flush=True)
    ones = torch.sign(A) + (A == 0).float()
    old, new = both(mx.quantize(ones.to(torch.bfloat16)), mx.quantize(torch.sign(W).to(torch.bfloat16)))
    print("constant scales (+-1):", summary(old != new), flush=True)
    for kb in range(min(K // 32, 12)):
        Ak = torch.zeros_like(A)
        Ak[:, kb * 32:(kb + 1) * 32] = A[:, kb * 32:(kb + 1) * 32]
        old, new = both(mx.quantize(Ak.to(torch.bfloat16)), wq)
        print(f"block {kb}: {summary(old != new)}  old|max| {old.float().abs().max().item():.3g} "
              f"new|max| {new.float().abs().max().item():.3g}", flush=True)


if __name__ == "__main__":
    main()
