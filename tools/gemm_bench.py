#!/usr/bin/env python3
"""GEMM microbenchmark on the SigLIP-400M encoder shapes (HIP-event timed).

Usage: python tools/gemm_bench.py [--rows 186624] [--iters 10] [--variants V,..] [--mx --mx-variants F,..]
Prints per-shape ms and TFLOP/s; --variants / --mx-variants are per-call kernel forms
(ops.kernel_forms; dev-only forms need MME_DEV=1, i.e. libmme_dev.so).
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-embedding_amd"))
import torch  # noqa: E402
from mme import _lib, ops  # noqa: E402

DIAG_VARIANTS = {22, 23, 26, 27, 33, 34, 35, 36, 37, 38, 39, 52, 53, 65, 66, 67}  # diagnostic builds with deliberately wrong results
SHAPES = {  # name: (N, K)  with M = rows (SigLIP vision: 256 images x 729 tokens)
    "qkv": (3456, 1152), "o_proj": (1152, 1152), "fc1": (4352, 1152), "fc2": (1152, 4352),
    # DFN5B-H / ViT-H (d 1280, I 5120): rows 256 x 730
    "h_qkv": (3840, 1280), "h_fc1": (5120, 1280), "h_fc2": (1280, 5120),
}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rows", type=int, default=256 * 729)
    p.add_argument("--iters", type=int, default=10)
    p.add_argument("--variants", default="")
    p.add_argument("--shapes", default="qkv,o_proj,fc1,fc2")
    p.add_argument("--mx", action="store_true", help="also time the mx8 (block-scaled fp8) GEMM")
    p.add_argument("--mx-variants", default="-1", help="mx GEMM forms to time with --mx (-1 = production, "
                   "10 = mx10, 0 = round-2 form, 2 = per-wave epilogue alone, 3 = + scale wave; dev: 4, 9)")
    p.add_argument("--mx-epi", default="none", help="mx8 epilogue: none | job (the fp8 job's: QKV bias, fc1 "
                   "bias + quick_gelu to an mx8 output, fc2 bias + residual in place) | bias | quick (bias + "
                   "quick_gelu, bf16 out) | mx8 (bias, mx8 out): the parts of fc1's job epilogue")
    p.add_argument("--torch", action="store_true", help="also time torch F.linear (hipBLASLt) on each shape")
    p.add_argument("--epi", default="none", help="epilogue: none | bias | res (residual in place) | resstats (res + LayerNorm "
                   "statistics, mme_gemm_res_stats) | gelu (bias+gelu_tanh) | erf (bias+exact GELU) | quick (bias+quick_gelu)")
    a = p.parse_args()
    variants = [int(v) for v in a.variants.split(",")] if a.variants else [-1]
    g = torch.Generator(device="cuda").manual_seed(0)
    M = a.rows
    res = {}
    for name in a.shapes.split(","):
        N, K = SHAPES[name] if name in SHAPES else map(int, name.split(":"))  # "N:K" custom shape
        A = (torch.randn(M, K, device="cuda", generator=g)).to(torch.bfloat16)
        W = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).to(torch.bfloat16)
        C = torch.randn(M, N, device="cuda", generator=g).to(torch.bfloat16)
        bias = (torch.randn(N, device="cuda", generator=g) * 0.1).to(torch.bfloat16)
        R256 = C[:256].clone()  # "resper": residual rows r % 256 (an L2-resident residual table)
        kw = {"none": {}, "bias": {"bias": bias}, "res": {"bias": bias, "residual": C}, "resstats": {},
              "resper": {"bias": bias, "residual": R256, "res_period": 256},
              "gelu": {"bias": bias, "act": _lib.ACT_GELU_TANH}, "erf": {"bias": bias, "act": _lib.ACT_GELU_ERF},
              "quick": {"bias": bias, "act": _lib.ACT_QUICK_GELU}}[a.epi]
        st = torch.empty(M, 2, device="cuda")
        part = torch.empty(M, max(1, N // 64), 2, device="cuda")

        form = {"v": None}

        def run():
            with ops.kernel_forms(**({} if form["v"] is None else {"gemm": form["v"]})):
                if a.epi == "resstats":
                    ops.gemm_res_stats(A, W, bias, C, 1e-6, st, part, out=C)
                else:
                    ops.gemm(A, W, out=C, **kw)
        ref = None
        for v in variants:
            form["v"] = None if v == -1 else v  # -1 = production dispatch
            run()
            err = float("nan")
            if ref is None or a.epi in ("res", "resstats"):
                ref = C.clone()
            else:
                err = (C.float() - ref.float()).abs().max().item()
                if v not in DIAG_VARIANTS:
                    assert err < 0.05, f"variant {v} differs: {err}"
            for _ in range(3):  # warm the clocks / caches for this variant
                run()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ms = 1e30
            for rep in range(3):  # best of 3 timed groups
                s.record()
                for _ in range(a.iters):
                    run()
                e.record()
                torch.cuda.synchronize()
                ms = min(ms, s.elapsed_time(e) / a.iters)
            tf = 2.0 * M * N * K / ms / 1e9
            res[f"{name}/v{v}"] = {"ms": round(ms, 4), "tflops": round(tf, 1)}
            print(f"{name:7s} v{v:<2d} M={M} N={N} K={K} epi={a.epi}: {ms:8.3f} ms  {tf:7.1f} TFLOP/s  "
                  f"max|diff| vs first {err:.3g}", flush=True)
        if a.torch:  # vendor library baseline on the same operands (bias-free X @ W^T)
            Ct = torch.nn.functional.linear(A, W)
            err = (Ct.float() - ref.float()).abs().max().item() if (ref is not None and a.epi == "none") else 0.0
            for _ in range(3):
                torch.matmul(A, W.t(), out=Ct)
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ms = 1e30
            for rep in range(3):
                s.record()
                for _ in range(a.iters):
                    torch.matmul(A, W.t(), out=Ct)
                e.record()
                torch.cuda.synchronize()
                ms = min(ms, s.elapsed_time(e) / a.iters)
            tf = 2.0 * M * N * K / ms / 1e9
            res[f"{name}/torch"] = {"ms": round(ms, 4), "tflops": round(tf, 1)}
            print(f"{name:7s} torch M={M} N={N} K={K}: {ms:8.3f} ms  {tf:7.1f} TFLOP/s  (max |torch - mme| {err:.3g})",
                  flush=True)
            del Ct
        if a.mx:
            from mme import mx
            Aq, Wq = mx.quantize(A), mx.quantize(W)
            mkw, omx = {}, None
            if a.mx_epi == "job":
                mkw = {"bias": bias}
                if name.endswith("fc1"):
                    omx = mx.MXTensor.empty(M, N, "cuda")
                    mkw.update(act=_lib.ACT_QUICK_GELU, out_mx=omx)
                elif name.endswith("fc2"):
                    mkw.update(residual=C)
            elif a.mx_epi in ("bias", "quick", "mx8"):
                mkw = {"bias": bias}
                if a.mx_epi == "quick":
                    mkw.update(act=_lib.ACT_QUICK_GELU)
                if a.mx_epi == "mx8":
                    omx = mx.MXTensor.empty(M, N, "cuda")
                    mkw.update(out_mx=omx)
            if "out_mx" not in mkw:
                mkw["out"] = C
            first = None
            C0 = C.clone()  # the in-place residual's operand, restored before every variant's check
            r = torch.arange(M, device="cuda")
            srow = (r & ~127) | ((r & 31) << 2) | ((r >> 5) & 3)  # scale-plane position of row r (include/mme.h)

            def mrun(mv):
                with ops.kernel_forms(**({} if mv == -1 else {"mx": mv})):
                    return mx.gemm(Aq, Wq, **mkw)
            for mv in [int(v) for v in a.mx_variants.split(",")]:
                C.copy_(C0)
                Cm = mrun(mv)
                snap = (omx.q.clone(), omx.scales[:, srow].clone()) if omx is not None else (Cm.clone(),)
                if omx is None:
                    err = (Cm.float() - ref.float()).abs().max().item() if ref is not None and not a.mx_epi == "job" else 0.0
                else:
                    err = 0.0
                if first is None:
                    first = snap
                same = all(bool(torch.equal(x, y)) for x, y in zip(snap, first))
                for _ in range(3):
                    mrun(mv)
                torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                ms = 1e30
                for rep in range(3):  # best of 3 timed groups
                    s.record()
                    for _ in range(a.iters):
                        mrun(mv)
                    e.record()
                    torch.cuda.synchronize()
                    ms = min(ms, s.elapsed_time(e) / a.iters)
                tf = 2.0 * M * N * K / ms / 1e9
                res[f"{name}/mx{mv}"] = {"ms": round(ms, 4), "tflops": round(tf, 1)}
                print(f"{name:7s} mx8 v{mv:<2d} M={M} N={N} K={K}: {ms:8.3f} ms  {tf:7.1f} TFLOP/s  "
                      f"(max |mx - bf16| {err:.3g}, identical to first mx variant: {same})", flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
