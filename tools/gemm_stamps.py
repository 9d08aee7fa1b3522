#!/usr/bin/env python3
"""Per-tile timeline of the production GEMM (dev variant 63: pipe6 with s_memrealtime stamps).

Each tile records [entry, main loop done, epilogue issued, epilogue stores retired] at 100 MHz.
Prints the phase durations and how many tiles are in their epilogue at the same time (are the
CUs' epilogues synchronised into HBM bursts?).

    python tools/gemm_stamps.py [--rows 174231] [--shape 1152:1152] [--epi res|bias]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-embedding_amd"))
import torch  # noqa: E402
from mme import _lib, ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=239 * 729)
    ap.add_argument("--shape", default="1152:1152")
    ap.add_argument("--epi", default="res")
    a = ap.parse_args()
    lib = _lib.load()
    lib.mme_gemm_variant.argtypes = [ctypes.c_int]
    lib.mme_gemm_debug_buffer.argtypes = [ctypes.c_void_p]
    N, K = map(int, a.shape.split(":"))
    M = a.rows
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).to(torch.bfloat16)
    b = (torch.randn(N, device="cuda", generator=g) * 0.1).to(torch.bfloat16)
    r = torch.randn(M, N, device="cuda", generator=g).to(torch.bfloat16)
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    dbg = torch.zeros(200000 * 4, dtype=torch.int64, device="cuda")
    assert lib.mme_gemm_debug_buffer(ctypes.c_void_p(dbg.data_ptr())) == 0
    lib.mme_gemm_variant(63)
    kw = {"residual": r} if a.epi == "res" else {}
    for _ in range(3):
        ops.gemm(x, w, b, out=out, **kw)
    torch.cuda.synchronize()
    dbg.zero_()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    ops.gemm(x, w, b, out=out, **kw)
    e.record()
    torch.cuda.synchronize()
    lib.mme_gemm_variant(-1)
    st = dbg.view(-1, 4).cpu().numpy().astype(np.float64)
    st = st[st[:, 0] > 0]
    t0 = st[:, 0].min()
    st = (st - t0) / 100.0  # us
    loop, epi, drain = st[:, 1] - st[:, 0], st[:, 2] - st[:, 1], st[:, 3] - st[:, 2]
    span = st[:, 3].max()
    res = {"shape": [M, N, K], "epi": a.epi, "tiles": int(len(st)), "kernel_ms": round(s.elapsed_time(e), 4),
           "span_us": round(span, 1),
           "loop_us": [round(float(np.percentile(loop, q)), 2) for q in (5, 50, 95)],
           "epi_issue_us": [round(float(np.percentile(epi, q)), 2) for q in (5, 50, 95)],
           "store_drain_us": [round(float(np.percentile(drain, q)), 2) for q in (5, 50, 95)]}
    # concurrency timeline: tiles in main loop / in epilogue per 1 us bin
    bins = np.arange(0, span + 1, 1.0)
    in_loop = [int(((st[:, 0] <= t) & (t < st[:, 1])).sum()) for t in bins]
    in_epi = [int(((st[:, 1] <= t) & (t < st[:, 3])).sum()) for t in bins]
    res["epilogue_share_of_tile_time"] = round(float((epi + drain).sum() / (st[:, 3] - st[:, 0]).sum()), 3)
    res["timeline_in_loop"] = in_loop[:120]
    res["timeline_in_epilogue"] = in_epi[:120]
    # wave-of-tiles alignment: start times of the first 256 tiles and of tiles 256..511
    order = np.argsort(st[:, 0])
    res["first_wave_start_spread_us"] = round(float(st[order[:256], 0].max() - st[order[:256], 0].min()), 2)
    res["second_wave_start_spread_us"] = round(float(st[order[256:512], 0].max() - st[order[256:512], 0].min()), 2)
    res["last_wave_start_spread_us"] = round(float(st[order[-256:], 0].max() - st[order[-256:], 0].min()), 2)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
