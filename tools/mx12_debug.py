#!/usr/bin/env python3
"""mx12 vs mx11 on the mx8-output epilogue: where the outputs differ (tile rows / columns, q vs scales)."""
import math, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-embedding_amd")); sys.path.insert(0, ROOT)
import numpy as np, torch
from mme import mx, ops, _lib
from oracle import mx as omx
M, N, K = [int(v) for v in (sys.argv[1:4] if len(sys.argv) > 3 else (304410, 5120, 1280))]
act = int(sys.argv[4]) if len(sys.argv) > 4 else _lib.ACT_QUICK_GELU
g = torch.Generator(device="cuda").manual_seed(M + N + K)
a = mx.quantize((torch.randn(M, K, device="cuda", generator=g)).to(torch.bfloat16))
w = mx.quantize((torch.randn(N, K, device="cuda", generator=g) / math.sqrt(K)).to(torch.bfloat16))
bias = (0.1 * torch.randn(N, device="cuda", generator=g)).to(torch.bfloat16)
srow = torch.from_numpy(omx.srow(np.arange(M))).cuda()
nbm, nbn = (M + 255) // 256, (N + 255) // 256
ntiles = nbm * nbn
def xcd_remap(bid, nwg):
    x, loc, q, r = bid & 7, bid >> 3, nwg >> 3, nwg & 7
    return (x * (q + 1) if x < r else r * (q + 1) + (x - r) * q) + loc
def coords(tile, G=4):
    pg = G * nbn; gid = tile // pg; fm = gid * G; gsz = min(nbm - fm, G); r = tile % pg
    return fm + r % gsz, r // gsz
where = {}
for v in range(ntiles):
    where[coords(xcd_remap(v, ntiles))] = v
outs = []
FORMS = [int(f) for f in os.environ.get("MX12_FORMS", "12").split(",")]
for v in [11] + [f for f in FORMS for _ in range(3)]:
    o = mx.MXTensor.empty(M, N, "cuda")
    o.q.fill_(0x7f); o.scales.fill_(0x55)
    with ops.kernel_forms(mx=v):
        mx.gemm(a, w, bias, act=act, out_mx=o)
    torch.cuda.synchronize()
    outs.append((o.q[:M, :N].clone(), o.scales[:, srow].clone()))
for k in range(1, len(outs)):
    dq = (outs[0][0] != outs[k][0]); ds = (outs[0][1] != outs[k][1])
    print(f"run {k}: q differ {int(dq.sum())} of {dq.numel()}, scales differ {int(ds.sum())} of {ds.numel()}")
    if dq.any():
        r, c = dq.nonzero(as_tuple=True)
        print("  rows", r.min().item(), r.max().item(), "cols", c.min().item(), c.max().item(),
              "distinct row tiles", torch.unique(r // 256).numel(), "col tiles", torch.unique(c // 256).tolist()[:20])
        print("  rows mod 256 range", (r % 256).min().item(), (r % 256).max().item(), "cols mod 256", torch.unique((c % 256) // 64).tolist())
        tl = torch.unique((r // 256) * 1000 + (c // 256)).tolist()
        vs = sorted(where[(t // 1000, t % 1000)] for t in tl)
        print("  tiles (v, block, k):", [(v, v % 256, v // 256) for v in vs][:12])
        i = 0
        print("  first", r[i].item(), c[i].item(), outs[0][0][r[i], c[i]].item(), outs[k][0][r[i], c[i]].item())
    if ds.any():
        b, r = ds.nonzero(as_tuple=True)
        print("  scale blocks", torch.unique(b).tolist()[:20], "rows", r.min().item(), r.max().item())
print("forms", FORMS, "x3 each")
