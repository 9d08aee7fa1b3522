import os, sys
sys.path.insert(0, "multimodal-embedding_amd")
import torch
from mme import _lib, ops
g = torch.Generator(device="cuda").manual_seed(0)
for M in (300, 301, 513, 1000):
    N, K = 3456, 1152
    x = (torch.randn(M, K, device="cuda", generator=g) + 0.2).to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).to(torch.bfloat16)
    bias = (torch.randn(N, device="cuda", generator=g) * 0.1).to(torch.bfloat16)
    gam = (1 + 0.1 * torch.randn(K, device="cuda", generator=g)).to(torch.bfloat16)
    bet = (0.1 * torch.randn(K, device="cuda", generator=g)).to(torch.bfloat16)
    f = ops.LNFolded(w, bias, gam, bet)
    st = ops.rowstats(x, 1e-6, d=K)
    outs = []
    for rep in range(3):
        o = torch.full((M, N), float("nan"), dtype=torch.bfloat16, device="cuda")
        ops.gemm_lnfold(x, f, st, act=_lib.ACT_NONE, out=o)
        torch.cuda.synchronize()
        outs.append(o)
    nan = int(torch.isnan(outs[0]).sum())
    d01 = int((outs[0] != outs[1]).sum() - torch.isnan(outs[0]).sum())
    ref = ops.gemm_lnfold(x, f, st, act=_lib.ACT_NONE)
    print(f"M={M}: NaN (unwritten) {nan}, rep0 vs rep1 differing {d01}, rep1 vs rep2 {int((outs[1] != outs[2]).sum())}")
    if nan:
        idx = torch.isnan(outs[0]).nonzero()
        print("  first unwritten", idx[:6].tolist(), "rows", idx[:,0].unique()[:10].tolist(), "cols", idx[:,1].unique()[:10].tolist())
