#!/usr/bin/env python3
"""Which hd-72 attention forms agree bit for bit (round-4 diagnostic of the last-tile skip).

Runs kinds 58 (attn_hyb_kernel, no skip), 62 (production: skip + literal-zero QK^T starts),
63 (round-2 skip form) and 70 (attn_pp_kernel: kind 62's arithmetic and skip in the ping-pong
structure) on the skip test's SigLIP case, prints the pairwise counts of differing outputs and,
for the first differing output, every form's value beside an fp64 reference of that (query, head).
Needs MME_DEV=1 (libmme_dev.so) for kinds 63 / 70.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-embedding_amd"))
import torch  # noqa: E402
from mme import ops  # noqa: E402

B, T, H, HD = 4, 729, 16, 72
KINDS = [58, 62, 63, 70] + ([76, 77] if "--trace" in sys.argv else [])
g = torch.Generator(device="cuda").manual_seed(B * T + HD)
qkv = (torch.randn(B * T, 3 * H * HD, device="cuda", generator=g) * 1.5).to(torch.bfloat16)
outs = {}
for k in KINDS:
    with ops.kernel_forms(attention=30 + k):
        outs[k] = ops.attention(qkv, B, T, H, HD)
    torch.cuda.synchronize()
for i, a in enumerate(KINDS):
    for b in KINDS[i + 1:]:
        d = (outs[a].float() - outs[b].float()).abs()
        print(f"kind {a} vs {b}: {int((d > 0).sum())} outputs differ, max {d.max().item():.3g}")
d = (outs[58].float() - outs[62].float()).abs()
nz = (d > 0).nonzero().tolist()
for row, col in nz[:3]:
    b, q, h = row // T, row % T, col // HD
    x = qkv[b * T:(b + 1) * T].double()
    Q, K, V = (x[:, j * H * HD + h * HD:j * H * HD + (h + 1) * HD] for j in range(3))
    s = (Q[q] @ K.T) / HD ** 0.5
    p = torch.softmax(s, 0)
    ref = (p @ V)[col % HD].item()
    vals = {k: outs[k][row, col].float().item() for k in KINDS}
    print(f"row {row} (batch {b}, query {q}) head {h} d {col % HD}: fp64 {ref:.6f}; " +
          ", ".join(f"kind {k} {v:.6f}" for k, v in vals.items()))

# race or hazard? the same kernels again while a GEMM stream competes for the CUs / memory: a
# timing race would move outputs, a deterministic codegen effect would not
if "--contend" in sys.argv:
    side = torch.cuda.Stream()
    A = torch.randn(16384, 8192, device="cuda", dtype=torch.bfloat16)
    for k in (58, 62):
        diffs = []
        for rep in range(4):
            torch.cuda.synchronize()
            with torch.cuda.stream(side):
                for _ in range(4):
                    A @ A.T[:, :4096]
            with ops.kernel_forms(attention=30 + k):
                o = ops.attention(qkv, B, T, H, HD)
            torch.cuda.synchronize()
            diffs.append(int((o != outs[k]).sum()))
        print(f"kind {k} under a concurrent GEMM stream, 4 runs: outputs differing from its solo run {diffs}")
