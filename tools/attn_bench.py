#!/usr/bin/env python3
"""Attention microbenchmark on encoder shapes (HIP-event timed)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-embedding_amd"))
import torch  # noqa: E402
from mme import ops  # noqa: E402

# --variants 0,F,...: per-call attention forms (ops.kernel_forms(attention=F)): 0 = production
# dispatch, 30 + kind = force kernel kind `kind` (dev kinds need MME_DEV=1: libmme_dev.so).
# --batch B overrides every case's batch (e.g. 417 = the SigLIP job's execution batch).
VARIANTS = [int(v) for v in sys.argv[sys.argv.index("--variants") + 1].split(",")] if "--variants" in sys.argv else [0]
BATCH = int(sys.argv[sys.argv.index("--batch") + 1]) if "--batch" in sys.argv else None
# --qs: Q pre-scaled by ops.attention_q_scale(hd), every call through mme_attention_qs (round 6: kinds
# 98-101 take their exp2 argument from the QK^T MFMA and exist on that entry only)
QS = "--qs" in sys.argv

CASES = [  # name, B, T, H, hd, causal
    ("siglip_vision", 256, 729, 16, 72, False),
    ("siglip_text", 1024, 64, 16, 72, False),
    ("siglip_text_pad", 1000, 64, 16, 72, False),
    ("siglip_text_2500", 2500, 64, 16, 72, False),
    ("clipL_vision", 256, 577, 16, 64, False),
    ("vitH_vision", 256, 257, 16, 80, False),
    ("vitH_256", 256, 256, 16, 80, False),  # ViT-H without the CLS row: whole 32-query waves
    ("dfn5b_vision", 128, 730, 16, 80, False),
    ("clip_text_causal", 1024, 77, 16, 64, True),
]
if "--cases" in sys.argv:
    _want = sys.argv[sys.argv.index("--cases") + 1].split(",")
    CASES = [c for c in CASES if c[0] in _want]
def run(v, *args, **kw):
    with ops.kernel_forms(**({"attention": v} if v else {})):
        return ops.attention(*args, q_prescaled=QS, **kw)


for (name, B, T, H, hd, causal), v in [(c, v) for c in CASES for v in VARIANTS]:
    B = BATCH or B
    torch.manual_seed(0)
    qkv = torch.randn(B * T, 3 * H * hd, device="cuda")
    if QS:
        qkv[:, : H * hd] *= ops.attention_q_scale(hd)
    qkv = qkv.to(torch.bfloat16)
    out = torch.empty(B * T, H * hd, device="cuda", dtype=torch.bfloat16)
    ref = run(0, qkv, B, T, H, hd, causal=causal)
    run(v, qkv, B, T, H, hd, causal=causal, out=out)
    torch.cuda.synchronize()
    err = (out.float() - ref.float()).abs().max().item()
    same = bool(torch.equal(out, ref))
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    it = 5
    for _ in range(3):  # warm the clocks / caches for this variant
        run(v, qkv, B, T, H, hd, causal=causal, out=out)
    ms = 1e30
    for rep in range(3):  # best of 3 timed groups
        s.record()
        for _ in range(it):
            run(v, qkv, B, T, H, hd, causal=causal, out=out)
        e.record()
        torch.cuda.synchronize()
        ms = min(ms, s.elapsed_time(e) / it)
    fl = 4.0 * B * H * T * T * hd * (0.5 if causal else 1.0)
    print(f"{name:18s} v{v} B={B} T={T} H={H} hd={hd}: {ms:7.3f} ms {fl / ms / 1e9:7.1f} TFLOP/s  maxdiff vs v0 {err:.3g} identical {same}", flush=True)
