"""Numerics of the libmme kernels against plain PyTorch fp32 references (MI355X)."""
import math

import numpy as np
import pytest
import torch

from helpers import bf16_bits, bits_to_bf16

pytestmark = pytest.mark.gpu

from mme import _lib, ops  # noqa: E402


def act_ref(y, act):
    if act == _lib.ACT_GELU_TANH:
        return torch.nn.functional.gelu(y, approximate="tanh")
    if act == _lib.ACT_QUICK_GELU:
        return y * torch.sigmoid(1.702 * y)
    if act == _lib.ACT_GELU_ERF:
        return torch.nn.functional.gelu(y)
    return y


def rnd(*shape, scale=1.0, gen=None, device="cuda"):
    return (torch.randn(*shape, generator=gen, device=device) * scale).to(torch.bfloat16)


@pytest.mark.parametrize("M,N,K", [(1, 128, 64), (100, 200, 128), (1458, 1152, 1152), (300, 64, 640),
                                   (4096, 4352, 1152), (2048, 3456, 1152), (517, 1152, 4352), (33, 8, 64),
                                   # pipelined-kernel stage-count edge cases (nk = K/32 = 2, 4, 6, 10)
                                   (2048, 1024, 64), (2048, 1024, 128), (1500, 1024, 192), (2048, 1536, 320)])
@pytest.mark.parametrize("act", [0, 1, 2, 3])
def test_gemm_bias_act(cuda, M, N, K, act):
    g = torch.Generator(device="cuda").manual_seed(M * 7 + N + act)
    a = rnd(M, K, gen=g)
    w = rnd(N, K, scale=1 / math.sqrt(K), gen=g)
    b = rnd(N, scale=0.1, gen=g)
    out = ops.gemm(a, w, b, act=act)
    ref = act_ref(a.float() @ w.float().T + b.float(), act)
    torch.testing.assert_close(out.float(), ref, atol=2e-2, rtol=1e-2)


@pytest.mark.parametrize("period", [0, 49, 729])
def test_gemm_residual_period_inplace(cuda, period):
    g = torch.Generator(device="cuda").manual_seed(period + 1)
    M, N, K = 729 * 3, 1152, 640
    a = rnd(M, K, gen=g)
    w = rnd(N, K, scale=1 / math.sqrt(K), gen=g)
    if period:
        res = rnd(period, N, gen=g)
        rows = torch.arange(M, device="cuda") % period
        ref = a.float() @ w.float().T + res.float()[rows]
        out = ops.gemm(a, w, residual=res, res_period=period)
    else:
        x = rnd(M, N, gen=g)
        ref = a.float() @ w.float().T + x.float()
        out = ops.gemm(a, w, residual=x, out=x)  # in place on the residual stream
        assert out.data_ptr() == x.data_ptr()
    torch.testing.assert_close(out.float(), ref, atol=3e-2, rtol=1e-2)


def test_gemm_strided_views_and_f32(cuda):
    g = torch.Generator(device="cuda").manual_seed(3)
    big = rnd(640, 4352, gen=g)
    a = big[:, :1152]  # ld = 4352
    w = rnd(256, 1152, scale=1 / 34, gen=g)
    out = torch.empty(640, 512, device="cuda", dtype=torch.float32)
    ops.gemm(a, w, out=out[:, 128:384], out_f32=True)
    ref = a.float() @ w.float().T
    torch.testing.assert_close(out[:, 128:384], ref, atol=1e-4, rtol=1e-4)


def test_gemm_rejects_bad_k(cuda):
    a = torch.zeros(4, 100, dtype=torch.bfloat16, device="cuda")
    w = torch.zeros(8, 100, dtype=torch.bfloat16, device="cuda")
    with pytest.raises(_lib.MMEError, match="multiple of 64"):
        ops.gemm(a, w)


def test_gemm_rejects_cpu_tensor():
    a = torch.zeros(4, 64, dtype=torch.bfloat16)
    with pytest.raises(ValueError, match="no host fallback"):
        ops.gemm(a, a)


def attn_ref(qkv, B, T, H, hd, lens, causal, scale):
    q, k, v = qkv.float().view(B, T, 3, H, hd).permute(2, 0, 3, 1, 4)
    s = (q @ k.transpose(-1, -2)) * scale
    mask = torch.zeros(B, 1, T, T, dtype=torch.bool, device=qkv.device)
    if lens is not None:
        ar = torch.arange(T, device=qkv.device)
        mask |= (ar[None, :] >= lens[:, None].long())[:, None, None, :]
    if causal:
        mask |= torch.triu(torch.ones(T, T, dtype=torch.bool, device=qkv.device), 1)
    s = s.masked_fill(mask, float("-inf"))
    p = torch.softmax(s, -1)
    return (p @ v).transpose(1, 2).reshape(B * T, H * hd)


@pytest.mark.parametrize("B,T,H,hd,causal,lens", [
    (2, 729, 16, 72, False, None),     # SigLIP-400M vision
    (2, 64, 16, 72, False, [64, 23]),  # SigLIP text with padding mask
    (3, 64, 3, 72, False, [64, 1, 30]),  # short kernel: odd unit count (9), last block half empty
    (5, 40, 1, 80, True, [40, 7, 40, 1, 33]),  # short kernel: causal + padding, T < 64
    (3, 64, 5, 64, True, None),
    (3, 77, 12, 64, True, None),       # CLIP-L text
    (3, 77, 16, 64, True, [77, 9, 40]),
    (2, 257, 16, 80, False, None),     # ViT-H/14-224 (9-wave blocks, one per batch-head)
    (2, 270, 3, 80, True, [270, 100]),  # 9-wave blocks: causal + padding
    (2, 257, 2, 72, False, [257, 200]),  # 9-wave blocks at hd 72 (ones column of V^T)
    (1, 730, 4, 80, False, None),      # DFN5B-H-378 (12-wave blocks)
    (2, 700, 2, 80, True, [700, 390]),  # 12-wave blocks: causal + padding
    (2, 577, 4, 64, False, None),      # CLIP-L-336
    (3, 17, 4, 80, False, None),
    (4, 16, 8, 72, False, [16, 5, 9, 13]),
    (2, 1, 2, 64, False, None),
    (2, 300, 4, 64, True, [300, 133]),     # LDS-DMA kernels: causal + padding, 4- and 8-wave blocks
    (2, 520, 4, 72, False, [520, 301]),
    (1, 1000, 2, 80, False, [999]),
    (2, 200, 3, 72, True, None),
])
def test_attention(cuda, B, T, H, hd, causal, lens):
    g = torch.Generator(device="cuda").manual_seed(B * T + hd)
    qkv = rnd(B * T, 3 * H * hd, scale=1.5, gen=g)
    sl = None if lens is None else torch.tensor(lens, dtype=torch.int32, device="cuda")
    out = ops.attention(qkv, B, T, H, hd, seq_lens=sl, causal=causal)
    ref = attn_ref(qkv, B, T, H, hd, sl, causal, hd ** -0.5)
    torch.testing.assert_close(out.float(), ref, atol=2e-2, rtol=2e-2)


PROD_ATTN_KINDS = (38, 41, 58, 62, 65, 83, 84, 86, 87, 88, 89, 94, 97, 102)  # in the production library; the rest are development forms (libmme_dev.so)


@pytest.mark.parametrize("kind", [k if k in PROD_ATTN_KINDS else pytest.param(k, marks=pytest.mark.dev)
                                  for k in (38, 39, 40, 41, 42, 43, 44, 45, 46, 47, 48, 49, 50, 51, 52, 54, 55, 56,
                                            57, 58, 59, 60, 61, 62, 63, 65, 78, 79, 80, 81, 82, 83, 84,
                                            86, 87, 88, 89, 91, 92, 93)])
@pytest.mark.parametrize("B,T,H,hd,causal,lens", [
    (2, 729, 4, 72, False, None),       # SigLIP vision geometry
    (2, 520, 3, 72, False, [520, 301]),  # key padding, partial last tile
    (2, 200, 3, 72, True, None),
    (1, 730, 3, 80, False, None),        # DFN5B
    (2, 257, 2, 80, True, [257, 100]),
    (2, 577, 3, 64, False, None),        # CLIP-L (f32 weight sums, no ones plane)
    (2, 300, 2, 64, True, [300, 133]),
])
def test_attention_m32(cuda, kind, B, T, H, hd, causal, lens):
    """attn_m32_kernel (v_mfma_f32_32x32x16_bf16 flash loop) forced through the dev switch."""
    g = torch.Generator(device="cuda").manual_seed(B * T + hd + kind)
    qkv = rnd(B * T, 3 * H * hd, scale=1.5, gen=g)
    sl = None if lens is None else torch.tensor(lens, dtype=torch.int32, device="cuda")
    with ops.kernel_forms(attention=30 + kind):
        out = ops.attention(qkv, B, T, H, hd, seq_lens=sl, causal=causal)
    torch.cuda.synchronize()
    ref = attn_ref(qkv, B, T, H, hd, sl, causal, hd ** -0.5)
    torch.testing.assert_close(out.float(), ref, atol=2e-2, rtol=2e-2)


SKIP_CASES = [
    (4, 257, 16, False, None),        # ViT-H/14-224: last tile 1 key
    (3, 730, 4, False, None),         # T = 730: last tile 26 keys
    (4, 729, 16, False, None),        # SigLIP-400M vision: last tile 25 keys
    (2, 300, 3, True, [300, 280]),    # key padding: the skip follows each sequence's length
    (2, 769, 2, False, [769, 700]),   # a tile whose second block holds keys (no skip) beside one that skips
    (2, 520, 3, False, [520, 301]),
]


def _skip_pair(qkv, B, T, H, hd, sl, causal, ref, kind):
    outs = []
    for k in (ref, ref, kind, kind):
        with ops.kernel_forms(attention=30 + k):
            outs.append(ops.attention(qkv, B, T, H, hd, seq_lens=sl, causal=causal))
        torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[2], outs[3]), "attention is not deterministic"
    a, b = outs[0].float(), outs[2].float()
    d = (a - b).abs()
    # one bf16 ulp of max(|x|, 1/16): near-cancelling outputs (|o| << the row's scale) carry the
    # absolute error of their terms, not a relative one
    ulp = torch.maximum(a.abs(), b.abs()).clamp_min(2.0 ** -4) * 2.0 ** -7
    return int((d > 0).sum()), d, ulp


@pytest.mark.parametrize("hd,kind,ref", [(80, 65, 41), (72, 62, 58), (72, 83, 84), (80, 86, 88)])
@pytest.mark.parametrize("B,T,H,causal,lens", SKIP_CASES)
def test_attention_skip_vs_unskipped(cuda, hd, kind, ref, B, T, H, causal, lens):
    """The production kernels that skip a tile's second 32-key block when it lies wholly past the keys
    (kind 65: attn_m32_kernel in 9-wave blocks, hd 80; kind 62: attn_hyb_kernel, hd 72; kind 83: kind 62
    with the 2^8 rescale threshold, production for hd 72 since round 4; kind 86: kind 65 with it) against
    the same kernels without the skip (kinds 41 / 58 / 84 / 88): bit-identical on every output. An MFMA
    with an all-zero operand leaves its accumulator unchanged (tools/mfma_zero_probe.hip), and since
    round 5 attention.hip is built with -ffp-contract=off and states its FMAs explicitly (the exp2
    argument fma(s, c, -m c)), so no kernel's arithmetic depends on where the compiler contracts a
    multiply-add: round 4's rare 1-2 ulp differences between these pairs were exactly that
    (profiles/r05_v1_skip_contract_on_off.log: 0 of every output differ with contraction off)."""
    g = torch.Generator(device="cuda").manual_seed(B * T + hd)
    qkv = rnd(B * T, 3 * H * hd, scale=1.5, gen=g)
    sl = None if lens is None else torch.tensor(lens, dtype=torch.int32, device="cuda")
    nd, d, _ = _skip_pair(qkv, B, T, H, hd, sl, causal, ref, kind)
    first = (d > 0).nonzero()[:4].tolist()
    assert nd == 0, f"kind {kind} differs from kind {ref} on {nd} outputs (max {d.max().item():.3g}, first {first})"


@pytest.mark.parametrize("B,T,H,lens", [
    (4, 257, 16, None),            # ViT-H/14-224
    (37, 257, 16, None),           # 592 units: more than one block per CU, uneven XCD ranges
    (512, 257, 16, None),          # the bench's execution batch: 8192 units, 32 per block
    (3, 257, 5, [257, 100, 1]),    # key padding: each unit's own tile count and skip
    (2, 200, 3, [200, 64]),
    (1, 257, 1, None),             # one unit: 7 of 8 blocks exit at once
    (2, 288, 2, None),             # a full 9-wave query block
    (3, 65, 2, None),
])
def test_attention_persistent_vith_bit_identical(cuda, B, T, H, lens):
    """Kind 94 (attn_m32p_kernel: kind 86's flash loop as a persistent walk over (image, head) units,
    the next unit's first K / V tile and Q fragments loaded under the last tile of the current one)
    against kind 86: bit-identical on every output, across unit counts below, near and far above the
    CU count and per-image key lengths."""
    g = torch.Generator(device="cuda").manual_seed(B * T + H)
    qkv = rnd(B * T, 3 * H * 80, scale=1.5, gen=g)
    sl = None if lens is None else torch.tensor(lens, dtype=torch.int32, device="cuda")
    nd, d, _ = _skip_pair(qkv, B, T, H, 80, sl, False, 86, 94)
    assert nd == 0, f"kind 94 differs from kind 86 on {nd} outputs (max {d.max().item():.3g}, " \
                    f"first {(d > 0).nonzero()[:4].tolist()})"


@pytest.mark.dev
@pytest.mark.parametrize("kind", [70, 71, 72])
@pytest.mark.parametrize("B,T,H,causal,lens", SKIP_CASES + [(2, 200, 2, True, None), (1, 64, 2, False, None),
                                                         (1, 65, 1, False, None)])
def test_attention_pingpong_skip_bit_identical_to_kind58(cuda, kind, B, T, H, causal, lens):
    """Dev kinds 70-72 (attn_pp_kernel: kind 62's arithmetic INCLUDING its last-tile skip, with the
    block's wave rows one matrix / vector phase apart) against kind 58 (no skip): bit-identical on every
    output -- the skipped block's MFMAs contribute exactly nothing."""
    g = torch.Generator(device="cuda").manual_seed(B * T + 72)
    qkv = rnd(B * T, 3 * H * 72, scale=1.5, gen=g)
    sl = None if lens is None else torch.tensor(lens, dtype=torch.int32, device="cuda")
    nd, d, _ = _skip_pair(qkv, B, T, H, 72, sl, causal, 58, kind)
    assert nd == 0, f"kind {kind} differs from kind 58 on {nd} outputs (max {d.max().item():.3g}, " \
                    f"first {(d > 0).nonzero()[:4].tolist()})"


@pytest.mark.dev
@pytest.mark.parametrize("kind", [78, 79, 81])
@pytest.mark.parametrize("B,T,H,causal,lens", SKIP_CASES + [(1, 64, 2, False, None), (1, 65, 1, False, None),
                                                         (2, 129, 2, False, None), (2, 200, 2, True, None),
                                                         (1, 320, 3, False, None)])
def test_attention_ring_forms_vs_kind62(cuda, kind, B, T, H, causal, lens):
    """Dev kinds 78 (kind 62 on a three-slot K / V ring, asm DMA), 79 (four slots, the late wave row's
    PV one tile behind: the stagger) and 81 (kind 79 with packed exp arguments: the same per-element
    fma) run kind 62's arithmetic in the same order: identical outputs
    expected, held to the skip test's bound (the hyb loop's rare 1-ulp code-generation effect), across
    tile counts 1-5 (the ring and its 3- / 4-way unrolled loops) and padded / causal rows."""
    g = torch.Generator(device="cuda").manual_seed(B * T + 72)
    qkv = rnd(B * T, 3 * H * 72, scale=1.5, gen=g)
    sl = None if lens is None else torch.tensor(lens, dtype=torch.int32, device="cuda")
    nd, d, ulp = _skip_pair(qkv, B, T, H, 72, sl, causal, 62, kind)
    print(f"kinds 62/{kind}: {nd} of {d.numel()} outputs differ, max {d.max().item():.3g}")
    assert nd <= 1e-5 * d.numel() + 1 and bool((d <= 2 * ulp).all())


@pytest.mark.dev
@pytest.mark.parametrize("B,T,H,causal,lens", SKIP_CASES)
def test_attention_m32_8wave_skip_vs_kind38(cuda, B, T, H, causal, lens):
    """Dev kind 64 (kind 38's 8-wave attn_m32_kernel with the skip; not built into production): the pair
    whose rare 1-ulp difference round 3 recorded (profiles/r03_v11_attn_m32_skip_diff.log); same bound
    as test_attention_skip_vs_unskipped."""
    g = torch.Generator(device="cuda").manual_seed(B * T + 80)
    qkv = rnd(B * T, 3 * H * 80, scale=1.5, gen=g)
    sl = None if lens is None else torch.tensor(lens, dtype=torch.int32, device="cuda")
    nd, d, ulp = _skip_pair(qkv, B, T, H, 80, sl, causal, 38, 64)
    print(f"kinds 38/64: {nd} of {d.numel()} outputs differ, max {d.max().item():.3g}, "
          f"first {(d > 0).nonzero()[:4].tolist()}")
    assert nd <= 1e-5 * d.numel() + 1 and bool((d <= 2 * ulp).all())


@pytest.mark.dev
@pytest.mark.parametrize("M,N,K,act", [(70001, 4352, 1152, 1), (5000, 5120, 1280, 2), (300, 1024, 192, 1),
                                       (2000, 4096, 1024, 0), (129, 512, 256, 1)])
def test_gemm_pipe10_bit_identical_to_pipe9(cuda, M, N, K, act):
    """Dev form 90 (pipe10: persistent pipe9 with the next tile's first units DMA'd under the epilogue,
    two-pass staging) runs pipe9's main loop and epilogue arithmetic: bit-identical outputs, with the
    LayerNorm-fold epilogue and with bias + activation, ragged M, fewer tiles than CUs and many per CU."""
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    x = rnd(M, K, gen=g)
    w = rnd(N, K, scale=K ** -0.5, gen=g)
    b = rnd(N, scale=0.1, gen=g)
    gam = (1 + 0.1 * torch.randn(K, device="cuda", generator=g)).to(torch.bfloat16)
    bet = rnd(K, scale=0.1, gen=g)
    f = ops.LNFolded(w, b, gam, bet)
    st = ops.rowstats(x, 1e-6, d=K)
    outs = []
    for form in (80, 90):  # dev form 80 = pipe9 forced (production picks other kernels below 1 M outputs)
        with ops.kernel_forms(gemm=form):
            outs.append((ops.gemm_lnfold(x, f, st, act=act), ops.gemm(x, w, b, act=act)))
        torch.cuda.synchronize()
    for a_, b_ in zip(outs[0], outs[1]):
        assert torch.equal(a_, b_), f"pipe10 differs from pipe9 ({M}x{N}x{K}, act {act})"


def test_attention_production_full_grid(cuda):
    """The production hd-72 kernel over the bench's full launch grid (417 images x 16 heads x
    3 query blocks of SigLIP vision; 239 before round 3's larger execution batches) against the fp32
    reference on the first and last images (grid-to-(batch, head, query block) mapping at production
    size)."""
    B, T, H, hd = 417, 729, 16, 72
    g = torch.Generator(device="cuda").manual_seed(729)
    qkv = rnd(B * T, 3 * H * hd, scale=1.5, gen=g)
    out = ops.attention(qkv, B, T, H, hd).float().view(B, T, H * hd)
    assert torch.isfinite(out).all()
    for b in (0, 1, B - 2, B - 1):
        ref = attn_ref(qkv[b * T:(b + 1) * T], 1, T, H, hd, None, False, hd ** -0.5)
        torch.testing.assert_close(out[b], ref.view(T, H * hd), atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("hd,T,exact,thr", [(72, 729, 62, 83), (80, 730, 38, 87), (80, 257, 65, 86),
                                            (64, 577, 0, 89)])
def test_attention_threshold_vs_exact_rescale(cuda, hd, T, exact, thr):
    """Round 4's production flash loops rescale O only when a query's running max grows by more than
    2^8 in the exp2 domain (kinds 83 / 87 / 86 / 89) instead of whenever it grows (kinds 62 / 38 / 65 /
    0). Against an fp64 reference on the encoder geometries the threshold forms' error stays at the
    exact-rescale forms' level: mean error within 1.3x, max within 1.5x + 2^-7 (measured: hd 72 T 729
    0.00052 vs 0.00045 / 0.0179 vs 0.0155, hd 80 T 730 0.00052 vs 0.00045, hd 80 T 257 0.00067 vs
    0.00060, hd 64 T 577 0.00058 vs 0.00048 / 0.025 vs 0.015; profiles/r04_v22_thr_pytest.log). The
    two forms are not compared output by output: where the dominant P is no longer exactly 1 its
    bf16 rounding moves near-cancelling outputs by more than their own ulp, in either form's favour."""
    B, H = 8, 16
    g = torch.Generator(device="cuda").manual_seed(T * hd)
    qkv = rnd(B * T, 3 * H * hd, scale=1.5, gen=g)
    q, k, v = qkv.double().view(B, T, 3, H, hd).permute(2, 0, 3, 1, 4)
    ref = (torch.softmax((q @ k.transpose(-1, -2)) * hd ** -0.5, -1) @ v).transpose(1, 2).reshape(B * T, H * hd)
    outs = {}
    for kind in (exact, thr):
        with ops.kernel_forms(attention=30 + kind):
            outs[kind] = ops.attention(qkv, B, T, H, hd).double()
        torch.cuda.synchronize()
    e_ex, e_th = (outs[exact] - ref).abs(), (outs[thr] - ref).abs()
    print(f"hd {hd} T {T}: mean err {e_ex.mean().item():.3g} (kind {exact}) / {e_th.mean().item():.3g} "
          f"(kind {thr}); max {e_ex.max().item():.3g} / {e_th.max().item():.3g}")
    assert e_th.mean().item() <= 1.3 * e_ex.mean().item()
    assert e_th.max().item() <= 1.5 * e_ex.max().item() + 2.0 ** -7


def _qs_inputs(B, T, H, hd, amp, g):
    """fp32 Q / K / V draws; qkv = their bf16 roundings, qkv_s the same with Q rounded from
    q * attention_q_scale(hd) (what the Q-scaled projection produces: one rounding either way)."""
    q32, k32, v32 = (torch.randn(B * T, H * hd, device="cuda", generator=g) * amp for _ in range(3))
    kb, vb = k32.to(torch.bfloat16), v32.to(torch.bfloat16)
    qkv = torch.cat([q32.to(torch.bfloat16), kb, vb], 1)
    qkv_s = torch.cat([(q32 * ops.attention_q_scale(hd)).to(torch.bfloat16), kb, vb], 1)
    return q32, kb, vb, qkv, qkv_s


def _hd72_production_kind(T):
    """mme_attention's dispatch at head dim 72 (attention.hip attention_entry)."""
    if T <= 64:
        return 16
    if T <= 128:
        return 89
    pad8, pad4, pad9 = -(-T // 256) * 256, -(-T // 128) * 128, -(-T // 288) * 288
    if pad9 * 10 < min(pad8, pad4) * 9:
        return 35
    return 83 if pad8 * 10 <= pad4 * 11 else 14


def _attn_f64(q32, kb, vb, B, T, H, hd, sl, causal):
    q, k, v = (t.double().view(B, T, H, hd).transpose(1, 2) for t in (q32, kb, vb))
    s = (q @ k.transpose(-1, -2)) * hd ** -0.5
    mask = torch.zeros(B, 1, T, T, dtype=torch.bool, device="cuda")
    if sl is not None:
        mask |= (torch.arange(T, device="cuda")[None, :] >= sl[:, None].long())[:, None, None, :]
    if causal:
        mask |= torch.triu(torch.ones(T, T, dtype=torch.bool, device="cuda"), 1)
    return (torch.softmax(s.masked_fill(mask, float("-inf")), -1) @ v).transpose(1, 2).reshape(B * T, H * hd)


@pytest.mark.parametrize("B,T,H,causal,lens", [(8, 729, 16, False, None), (2, 520, 3, False, [520, 301]),
                                                 (2, 200, 3, True, None), (3, 64, 2, False, [64, 1, 30]),
                                                 (2, 65, 2, False, None), (2, 300, 3, True, [300, 280]),
                                                 (1, 32, 2, False, None), (2, 769, 2, False, [769, 700]),
                                                 (2, 1024, 4, False, None)])
def test_attention_mfma_bias_vs_fp64(cuda, B, T, H, causal, lens):
    """Kind 98 (round 6, production for hd 72 through mme_attention_qs): kind 83's loop with the exp2
    argument c s - M produced by the QK^T MFMA -- Q arrives multiplied by c = scale log2 e (folded into
    the Q projection before its one bf16 rounding), Q^T row 72 = -M against a ones row of K, M the
    query's running max held as a bf16 value. Against an fp64 reference of the unrounded fp32 Q its
    error stays at that of kind 83's loop on the same pre-scaled Q (mean within 1.15x, max within 1.5x
    + 2^-7) and, where the sample is large, within 1.15x of kind 83 on the plain Q (one rounding of Q
    either way), on the SigLIP and ColPali (T 1024) geometries and on padded, causal, one- and two-tile
    sequences, with scores scaled up 4x as well (more rescales, larger M). Kind 97 (the same loop
    scaling Q in the kernel: a second rounding of Q, 1.3x kind 83's mean error) is reported only."""
    hd = 72
    g = torch.Generator(device="cuda").manual_seed(B * T + 97)
    sl = None if lens is None else torch.tensor(lens, dtype=torch.int32, device="cuda")
    for amp in (1.5, 6.0):
        q32, kb, vb, qkv, qkv_s = _qs_inputs(B, T, H, hd, amp, g)
        ref = _attn_f64(q32, kb, vb, B, T, H, hd, sl, causal)
        outs = {}
        for kind in (83, 97):
            with ops.kernel_forms(attention=30 + kind):
                outs[kind] = ops.attention(qkv, B, T, H, hd, seq_lens=sl, causal=causal).double()
        for kind in (83, 98):  # the same pre-scaled Q: kind 83's own loop at c = 1, and kind 98
            with ops.kernel_forms(attention=30 + kind):
                outs[f"{kind}qs"] = ops.attention(qkv_s, B, T, H, hd, seq_lens=sl, causal=causal,
                                                  q_prescaled=True).double()
        prod = ops.attention(qkv_s, B, T, H, hd, seq_lens=sl, causal=causal, q_prescaled=True).double()
        torch.cuda.synchronize()
        if _hd72_production_kind(T) == 83:  # where the plain entry runs kind 83, the qs entry runs kind 98
            assert torch.equal(prod, outs["98qs"]), "the qs production dispatch is not kind 98"
        assert torch.isfinite(outs["98qs"]).all()
        e = {k: (o - ref).abs() for k, o in outs.items()}
        print(f"B {B} T {T} amp {amp}: mean err " + " / ".join(f"{e[k].mean().item():.3g} ({k})" for k in e) +
              "; max " + " / ".join(f"{e[k].max().item():.3g}" for k in e))
        # the loop's arithmetic, same inputs: kind 98 against kind 83
        assert e["98qs"].mean().item() <= 1.15 * e["83qs"].mean().item()
        assert e["98qs"].max().item() <= 1.5 * e["83qs"].max().item() + 2.0 ** -7
        if B * T * H >= 10000:  # the Q-scaled projection against the plain one (one rounding each)
            assert e["98qs"].mean().item() <= 1.15 * e[83].mean().item()


@pytest.mark.parametrize("hd,kind,ref", [(72, 99, 87), (80, 100, 87), (80, 101, 86)])
@pytest.mark.parametrize("B,T,H,causal,lens", [(4, 730, 16, False, None), (8, 257, 16, False, None),
                                                 (2, 520, 3, False, [520, 301]), (2, 200, 3, True, None),
                                                 (2, 65, 2, False, None), (1, 32, 2, False, None),
                                                 (3, 257, 5, False, [257, 100, 1])])
def test_attention_m32_mfma_bias_vs_fp64(cuda, hd, kind, ref, B, T, H, causal, lens):
    """Kinds 99-101 (round 6): attn_m32_kernel with attn_hyb_kernel's MFMA bias (Q^T row hd = -M against a
    ones row of K; at hd 80 an extra k-step holds it), on the qs entry only. Same bounds as
    test_attention_mfma_bias_vs_fp64 against the kernel they extend (87: 8-wave blocks, 86: 9-wave blocks
    with the last-tile skip) run on the same pre-scaled Q at c = 1."""
    g = torch.Generator(device="cuda").manual_seed(B * T + hd + kind)
    sl = None if lens is None else torch.tensor(lens, dtype=torch.int32, device="cuda")
    for amp in (1.5, 6.0):
        q32, kb, vb, qkv, qkv_s = _qs_inputs(B, T, H, hd, amp, g)
        refo = _attn_f64(q32, kb, vb, B, T, H, hd, sl, causal)
        outs = {}
        for k in (ref, kind):
            with ops.kernel_forms(attention=30 + k):
                outs[k] = ops.attention(qkv_s, B, T, H, hd, seq_lens=sl, causal=causal, q_prescaled=True).double()
        torch.cuda.synchronize()
        assert torch.isfinite(outs[kind]).all()
        e = {k: (o - refo).abs() for k, o in outs.items()}
        print(f"hd {hd} B {B} T {T} amp {amp}: mean err {e[ref].mean().item():.3g} ({ref}) / "
              f"{e[kind].mean().item():.3g} ({kind}); max {e[ref].max().item():.3g} / {e[kind].max().item():.3g}")
        assert e[kind].mean().item() <= 1.15 * e[ref].mean().item()
        assert e[kind].max().item() <= 1.5 * e[ref].max().item() + 2.0 ** -7


@pytest.mark.parametrize("B,T,H,causal,lens", [(6, 77, 16, True, None), (5, 77, 16, True, [77, 9, 40, 1, 76]),
                                                 (3, 65, 3, True, [65, 64, 2]), (2, 128, 5, False, None),
                                                 (3, 100, 4, False, [100, 37, 99]), (4, 128, 3, True, [128, 127, 64, 65]),
                                                 (2, 40, 2, True, None)])
def test_attention_short2_vs_fp64(cuda, B, T, H, causal, lens):
    """attn_short2_kernel (kind 102, round 6: production for 64 < T <= 128 at head dim 64, the CLIP causal text
    towers) against the fp64 softmax attention, beside kind 89 (attn_fwd_kernel with the rescale threshold,
    production before): mean / max error within 1.15x / 1.5x of kind 89's on the same inputs (one softmax pass
    over all 128 keys instead of two online tiles), all outputs finite; T = 40 exercises the clamped rows."""
    g = torch.Generator(device="cuda").manual_seed(B * T + H)
    sl = None if lens is None else torch.tensor(lens, dtype=torch.int32, device="cuda")
    hd = 64
    for amp in (1.5, 4.0):
        q32, kb, vb, qkv, _ = _qs_inputs(B, T, H, hd, amp, g)
        refo = _attn_f64(q32, kb, vb, B, T, H, hd, sl, causal)
        outs = {}
        for kind in (89, 102):
            with ops.kernel_forms(attention=30 + kind):
                outs[kind] = ops.attention(qkv, B, T, H, hd, seq_lens=sl, causal=causal).double()
        torch.cuda.synchronize()
        assert torch.isfinite(outs[102]).all()
        e = {k: (o - refo).abs() for k, o in outs.items()}
        print(f"short2 B {B} T {T} H {H} causal {causal} amp {amp}: mean err {e[89].mean().item():.3g} (89) / "
              f"{e[102].mean().item():.3g} (102); max {e[89].max().item():.3g} / {e[102].max().item():.3g}")
        assert e[102].mean().item() <= 1.15 * e[89].mean().item()
        assert e[102].max().item() <= 1.5 * e[89].max().item() + 2.0 ** -7
    if T > 64:  # the production dispatch picks it
        plain = ops.attention(qkv, B, T, H, hd, seq_lens=sl, causal=causal)
        with ops.kernel_forms(attention=30 + 102):
            forced = ops.attention(qkv, B, T, H, hd, seq_lens=sl, causal=causal)
        assert torch.equal(plain, forced)


@pytest.mark.parametrize("B,T,H,hd,causal,lens", [(2, 729, 4, 72, False, None), (3, 64, 3, 72, False, [64, 1, 30]),
                                                   (3, 77, 4, 64, True, [77, 9, 40]), (2, 577, 3, 64, False, None),
                                                   (1, 730, 3, 80, False, None), (2, 257, 4, 80, False, [257, 100]),
                                                   (2, 100, 2, 72, False, None), (2, 300, 2, 80, True, None)])
def test_attention_qs_entry_every_kernel(cuda, B, T, H, hd, causal, lens):
    """mme_attention_qs on every production kernel (short, attn_fwd, attn_m32, attn_hyb): with Q scaled by
    attention_q_scale the outputs match the fp32 reference at test_attention's tolerance, like the plain
    entry on the plain Q."""
    g = torch.Generator(device="cuda").manual_seed(B * T + hd + 1)
    sl = None if lens is None else torch.tensor(lens, dtype=torch.int32, device="cuda")
    q32, kb, vb, qkv, qkv_s = _qs_inputs(B, T, H, hd, 1.5, g)
    ref = _attn_f64(q32, kb, vb, B, T, H, hd, sl, causal)
    out = ops.attention(qkv_s, B, T, H, hd, seq_lens=sl, causal=causal, q_prescaled=True)
    plain = ops.attention(qkv, B, T, H, hd, seq_lens=sl, causal=causal)
    torch.testing.assert_close(out.double(), ref, atol=2e-2, rtol=2e-2)
    torch.testing.assert_close(plain.double(), ref, atol=2e-2, rtol=2e-2)


@pytest.mark.dev
def test_attention_hd72_production_grid_vs_kind30(cuda):
    """Round 3's production hd-72 kernel (attn_hyb_kernel, kind 62; round 4's kind 83 adds the rescale
    threshold, test above) over the bench's full launch grid (239 images x 16 heads x 3 query blocks of
    SigLIP vision) against the round-1 production kernel (kind 30, 16x16x32 throughout): the two differ
    only in MFMA shape and summation order, so every output agrees within a few bf16 ulps (the fp32
    reference comparison of both is test_attention / test_attention_m32 at smaller batches)."""
    B, T, H, hd = 239, 729, 16, 72
    g = torch.Generator(device="cuda").manual_seed(729)
    qkv = rnd(B * T, 3 * H * hd, scale=1.5, gen=g)
    outs = {}
    for kind in (0, 30):
        with ops.kernel_forms(attention=30 + 62 if kind == 0 else 30 + kind):
            outs[kind] = ops.attention(qkv, B, T, H, hd).float()
        torch.cuda.synchronize()
    diff = (outs[0] - outs[30]).abs()
    print(f"hd-72 production grid: max |diff| {diff.max().item():.3g}, mean {diff.mean().item():.3g}")
    assert torch.isfinite(outs[0]).all()
    # bf16(p) may round differently where the two fp32 score sums straddle a rounding boundary
    # (an error on the scale of |v|, not of the output, which can be a cancellation): the same
    # absolute bound as the fp32-reference tests, and almost every output bit-identical
    frac = (diff > 0).float().mean().item()
    print(f"hd-72 production grid: outputs differing {frac:.2e}")
    assert diff.max().item() <= 2e-2, "hd-72 kernels disagree beyond the fp32-reference tolerance"
    assert diff.mean().item() < 1e-5 and frac < 1e-3


def test_attention_strided_qkv(cuda):
    B, T, H, hd = 2, 100, 16, 72
    g = torch.Generator(device="cuda").manual_seed(9)
    wide = rnd(B * T, 4352, gen=g)
    qkv = wide[:, : 3 * H * hd]
    out = ops.attention(qkv, B, T, H, hd)
    torch.testing.assert_close(out.float(), attn_ref(qkv.contiguous(), B, T, H, hd, None, False, hd ** -0.5),
                               atol=2e-2, rtol=2e-2)


# (image, all heads) blocks for H * hd <= 1152 (SigLIP MAP head: 16 x 72); per-(image, head)
# blocks otherwise (H = 5: 256 % H != 0)
@pytest.mark.parametrize("B,T,H,hd", [(3, 729, 16, 72), (2, 49, 8, 72), (239, 729, 16, 72), (417, 729, 16, 72),
                                     (2, 100, 5, 64)])
def test_probe_attention(cuda, B, T, H, hd):
    g = torch.Generator(device="cuda").manual_seed(T)
    d = H * hd
    q = rnd(d, gen=g)
    kv = rnd(B * T, 2 * d, gen=g)
    out = ops.probe_attention(q, kv, B, T, H, hd)
    k = kv.float()[:, :d].view(B, T, H, hd).transpose(1, 2)
    v = kv.float()[:, d:].view(B, T, H, hd).transpose(1, 2)
    qq = q.float().view(1, H, 1, hd)
    p = torch.softmax((qq @ k.transpose(-1, -2)) * hd ** -0.5, -1)
    ref = (p @ v).reshape(B, d)
    torch.testing.assert_close(out.float(), ref, atol=2e-2, rtol=2e-2)


# SigLIP MAP head with the probe absorbed into the key projection (mme_map_pool): the full
# head geometry (16 heads, d 1152, T 729) at the production batch, tiny heads, odd T, and the
# score halves of a real U (hi + lo) against an fp32 torch reference of the same op
@pytest.mark.parametrize("B,T,H,D", [(3, 729, 16, 1152), (417, 729, 16, 1152), (2, 49, 4, 64), (2, 17, 5, 320)])
def test_map_pool(cuda, B, T, H, D):
    g = torch.Generator(device="cuda").manual_seed(T + D)
    x = rnd(B * T, D, gen=g)
    u = torch.randn(H, D, generator=g, device="cuda") * D ** -0.5 * 3.0
    u_hi = u.to(torch.bfloat16)
    u2 = torch.cat([u_hi, (u - u_hi.float()).to(torch.bfloat16)]).contiguous()
    S = ops.gemm(x, u2, out_f32=True)
    out = ops.map_pool(S, x, B, T, H)
    s_ref = (x.float() @ u.t()).view(B, T, H)                  # fp32 scores with the unsplit U
    p = torch.softmax(s_ref, dim=1)                            # over tokens
    ref = torch.einsum("bth,btc->bhc", p, x.float().view(B, T, D)).reshape(B * H, D)
    torch.testing.assert_close(out.float(), ref, atol=2e-3, rtol=1e-2)
    # the hi / lo split carries the scores to ~2^-16 relative
    torch.testing.assert_close((S[:, :H] + S[:, H:2 * H]).view(B, T, H), s_ref, atol=1e-4, rtol=1e-4)


@pytest.mark.parametrize("rows,d", [(1, 64), (1000, 1152), (37, 1280), (5, 768), (9, 320)])
def test_layernorm(cuda, rows, d):
    g = torch.Generator(device="cuda").manual_seed(rows + d)
    x = rnd(rows, d, scale=3.0, gen=g) + 0.5
    gm = rnd(d, gen=g)
    bt = rnd(d, gen=g)
    out = ops.layernorm(x, gm, bt, 1e-6)
    ref = torch.nn.functional.layer_norm(x.float(), (d,), gm.float(), bt.float(), 1e-6)
    torch.testing.assert_close(out.float(), ref, atol=3e-2, rtol=1e-2)
    idx = torch.tensor([rows - 1, 0], dtype=torch.int32, device="cuda")
    out2 = ops.layernorm(x, gm, bt, 1e-6, rows_idx=idx)
    torch.testing.assert_close(out2.float(), ref[idx.long()], atol=3e-2, rtol=1e-2)


@pytest.mark.parametrize("rows,d", [(1, 64), (1000, 1152), (37, 1280), (5, 768)])
def test_rowstats(cuda, rows, d):
    g = torch.Generator(device="cuda").manual_seed(rows * 3 + d)
    x = rnd(rows, d, scale=3.0, gen=g) + 0.5
    st = ops.rowstats(x, 1e-6)
    xf = x.float()
    mean = xf.mean(dim=1)
    rstd = torch.rsqrt(xf.var(dim=1, unbiased=False) + 1e-6)
    torch.testing.assert_close(st[:, 0], mean, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(st[:, 1], rstd, atol=1e-5, rtol=1e-4)


# LayerNorm -> Linear with the LayerNorm folded into the weights (mme_gemm_lnfold) against
# the unfused fp32 chain; the residual-stream rows carry an offset (mean) and a scale so
# the mean-subtraction term matters. Shapes cover the generic (small) and pipelined
# (incl. split-grid N = 1152 / 3456) kernels.
@pytest.mark.parametrize("M,N,K", [(100, 200, 128), (2048, 3456, 1152), (1500, 4352, 1152), (4096, 1152, 1152)])
@pytest.mark.parametrize("act", [0, 1])
def test_gemm_lnfold(cuda, M, N, K, act):
    g = torch.Generator(device="cuda").manual_seed(M + N + act)
    x = rnd(M, K, scale=4.0, gen=g) + 2.0
    gm = (1.0 + 0.2 * torch.randn(K, generator=g, device="cuda")).to(torch.bfloat16)
    bt = rnd(K, scale=0.1, gen=g)
    w = rnd(N, K, scale=1 / math.sqrt(K), gen=g)
    b = rnd(N, scale=0.1, gen=g)
    fold = ops.LNFolded(w, b, gm, bt)
    out = ops.gemm_lnfold(x, fold, ops.rowstats(x, 1e-6), act=act)
    h = torch.nn.functional.layer_norm(x.float(), (K,), gm.float(), bt.float(), 1e-6)
    ref = act_ref(h @ w.float().T + b.float(), act)
    torch.testing.assert_close(out.float(), ref, atol=3e-2, rtol=2e-2)
    # and within the same error budget as the unfolded bf16 chain (LayerNorm rounded to bf16)
    unf = ops.gemm(ops.layernorm(x, gm, bt, 1e-6), w, b, act=act).float()
    e_fold = (out.float() - ref).abs().mean().item()
    e_unf = (unf - ref).abs().mean().item()
    assert e_fold <= 1.5 * e_unf + 1e-4, (e_fold, e_unf)


@pytest.mark.parametrize("act", [1, 2, 3])
@pytest.mark.parametrize("M,N", [(4096, 4352), (2048, 1152)])
def test_gemm_activation_vs_float64(cuda, M, N, act):
    """The epilogue activations on exactly representable pre-activations: A[m, 0] = x_m (bf16), B[n, 0] = 1,
    everything else 0, so acc = x_m exactly and the output is bf16(act(x_m)) (every column the same). Against
    the float64 formula rounded to bf16: gelu_tanh / quick_gelu on v_exp_f32 + v_rcp_f32, gelu_erf
    (nn.GELU's exact form, LAION-CLIP-H) through the sigmoid-of-polynomial form of common.h (round 6; an
    erfc fit in round 5, libm erff before): >= 99.5 % bit-identical, the rest one bf16 ulp, over x in
    [-10, 10] and the tails (gelu_erf: on |x| <= 4, an absolute bound below; the fp32-level bound:
    test_gemm_gelu_erf_fp32_accuracy)."""
    K = 64
    x = torch.cat([torch.linspace(-10, 10, M - 64, device="cuda"), torch.logspace(-6, 1.2, 64, device="cuda")])
    xb = x.to(torch.bfloat16)
    A = torch.zeros(M, K, device="cuda", dtype=torch.bfloat16)
    A[:, 0] = xb
    B = torch.zeros(N, K, device="cuda", dtype=torch.bfloat16)
    B[:, 0] = 1
    out = ops.gemm(A, B, None, act=act)
    xd = xb.double()
    if act == 1:  # 0.5 x (1 + tanh u) = x sigmoid(2 u): the form without cancellation in the negative tail
        ref = xd * torch.sigmoid(2 * math.sqrt(2 / math.pi) * (xd + 0.044715 * xd ** 3))
    elif act == 2:
        ref = xd * torch.sigmoid(1.702 * xd)
    else:
        ref = 0.5 * xd * torch.special.erfc(-xd / math.sqrt(2))
    rb = ref.float().to(torch.bfloat16)
    got = out[:, 0]
    assert torch.equal(out, got[:, None].expand(-1, N)), "columns differ"
    ulp = (rb.float().abs().clamp_min(2.0 ** -126) * 2.0 ** -7)
    err = (got.float() - rb.float()).abs()
    # gelu_erf (round 6): an absolute bound. Its sigmoid-of-polynomial Phi carries an absolute error (erf-
    # equivalent <= 6e-7, test_gemm_gelu_erf_fp32_accuracy), so below x ~ -4, where |gelu| < 1.3e-4 and torch's
    # own fp32 0.5 x (1 + erf) is itself off by up to ~10 % relative, the bf16 outputs may differ by more than an
    # ulp; there every output must stay within 0.5 |x| 6e-7 + 1 bf16 ulp of the float64 value
    core = xb.float().abs() <= 4 if act == 3 else torch.ones_like(got, dtype=torch.bool)
    same = (got == rb)[core].float().mean().item()
    print(f"act {act}: {same:.5f} bit-identical to the float64 formula (|x| <= 4 for gelu_erf), max err / ulp "
          f"{(err / ulp)[core].max().item():.2f}")
    assert same >= 0.995 and bool((err[core] <= ulp[core] * 1.01).all())
    if act == 3:
        absb = 0.5 * xd.abs() * 6e-7 + ulp.double()
        assert bool(((got.double() - ref).abs() <= absb).all())


def test_gemm_gelu_erf_fp32_accuracy(cuda):
    """The exact-erf GELU (act 3, csrc/common.h gelu_erf2) at fp32 resolution, through the GEMM's fp32-output
    epilogue (the same device function every fc1 epilogue inlines): A[m, 0] = x_m exactly (bf16 values over
    [-12, 12] and a log grid near 0), B[n, 0] = 1. Erf-equivalent absolute error 2 |g - x Phi(x)| / |x| against
    float64 below 6e-7 (host restatement 3.5e-7 with correctly rounded exp2 / rcp; the device's v_exp_f32 /
    v_rcp_f32 are 1 ulp), and within 7e-7 of torch's own fp32 0.5 x (1 + erf(x / sqrt2)) on the device."""
    K = 64
    xs = torch.cat([torch.linspace(-12, 12, 60000, device="cuda"), torch.logspace(-3, 1.1, 4000, device="cuda"),
                    -torch.logspace(-3, 1.1, 4000, device="cuda")]).to(torch.bfloat16)
    xs = xs[xs.float().abs() > 1e-3]
    M = xs.numel()
    A = torch.zeros(M, K, device="cuda", dtype=torch.bfloat16)
    A[:, 0] = xs
    B = torch.zeros(8, K, device="cuda", dtype=torch.bfloat16)
    B[:, 0] = 1
    out = ops.gemm(A, B, None, act=3, out_f32=True)
    g = out[:, 0].double()
    xd = xs.double()
    ref = 0.5 * xd * torch.special.erfc(-xd / math.sqrt(2))
    xf = xs.float()
    gt = (xf * 0.5 * (1 + torch.erf(xf * 0.7071067811865476))).double()
    e_ours = (2 * (g - ref).abs() / xd.abs()).max().item()
    e_torch = (2 * (gt - ref).abs() / xd.abs()).max().item()
    e_diff = (2 * (g - gt).abs() / xd.abs()).max().item()
    print(f"gelu_erf fp32: erf-equivalent abs error {e_ours:.3g} (torch fp32 formula on the device {e_torch:.3g}); "
          f"difference from torch {e_diff:.3g}")
    assert e_ours < 6e-7 and e_diff < 7e-7


@pytest.mark.parametrize("M,N,K,act", [(303993, 4352, 1152, 1), (70001, 4352, 1152, 2), (5000, 5120, 1280, 2),
                                       (300, 4096, 1024, 1), (129, 8192, 256, 2), (116935, 5120, 1280, 3)])
def test_gemm_dispatched_fc1_bit_identical_to_pipe6(cuda, M, N, K, act):
    """The production fc1 dispatch (LayerNorm fold + gelu_tanh / quick_gelu on the persistent GEMM, grid
    from the device's CU count) against form 47 (pipe6, in the production library): the kernels share
    K order, MFMAs and epilogue arithmetic, so every output is bit-identical -- SigLIP's execution batch
    (417 images), ragged M, fewer tiles than CUs and many per CU."""
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    x = rnd(M, K, gen=g)
    w = rnd(N, K, scale=K ** -0.5, gen=g)
    b = rnd(N, scale=0.1, gen=g)
    gam = (1 + 0.1 * torch.randn(K, device="cuda", generator=g)).to(torch.bfloat16)
    bet = rnd(K, scale=0.1, gen=g)
    f = ops.LNFolded(w, b, gam, bet)
    st = ops.rowstats(x, 1e-6, d=K)
    prod = (ops.gemm_lnfold(x, f, st, act=act), ops.gemm(x, w, b, act=act))
    with ops.kernel_forms(gemm=47):
        ref = (ops.gemm_lnfold(x, f, st, act=act), ops.gemm(x, w, b, act=act))
    torch.cuda.synchronize()
    for p_, r_ in zip(prod, ref):
        assert torch.equal(p_, r_), f"dispatched fc1 differs from pipe6 ({M}x{N}x{K}, act {act})"


@pytest.mark.parametrize("M,N,K", [(116935, 1280, 1280), (116935, 1280, 5120), (5000, 3840, 1280), (300, 1024, 1024),
                                   (20000, 1152, 1152), (20000, 3456, 1152), (20111, 1152, 4352), (4000, 384, 4352),
                                   (303993, 1152, 1152)])
def test_gemm_form95_bit_identical_to_pipe6(cuda, M, N, K):
    """The production dispatch (pipe9 / pipe10 with every epilogue compiled for its operand set:
    bias, residual + the next LayerNorm's row statistics, LayerNorm fold), form 93 (the same kernels
    branching on their operands at run time) and form 95 (pipe10, the persistent GEMM, on every
    non-split epilogue) against form 47 (pipe6): bit-identical outputs and row statistics at ViT-H /
    CLIP shapes (whole 256-column tiles), SigLIP's split grid (N = 256 k + 128), ragged M, fewer tiles
    than CUs."""
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    x = rnd(M, K, gen=g)
    w = rnd(N, K, scale=K ** -0.5, gen=g)
    b = rnd(N, scale=0.1, gen=g)
    res = rnd(M, N, gen=g)
    gam = (1 + 0.1 * torch.randn(K, device="cuda", generator=g)).to(torch.bfloat16)
    bet = rnd(K, scale=0.1, gen=g)
    f = ops.LNFolded(w, b, gam, bet)
    fold = K <= 2048  # the LayerNorm fold precedes the qkv / fc1 GEMMs (K = the model width)
    st = ops.rowstats(x, 1e-6, d=K) if fold else None
    outs = []
    for form in (47, -1, 93, 95):
        with ops.kernel_forms(**({} if form == -1 else {"gemm": form})):
            y = ops.gemm(x, w, b)
            yl = ops.gemm_lnfold(x, f, st, act=0) if fold else y
            sr = torch.empty(M, 2, device="cuda", dtype=torch.float32)
            part = torch.empty(M * (N // 64) * 2, device="cuda", dtype=torch.float32)
            yr = ops.gemm_res_stats(x, w, b, res, 1e-6, sr, part)
            outs.append((y, yl, yr, sr))
        torch.cuda.synchronize()
    for form, o in zip((-1, 93, 95), outs[1:]):
        if form == -1 and M * N < 1024 * 1024:
            continue  # production takes the generic kernel below 1M outputs
        for a_, b_ in zip(outs[0], o):
            assert torch.equal(a_, b_), f"form {form} differs from pipe6 ({M}x{N}x{K})"


@pytest.mark.parametrize("M,N,K", [(116935, 5120, 1280), (60001, 4352, 1152), (2000, 1024, 1024), (4100, 768, 512)])
def test_gemm_fc1_compiled_epilogues_bit_identical(cuda, M, N, K):
    """The fc1 GEMMs as dispatched (pipe10, the epilogue compiled for its operand set: FOLD 1 LayerNorm
    fold, FOLD 2 bias) against pipe6 (form 47) and the run-time-branched epilogue (form 93), for every
    fc1 activation: bit-identical. Ragged M, fewer tiles than CUs; M * N >= 1M throughout (smaller
    shapes take the generic kernel)."""
    g = torch.Generator(device="cuda").manual_seed(M + N + K + 1)
    x = rnd(M, K, gen=g)
    w = rnd(N, K, scale=K ** -0.5, gen=g)
    b = rnd(N, scale=0.1, gen=g)
    gam = (1 + 0.1 * torch.randn(K, device="cuda", generator=g)).to(torch.bfloat16)
    bet = rnd(K, scale=0.1, gen=g)
    f = ops.LNFolded(w, b, gam, bet)
    st = ops.rowstats(x, 1e-6, d=K)
    for act in (_lib.ACT_GELU_TANH, _lib.ACT_QUICK_GELU, _lib.ACT_GELU_ERF):
        outs = []
        for form in (47, -1, 93):
            with ops.kernel_forms(**({} if form == -1 else {"gemm": form})):
                outs.append((ops.gemm_lnfold(x, f, st, act=act), ops.gemm(x, w, b, act=act)))
        torch.cuda.synchronize()
        for form, o in zip((-1, 93), outs[1:]):
            for a_, b_ in zip(outs[0], o):
                assert torch.equal(a_, b_), f"form {form} act {act} differs from pipe6 ({M}x{N}x{K})"


@pytest.mark.parametrize("M,N,K", [(4100, 4096, 1024), (20000, 8192, 2048)])
def test_gemm_geglu_compiled_epilogue_bit_identical(cuda, M, N, K):
    """ColPali's gate / up GEMM (GeGLU, bias, no residual) with the epilogue compiled for its
    operands (FOLD 2) against pipe6 (form 47) and the run-time form (93): bit-identical."""
    g = torch.Generator(device="cuda").manual_seed(M + N + K + 7)
    x = rnd(M, K, gen=g)
    w = rnd(N, K, scale=K ** -0.5, gen=g)
    b = rnd(N, scale=0.1, gen=g)
    outs = []
    for form in (47, -1, 93):
        with ops.kernel_forms(**({} if form == -1 else {"gemm": form})):
            outs.append(ops.gemm(x, w, b, act=_lib.ACT_GEGLU_TANH))
    torch.cuda.synchronize()
    for form, o in zip((-1, 93), outs[1:]):
        assert torch.equal(outs[0], o), f"GeGLU form {form} differs from pipe6 ({M}x{N}x{K})"


# mme_gemm_res_stats: the residual GEMM's output is bit-identical to mme_gemm's, and the
# row statistics reduced in its epilogue (64-column slices, Chan-combined) match a separate
# mme_rowstats pass over that output up to fp32 summation order. Shapes: split grid
# (N = 1152), whole 256-column tiles (N = 1280), the non-pipelined fallback (M * N < 1M),
# and a shifted residual stream (mean >> std: the two-pass slices keep the variance exact).
@pytest.mark.parametrize("M,N,K,shift", [(4096, 1152, 1152, 0.0), (3000, 1280, 512, 0.0), (100, 256, 64, 0.0),
                                         (2048, 1152, 4352, 40.0),
                                         (2048, 576, 256, 0.0),  # N % 256 == 64: partial last column tile
                                         (2048, 704, 256, 0.0),  # N % 256 == 192: odd slice count (11)
                                         (1500, 448, 320, 3.0)])
def test_gemm_res_stats(cuda, M, N, K, shift):
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    a = rnd(M, K, gen=g)
    w = rnd(N, K, scale=1 / math.sqrt(K), gen=g)
    b = rnd(N, scale=0.1, gen=g)
    x = (rnd(M, N, scale=2.0, gen=g).float() + shift).to(torch.bfloat16)
    ref_out = ops.gemm(a, w, b, residual=x)
    st = torch.empty(M, 2, dtype=torch.float32, device="cuda")
    part = torch.full((M, N // 64, 2), float("nan"), dtype=torch.float32, device="cuda")
    out = ops.gemm_res_stats(a, w, b, x.clone(), 1e-6, st, part)
    assert torch.equal(out, ref_out), "mme_gemm_res_stats output differs from mme_gemm"
    if M * N >= 1 << 20:  # the pipelined kernel's epilogue wrote every slice (not the fallback pass)
        assert torch.isfinite(part).all(), "fused epilogue statistics not written"
    ref_st = ops.rowstats(ref_out, 1e-6)
    torch.testing.assert_close(st[:, 0], ref_st[:, 0], rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(st[:, 1], ref_st[:, 1], rtol=1e-4, atol=0)
    # in place on the residual stream, as the encoder layers run it
    xi = x.clone()
    ops.gemm_res_stats(a, w, b, xi, 1e-6, st, part, out=xi)
    assert torch.equal(xi, ref_out)


# The LDS-staged statistics combine (production for an even slice count <= 20) runs the per-row
# kernel's arithmetic in the same order: bit-identical statistics (dev variant 48 = per-row form),
# including a ragged last block of rows.
@pytest.mark.parametrize("M,N,K", [(4096, 1152, 1152), (3001, 1280, 512), (2000, 1024, 256)])
def test_row_part_combine_lds_bit_identical(cuda, M, N, K):
    g = torch.Generator(device="cuda").manual_seed(M + 3 * N + K)
    a = rnd(M, K, gen=g)
    w = rnd(N, K, scale=1 / math.sqrt(K), gen=g)
    b = rnd(N, scale=0.1, gen=g)
    x = rnd(M, N, scale=2.0, gen=g)
    res = []
    for v in (-1, 48):
        st = torch.full((M, 2), float("nan"), dtype=torch.float32, device="cuda")
        part = torch.empty(M, N // 64, 2, dtype=torch.float32, device="cuda")
        with ops.kernel_forms(gemm=v):
            out = ops.gemm_res_stats(a, w, b, x.clone(), 1e-6, st, part)
        torch.cuda.synchronize()
        res.append((out, st))
    assert torch.equal(res[0][0], res[1][0])
    assert torch.isfinite(res[0][1]).all()
    assert torch.equal(res[0][1], res[1][1]), "LDS-staged combine differs from the per-row combine"


# pipe8 (production where K % 64 == 0 and K >= 192: 64-deep stages of whole-line rows in a
# 5-unit LDS ring) keeps pipe6's K-step order and per-MFMA k ranges, so its outputs are
# bit-identical to pipe6 (dev variant 47) on every epilogue: the ring's minimum depth
# (K = 192), ragged row bands, the split grid (N = 256 k + 128), K = 4352, folded LayerNorm,
# GeGLU, residual + fused statistics.
@pytest.mark.parametrize("M,N,K,epi", [(2048, 1024, 192, "bias"), (1500, 1536, 256, "gelu"),
                                       (4096, 1152, 1152, "res"), (1000, 3456, 1152, "lnfold"),
                                       (1024, 1152, 4352, "bias"), (2048, 4352, 320, "geglu"),
                                       (3000, 1152, 1152, "resstats"), (3000, 576, 320, "resstats"),
                                       (2048, 704, 256, "resstats"), (3000, 448, 320, "resstats")])
def test_gemm_pipe8_bit_identical_to_pipe6(cuda, M, N, K, epi):
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    a = rnd(M, K, scale=2.0, gen=g) + 0.5
    w = rnd(N, K, scale=1 / math.sqrt(K), gen=g)
    b = rnd(N, scale=0.1, gen=g)
    x = rnd(M, N, gen=g)
    if epi == "lnfold":
        fold = ops.LNFolded(w, b, (1.0 + 0.2 * torch.randn(K, generator=g, device="cuda")).to(torch.bfloat16),
                            rnd(K, scale=0.1, gen=g))
        stats = ops.rowstats(a, 1e-6)

    def run():
        if epi == "bias":
            return (ops.gemm(a, w, b),)
        if epi == "gelu":
            return (ops.gemm(a, w, b, act=_lib.ACT_GELU_TANH),)
        if epi == "res":
            return (ops.gemm(a, w, b, residual=x),)
        if epi == "lnfold":
            return (ops.gemm_lnfold(a, fold, stats, act=_lib.ACT_GELU_TANH),)
        if epi == "geglu":
            return (ops.gemm(a, w, b, act=_lib.ACT_GEGLU_TANH),)
        st = torch.empty(M, 2, dtype=torch.float32, device="cuda")
        part = torch.empty(M, N // 64, 2, dtype=torch.float32, device="cuda")
        out = ops.gemm_res_stats(a, w, b, x.clone(), 1e-6, st, part)
        return out, st

    new = run()
    with ops.kernel_forms(gemm=47):
        old = run()
    torch.cuda.synchronize()
    for n_, o_ in zip(new, old):
        assert torch.equal(n_, o_), f"pipe8 differs from pipe6 ({epi}, {M}x{N}x{K})"


def test_l2norm_bit_exact(cuda, golden):
    g = golden("l2norm")
    x = bits_to_bf16(g["x"]).cuda()
    y = ops.l2norm(x)
    assert np.array_equal(bf16_bits(y), g["y"]), "mme_l2norm differs from main.py:414 semantics"


def test_token_embed(cuda):
    g = torch.Generator(device="cuda").manual_seed(1)
    tok = rnd(1000, 256, gen=g)
    pos = rnd(20, 256, gen=g)
    ids = torch.randint(0, 1000, (3, 20), device="cuda", generator=g)
    out = ops.token_embed(ids, tok, pos)
    ref = (tok.float()[ids] + pos.float()[None]).to(torch.bfloat16).view(60, 256)
    assert torch.equal(out, ref)


def test_clip_embed_ln(cuda):
    g = torch.Generator(device="cuda").manual_seed(2)
    B, P, d = 3, 16, 320
    patch = rnd(B * P, d, gen=g)
    cls = rnd(d, gen=g)
    pos = rnd(P + 1, d, gen=g)
    gm, bt = rnd(d, gen=g), rnd(d, gen=g)
    out = ops.clip_embed_ln(patch, cls, pos, gm, bt, 1e-5, B, P)
    x = torch.cat([cls.view(1, 1, d).expand(B, 1, d), patch.view(B, P, d)], 1)
    x = (x.float() + pos.float()).to(torch.bfloat16).float()
    ref = torch.nn.functional.layer_norm(x, (d,), gm.float(), bt.float(), 1e-5).view(B * (P + 1), d)
    torch.testing.assert_close(out.float(), ref, atol=3e-2, rtol=1e-2)


def test_text_pool_rows(cuda):
    ids = torch.tensor([[5, 9, 7, 2, 2], [5, 3, 2, 8, 1], [1, 1, 1, 1, 1]], device="cuda")
    assert ops.text_pool_rows(ids, 2, 0).tolist() == [3, 5 + 2, 10 + 0]  # first eos (argmax of mask)
    assert ops.text_pool_rows(ids, 2, 1).tolist() == [1, 5 + 3, 10 + 0]  # argmax of ids (first max)
    assert ops.text_pool_rows(ids, 2, 2).tolist() == [4, 9, 14]


def test_im2col(cuda):
    pv = torch.randn(2, 3, 56, 56, device="cuda")
    out = ops.im2col(pv, 14, 640)
    ref = torch.nn.functional.unfold(pv, 14, stride=14).transpose(1, 2).reshape(2 * 16, 588)
    assert torch.equal(out[:, :588], ref.to(torch.bfloat16))
    assert not out[:, 588:].any()


# pipe9 (production since round 3: pipe8 without the per-stage scalar bookkeeping) is bit-identical
# to pipe8 with the per-wave epilogue (dev variant 71) on every epilogue it takes, at every peeling case of its stage loop
# (nk = K / 64 = 3 .. 8, 18, 68: empty / partial / full unrolled main loops) and the split grid
# (M * N >= 2^20 throughout: smaller products take the non-pipelined kernel in production).
@pytest.mark.dev
@pytest.mark.parametrize("M,N,K,epi", [(2048, 1024, 192, "bias"), (1500, 1536, 256, "gelu"), (1000, 1280, 320, "res"),
                                       (1500, 1024, 384, "lnfold"), (2048, 1152, 448, "bias"), (1024, 1024, 512, "res"),
                                       (4096, 1152, 1152, "res"), (1000, 3456, 1152, "lnfold"),
                                       (1024, 1152, 4352, "bias"), (3000, 4352, 1152, "gelu")])
def test_gemm_pipe9_bit_identical_to_pipe8(cuda, M, N, K, epi):
    g = torch.Generator(device="cuda").manual_seed(M + 2 * N + K)
    a = rnd(M, K, scale=2.0, gen=g) + 0.5
    w = rnd(N, K, scale=1 / math.sqrt(K), gen=g)
    b = rnd(N, scale=0.1, gen=g)
    x = rnd(M, N, gen=g)
    if epi == "lnfold":
        fold = ops.LNFolded(w, b, (1.0 + 0.2 * torch.randn(K, generator=g, device="cuda")).to(torch.bfloat16),
                            rnd(K, scale=0.1, gen=g))
        stats = ops.rowstats(a, 1e-6)

    def run():
        if epi == "bias":
            return ops.gemm(a, w, b)
        if epi == "gelu":
            return ops.gemm(a, w, b, act=_lib.ACT_GELU_TANH)
        if epi == "res":
            return ops.gemm(a, w, b, residual=x)
        return ops.gemm_lnfold(a, fold, stats, act=_lib.ACT_GELU_TANH)

    with ops.kernel_forms(gemm=71):
        ref = run()
    new = run()
    torch.cuda.synchronize()
    assert torch.equal(new, ref), f"pipe9 differs from pipe8 ({epi}, {M}x{N}x{K})"
