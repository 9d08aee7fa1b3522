"""Tensor-level wrappers over the libmme C ABI.

PyTorch is plumbing here: it owns device memory and streams. Every function
checks shapes / dtypes / devices on the host, then hands raw device pointers
and the current HIP stream to libmme. Nothing in this module computes on the
host or falls back to torch ops: a missing library or a CPU tensor raises.
"""
from __future__ import annotations

import contextlib
import math
import threading
from typing import Optional, Sequence

import torch

from . import _lib
from ._lib import call, query

BF16 = torch.bfloat16

_forms = threading.local()


@contextlib.contextmanager
def kernel_forms(**forms: int):
    """Kernel forms for the calls this thread makes inside the block (bit-identity tests, A/B):
    gemm=47 (pipe6) / 48 (per-row statistics combine), mx=0 / 2 / 3 / 10 (earlier mx GEMM forms),
    attention=30 + kind (force an attention kernel kind), attention_long=30 + kind (the same for calls
    with T > 128 only, i.e. the vision towers: a job A/B that leaves text attention alone). Each call passes its form to the library
    through the mme_*_form entry points; the library itself holds no switch."""
    old = dict(getattr(_forms, "d", {}))
    _forms.d = {**old, **forms}
    try:
        yield
    finally:
        _forms.d = old


def _form(name: str) -> Optional[int]:
    return getattr(_forms, "d", {}).get(name)


def _call_form(entry: str, family: str, *args) -> None:
    """call(entry, *args), or call(entry + "_form", form, *args) when this thread set a form."""
    f = _form(family)
    if f is None:
        call(entry, *args)
    else:
        call(entry + "_form", int(f), *args)


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def _dev(*ts: Optional[torch.Tensor]) -> None:
    for t in ts:
        if t is not None and not t.is_cuda:
            raise ValueError("mme ops take device tensors (got a CPU tensor); there is no host fallback")


def _rowmajor(t: torch.Tensor, name: str) -> int:
    """Return the leading dimension of a 2-D tensor with unit column stride."""
    if t.dim() != 2 or t.stride(1) != 1:
        raise ValueError(f"{name}: expected a 2-D tensor with contiguous rows, got shape {tuple(t.shape)} "
                         f"stride {t.stride()}")
    return t.stride(0)


class Workspace:
    """Grow-only device scratch buffer (one per stream/user)."""

    def __init__(self) -> None:
        self.buf: Optional[torch.Tensor] = None

    def get(self, nbytes: int, device) -> torch.Tensor:
        nbytes = max(256, int(nbytes))
        if self.buf is None or self.buf.numel() < nbytes or self.buf.device != torch.device(device):
            self.buf = torch.empty(nbytes, dtype=torch.uint8, device=device)
        return self.buf


_ws = Workspace()


class KernelTimer:
    """Optional HIP-event timing of libmme launches (bench.py's roofline).

    When enabled, each timed op records a start/end event pair on the stream it
    launches on and the op's algorithmic FLOPs; summary() syncs once and
    aggregates. Disabled (the default) it costs one attribute check."""

    enabled = False
    records = []
    _pool = []   # timing events, created once and re-recorded by every timed step
    _used = 0

    @classmethod
    def start(cls):
        cls.records = []
        cls._used = 0
        cls.enabled = True

    @classmethod
    def stop(cls):
        cls.enabled = False

    @classmethod
    def reserve(cls, n: int):
        """Create the timing events up front (no hipEventCreate inside a timed region)."""
        while len(cls._pool) < n:
            cls._pool.append(torch.cuda.Event(enable_timing=True))

    @classmethod
    def used(cls) -> int:
        return cls._used

    @classmethod
    def _event(cls):
        if cls._used == len(cls._pool):
            cls._pool.append(torch.cuda.Event(enable_timing=True))
        ev = cls._pool[cls._used]
        cls._used += 1
        return ev

    @classmethod
    def begin(cls):
        if not cls.enabled:
            return None
        ev = cls._event()
        ev.record()
        return ev

    @classmethod
    def end(cls, ev, name: str, flops: float, nbytes: float = 0.0):
        if ev is None:
            return
        e = cls._event()
        e.record()
        cls.records.append((name, ev, e, flops, nbytes))

    @classmethod
    def summary(cls):
        torch.cuda.synchronize()
        out = {}
        for name, s, e, fl, nb in cls.records:
            d = out.setdefault(name, {"launches": 0, "ms": 0.0, "flops": 0.0, "bytes": 0.0})
            d["launches"] += 1
            d["ms"] += s.elapsed_time(e)
            d["flops"] += fl
            d["bytes"] += nb
        return out


# ---------------------------------------------------------------- GEMM / norms
def gemm(a: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None, *,
         residual: Optional[torch.Tensor] = None, res_period: int = 0, act: int = _lib.ACT_NONE,
         out: Optional[torch.Tensor] = None, out_f32: bool = False,
         algo_flops: Optional[float] = None) -> torch.Tensor:
    """out = act(a @ w.T + bias) + residual[row % res_period or row]  (bf16, fp32 accumulate).

    a: [M, K] bf16, w: [N, K] bf16 (nn.Linear layout), K % 64 == 0.
    algo_flops: the algorithmic FLOPs of this product when the operands carry
    zero padding (KernelTimer accounting only; default 2*M*N*K).
    """
    _dev(a, w, bias, residual, out)
    M, K = a.shape
    N = w.shape[0]
    if w.shape[1] != K:
        raise ValueError(f"gemm: a is [*, {K}] but w is {tuple(w.shape)}")
    n_out = N // 2 if act == _lib.ACT_GEGLU_TANH else N  # gated: gate/up rows interleaved by 4 (mme.h)
    if out is None:
        out = torch.empty(M, n_out, dtype=torch.float32 if out_f32 else BF16, device=a.device)
    lda, ldb, ldc = _rowmajor(a, "a"), _rowmajor(w, "w"), _rowmajor(out, "out")
    ldr = 0
    if residual is not None:
        ldr = _rowmajor(residual, "residual")
    if bias is not None and bias.numel() < N:
        raise ValueError("gemm: bias shorter than N")
    ev = KernelTimer.begin()
    _call_form("mme_gemm", "gemm", a.data_ptr(), lda, w.data_ptr(), ldb, out.data_ptr(), ldc, M, N, K, _ptr(bias),
         _ptr(residual), ldr, res_period, act, int(out_f32), _stream())
    res_bytes = 2.0 * M * N if residual is not None else 0.0
    KernelTimer.end(ev, "gemm", algo_flops if algo_flops is not None else 2.0 * M * N * K,
                    2.0 * (M * K + N * K + M * n_out) + res_bytes)
    return out


def gemm_res_stats(a: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor], residual: torch.Tensor,
                   eps: float, stats: torch.Tensor, part: torch.Tensor, *, out: Optional[torch.Tensor] = None,
                   algo_flops: Optional[float] = None) -> torch.Tensor:
    """out = a @ w.T + bias + residual (bf16) and stats = rowstats(out, eps), the statistics
    reduced in the GEMM epilogue (mme_gemm_res_stats). part: fp32 scratch >= [M, N / 64, 2]."""
    _dev(a, w, bias, residual, stats, part, out)
    M, K = a.shape
    N = w.shape[0]
    if w.shape[1] != K or residual.shape[0] < M or stats.shape[0] < M:
        raise ValueError(f"gemm_res_stats: a {tuple(a.shape)} vs w {tuple(w.shape)} / residual / stats")
    if N % 64 or part.dtype != torch.float32 or not part.is_contiguous() or part.numel() < M * (N // 64) * 2:
        raise ValueError("gemm_res_stats: N % 64 != 0 or part is not contiguous fp32 >= [M, N / 64, 2]")
    if stats.dtype != torch.float32 or not stats.is_contiguous():
        raise ValueError("gemm_res_stats: stats must be contiguous fp32 [M, 2]")
    if bias is not None and bias.numel() < N:
        raise ValueError("gemm_res_stats: bias shorter than N")
    if out is None:
        out = torch.empty(M, N, dtype=BF16, device=a.device)
    ev = KernelTimer.begin()
    _call_form("mme_gemm_res_stats", "gemm", a.data_ptr(), _rowmajor(a, "a"), w.data_ptr(), _rowmajor(w, "w"), out.data_ptr(),
         _rowmajor(out, "out"), M, N, K, _ptr(bias), residual.data_ptr(), _rowmajor(residual, "residual"),
         float(eps), part.data_ptr(), stats.data_ptr(), _stream())
    # the "gemm" family's time includes the statistics combine pass (row_part_combine_kernel, one
    # launch inside this C-ABI call); its bytes: residual read, the per-slice (mean, M2) pairs
    # written by the GEMM epilogue and read back by the combine, and the [M, 2] statistics
    KernelTimer.end(ev, "gemm", algo_flops if algo_flops is not None else 2.0 * M * N * K,
                    2.0 * (M * K + N * K + M * N) + 2.0 * M * N + 2 * 8.0 * M * (N // 64) + 8.0 * M)
    return out


def rowstats(x: torch.Tensor, eps: float, *, d: Optional[int] = None,
             out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """LayerNorm statistics [rows, 2] fp32 = (mean, rsqrt(var + eps)) over the first d columns."""
    _dev(x, out)
    rows = x.shape[0]
    d = d or x.shape[1]
    if out is None:
        out = torch.empty(rows, 2, dtype=torch.float32, device=x.device)
    if out.dtype != torch.float32 or not out.is_contiguous() or out.numel() < 2 * rows:
        raise ValueError("rowstats: out must be contiguous fp32 [rows, 2]")
    ev = KernelTimer.begin()
    call("mme_rowstats", x.data_ptr(), _rowmajor(x, "x"), rows, d, float(eps), out.data_ptr(), _stream())
    KernelTimer.end(ev, "rowstats", 0.0, 2.0 * rows * d + 8.0 * rows)  # HBM-bound: rows read, 8 B per row out
    return out


def gemm_lnfold(x: torch.Tensor, folded: "LNFolded", stats: torch.Tensor, *, act: int = _lib.ACT_NONE,
                out: Optional[torch.Tensor] = None, algo_flops: Optional[float] = None) -> torch.Tensor:
    """act(LayerNorm(x) @ W.T + b) with the LayerNorm folded into the weights (mme_gemm_lnfold):
    x is the raw residual stream, stats its rowstats()."""
    _dev(x, folded.w, stats, out)
    M, K = x.shape
    N = folded.w.shape[0]
    if folded.w.shape[1] != K or stats.shape[0] < M:
        raise ValueError(f"gemm_lnfold: x {tuple(x.shape)} vs w {tuple(folded.w.shape)} / stats {tuple(stats.shape)}")
    if out is None:
        out = torch.empty(M, N, dtype=BF16, device=x.device)
    ev = KernelTimer.begin()
    _call_form("mme_gemm_lnfold", "gemm", x.data_ptr(), _rowmajor(x, "x"), folded.w.data_ptr(), _rowmajor(folded.w, "w"),
         out.data_ptr(), _rowmajor(out, "out"), M, N, K, stats.data_ptr(), folded.cs.data_ptr(),
         folded.b.data_ptr(), act, _stream())
    KernelTimer.end(ev, "gemm", algo_flops if algo_flops is not None else 2.0 * M * N * K,
                    2.0 * (M * K + N * K + M * N))
    return out


def attention_q_scale(hd: int, scale: Optional[float] = None) -> float:
    """The factor mme_attention_qs expects in the Q columns: scale * log2(e) (scale = hd^-0.5)."""
    return (hd ** -0.5 if scale is None else scale) * 1.4426950408889634


class LNFolded:
    """nn.LayerNorm(gamma, beta) followed by nn.Linear(w, bias), folded for mme_gemm_lnfold:
    w' = bf16(w * gamma) (per input column), cs = sum_k w'[n, k] (fp32), b' = bias + w . beta (fp32).
    row_scale (fp32 [N], optional) multiplies output row n of the linear map before w' is rounded
    (the attention's Q rows by attention_q_scale: one bf16 rounding, as without it)."""

    def __init__(self, w: torch.Tensor, bias: Optional[torch.Tensor], gamma: torch.Tensor, beta: torch.Tensor,
                 row_scale: Optional[torch.Tensor] = None):
        K = w.shape[1]
        g = torch.zeros(K, dtype=torch.float32, device=w.device)
        bt = torch.zeros(K, dtype=torch.float32, device=w.device)
        g[: gamma.numel()] = gamma.float()  # K may be zero-padded past the LayerNorm width
        bt[: beta.numel()] = beta.float()
        wf = w.float()
        bf = bias.float() if bias is not None else None
        if row_scale is not None:
            rs = row_scale.float().to(w.device)
            wf = wf * rs[:, None]
            bf = bf * rs[: bf.numel()] if bf is not None else None
        self.w = (wf * g).to(BF16).contiguous()
        self.cs = self.w.float().sum(dim=1).contiguous()
        b = wf @ bt
        if bf is not None:
            b[: bf.numel()] += bf[: b.numel()]
        self.b = b.contiguous()


def layernorm(x: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor, eps: float, *,
              rows_idx: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None,
              d: Optional[int] = None) -> torch.Tensor:
    """LayerNorm over the first `d` columns of each row (optionally of rows x[rows_idx])."""
    _dev(x, gamma, beta, rows_idx, out)
    d = d or gamma.numel()
    rows = rows_idx.numel() if rows_idx is not None else x.shape[0]
    if out is None:
        out = torch.empty(rows, d, dtype=BF16, device=x.device)
    if rows_idx is not None and rows_idx.dtype != torch.int32:
        raise ValueError("layernorm: rows_idx must be int32")
    ev = KernelTimer.begin()
    call("mme_layernorm", x.data_ptr(), _rowmajor(x, "x"), gamma.data_ptr(), beta.data_ptr(), out.data_ptr(),
         _rowmajor(out, "out"), rows, d, float(eps), _ptr(rows_idx), _stream())
    KernelTimer.end(ev, "layernorm", 0.0, 4.0 * rows * d + 4.0 * d)  # rows in + out bf16, gamma / beta
    return out


def l2norm(x: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """bf16(x / bf16(||x||)) per row — main.py:414,434 semantics."""
    _dev(x, out)
    rows, d = x.shape
    if out is None:
        out = torch.empty(rows, d, dtype=BF16, device=x.device)
    ev = KernelTimer.begin()
    call("mme_l2norm", x.data_ptr(), _rowmajor(x, "x"), out.data_ptr(), _rowmajor(out, "out"), rows, d, _stream())
    KernelTimer.end(ev, "l2norm", 0.0, 4.0 * rows * d)
    return out


# ---------------------------------------------------------------- attention
def attention(qkv: torch.Tensor, B: int, T: int, H: int, hd: int, *, seq_lens: Optional[torch.Tensor] = None,
              causal: bool = False, scale: Optional[float] = None, out: Optional[torch.Tensor] = None,
              q_prescaled: bool = False) -> torch.Tensor:
    """softmax(Q K^T scale + mask) V per head (mme_attention). q_prescaled: the Q columns already hold
    q * scale * log2(e) (LNFolded(row_scale=attention_q_scale(hd)) on the projection; mme_attention_qs),
    and `scale` is not used."""
    _dev(qkv, seq_lens, out)
    if qkv.shape[0] != B * T:
        raise ValueError(f"attention: qkv has {qkv.shape[0]} rows, expected B*T={B * T}")
    if out is None:
        out = torch.empty(B * T, H * hd, dtype=BF16, device=qkv.device)
    if seq_lens is not None and (seq_lens.dtype != torch.int32 or seq_lens.numel() != B):
        raise ValueError("attention: seq_lens must be int32 [B]")
    scale = hd ** -0.5 if scale is None else scale
    ev = KernelTimer.begin()
    fl = _form("attention_long") if T > 128 else None  # a job A/B of the long-sequence (vision) kernel only
    entry = "mme_attention_qs" if q_prescaled else "mme_attention"
    args = (qkv.data_ptr(), _rowmajor(qkv, "qkv"), out.data_ptr(), _rowmajor(out, "out"), B, T, H, hd,
            _ptr(seq_lens), int(causal)) + (() if q_prescaled else (float(scale),)) + (_stream(),)
    if fl is not None:
        call(entry + "_form", int(fl), *args)
    else:
        _call_form(entry, "attention", *args)
    # T <= 64 (SigLIP text) runs attn_short_kernel: one key tile per (batch, head), HBM-bound (Q, K, V in, O out);
    # 64 < T <= 128 at head dim 64 (the CLIP causal text towers, round 6) attn_short2_kernel, HBM-bound as well
    fam = "attention_short" if T <= 64 else "attention_short2" if (T <= 128 and hd == 64) else "attention"
    KernelTimer.end(ev, fam, 4.0 * B * H * T * T * hd * (0.5 if causal else 1.0), 8.0 * B * T * H * hd)
    return out


def probe_attention(q: torch.Tensor, kv: torch.Tensor, B: int, T: int, H: int, hd: int, *,
                    scale: Optional[float] = None, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    _dev(q, kv, out)
    if out is None:
        out = torch.empty(B, H * hd, dtype=BF16, device=kv.device)
    scale = hd ** -0.5 if scale is None else scale
    call("mme_probe_attention", q.data_ptr(), kv.data_ptr(), _rowmajor(kv, "kv"), out.data_ptr(),
         _rowmajor(out, "out"), B, T, H, hd, float(scale), _stream())
    return out


def map_pool(S: torch.Tensor, x: torch.Tensor, B: int, T: int, H: int, *,
             out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """SigLIP MAP head, probe absorbed (mme_map_pool): S fp32 [B*T, >= 2H] (x . [U_hi; U_lo]^T),
    x bf16 [B*T, D] -> bf16 [B*H, D], row b*H + h = sum_t softmax_t(S[., h] + S[., H + h]) x_t."""
    _dev(S, x, out)
    D = x.shape[1]
    if S.dtype != torch.float32 or S.shape[0] < B * T or x.shape[0] < B * T:
        raise ValueError(f"map_pool: S {tuple(S.shape)} {S.dtype} / x {tuple(x.shape)} vs B*T = {B * T}")
    if out is None:
        out = torch.empty(B * H, D, dtype=BF16, device=x.device)
    call("mme_map_pool", S.data_ptr(), _rowmajor(S, "S"), x.data_ptr(), _rowmajor(x, "x"), out.data_ptr(),
         _rowmajor(out, "out"), B, T, H, D, _stream())
    return out


# ---------------------------------------------------------------- Gemma / ColPali pieces
def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float, *, unit_offset: bool = True,
            out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """GemmaRMSNorm: bf16(x * rsqrt(mean x^2 + eps) * (1 + w)) with fp32 statistics."""
    _dev(x, w, out)
    rows, d = x.shape[0], w.numel()
    if out is None:
        out = torch.empty(rows, d, dtype=BF16, device=x.device)
    call("mme_rmsnorm", x.data_ptr(), _rowmajor(x, "x"), w.data_ptr(), out.data_ptr(), _rowmajor(out, "out"), rows, d,
         float(eps), int(unit_offset), None, _stream())
    return out


def rope_(qkv: torch.Tensor, T: int, nheads: int, hd: int, pos_offset: int, theta: float) -> torch.Tensor:
    """Rotary embedding in place on heads [0, nheads) of packed rows (position = row % T + pos_offset)."""
    _dev(qkv)
    call("mme_rope", qkv.data_ptr(), _rowmajor(qkv, "qkv"), qkv.shape[0], T, nheads, hd, int(pos_offset),
         float(theta), _stream())
    return qkv


def gemma_embed(ids: torch.Tensor, tok: torch.Tensor, scale: float, *, img: Optional[torch.Tensor] = None,
                img_prefix: int = 0, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Decoder input rows: image features for t < img_prefix, bf16(tok[id] * scale) otherwise."""
    _dev(ids, tok, img, out)
    if ids.dtype != torch.int64 or ids.dim() != 2:
        raise ValueError("gemma_embed: ids must be int64 [B, L]")
    ids = ids.contiguous()
    B, L = ids.shape
    d = tok.shape[1]
    if img_prefix and (img is None or img.shape[0] != B * img_prefix):
        raise ValueError(f"gemma_embed: image features must be [B*{img_prefix}, d]")
    if out is None:
        out = torch.empty(B * L, d, dtype=BF16, device=ids.device)
    call("mme_gemma_embed", ids.data_ptr(), B, L, tok.data_ptr(), d, float(scale), _ptr(img),
         _rowmajor(img, "img") if img is not None else 0, int(img_prefix), out.data_ptr(), _rowmajor(out, "out"),
         _stream())
    return out


def l2norm_masked(x: torch.Tensor, mask: Optional[torch.Tensor], out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """bf16(bf16(x / bf16||x||) * mask[row]); mask int64 per row (the flattened attention_mask)."""
    _dev(x, mask, out)
    rows, d = x.shape
    if mask is not None and (mask.dtype != torch.int64 or mask.numel() != rows):
        raise ValueError("l2norm_masked: mask must be int64 with one entry per row")
    if out is None:
        out = torch.empty(rows, d, dtype=BF16, device=x.device)
    call("mme_l2norm_masked", x.data_ptr(), _rowmajor(x, "x"), out.data_ptr(), _rowmajor(out, "out"), rows, d,
         _ptr(mask.contiguous() if mask is not None else None), _stream())
    return out


def attention_mqa(qkv: torch.Tensor, B: int, T: int, Hq: int, hd: int, *, kstart: Optional[torch.Tensor] = None,
                  kend: Optional[torch.Tensor] = None, scale: Optional[float] = None,
                  out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Bidirectional multi-query attention (one K/V head) over packed [q heads | k | v] rows."""
    _dev(qkv, kstart, kend, out)
    if qkv.shape[0] != B * T:
        raise ValueError(f"attention_mqa: qkv has {qkv.shape[0]} rows, expected B*T={B * T}")
    for t in (kstart, kend):
        if t is not None and (t.dtype != torch.int32 or t.numel() != B):
            raise ValueError("attention_mqa: kstart / kend must be int32 [B]")
    if out is None:
        out = torch.empty(B * T, Hq * hd, dtype=BF16, device=qkv.device)
    scale = hd ** -0.5 if scale is None else scale
    ev = KernelTimer.begin()
    call("mme_attention_mqa", qkv.data_ptr(), _rowmajor(qkv, "qkv"), out.data_ptr(), _rowmajor(out, "out"), B, T, Hq,
         hd, _ptr(kstart), _ptr(kend), float(scale), _stream())
    KernelTimer.end(ev, "attention", 4.0 * B * Hq * T * T * hd)
    return out


# ---------------------------------------------------------------- embeddings
def token_embed(ids: torch.Tensor, tok: torch.Tensor, pos: torch.Tensor, out: Optional[torch.Tensor] = None):
    _dev(ids, tok, pos, out)
    if ids.dtype != torch.int64 or ids.dim() != 2:
        raise ValueError("token_embed: ids must be int64 [B, L]")
    B, L = ids.shape
    d = tok.shape[1]
    if L > pos.shape[0]:
        raise ValueError(f"token_embed: sequence length {L} exceeds max_position_embeddings {pos.shape[0]}")
    ids = ids.contiguous()
    if out is None:
        out = torch.empty(B * L, d, dtype=BF16, device=ids.device)
    call("mme_token_embed", ids.data_ptr(), B, L, tok.data_ptr(), pos.data_ptr(), d, out.data_ptr(),
         _rowmajor(out, "out"), _stream())
    return out


def clip_embed_ln(patch: torch.Tensor, cls: torch.Tensor, pos: torch.Tensor, gamma, beta, eps: float, B: int, P: int,
                  out: Optional[torch.Tensor] = None):
    _dev(patch, cls, pos, gamma, beta, out)
    d = cls.numel()
    if out is None:
        out = torch.empty(B * (P + 1), d, dtype=BF16, device=patch.device)
    call("mme_clip_embed_ln", patch.data_ptr(), _rowmajor(patch, "patch"), cls.data_ptr(), pos.data_ptr(),
         gamma.data_ptr(), beta.data_ptr(), float(eps), out.data_ptr(), _rowmajor(out, "out"), B, P, d, _stream())
    return out


def text_pool_rows(ids: torch.Tensor, eos_id: int, mode: int) -> torch.Tensor:
    """Row index (b*L + pos) of the pooled token per sequence (mode 0 eos, 1 argmax, 2 last)."""
    _dev(ids)
    B, L = ids.shape
    ids = ids.contiguous()
    rows = torch.empty(B, dtype=torch.int32, device=ids.device)
    call("mme_text_pool_rows", ids.data_ptr(), B, L, int(eos_id), int(mode), rows.data_ptr(), _stream())
    return rows


# ---------------------------------------------------------------- image preprocessing
def preprocess_u8(imgs: torch.Tensor, *, resize: Sequence[int], crop: Sequence[int], size: int,
                  mean: Sequence[float], std: Sequence[float], patch: int = 0, kpad: int = 0) -> torch.Tensor:
    """PIL-exact bicubic resize + crop + rescale + normalise of u8 NHWC images on the device.

    patch == 0 -> pixel_values fp32 [n,3,S,S]; patch > 0 -> bf16 im2col patches [n*(S/p)^2, kpad].
    """
    _dev(imgs)
    if imgs.dtype != torch.uint8 or imgs.dim() != 4 or imgs.shape[3] != 3:
        raise ValueError("preprocess_u8: expected uint8 [n, H, W, 3]")
    imgs = imgs.contiguous()
    n, H, W, _ = imgs.shape
    rh, rw = resize
    top, left = crop
    S = size
    dev = imgs.device
    wsb = query("mme_preprocess_workspace_bytes", n, H, W, rh, rw)
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
    if patch:
        G = S // patch
        out = torch.empty(n * G * G, kpad, dtype=BF16, device=dev)
        kind = _lib.PIX_PATCHES
    else:
        out = torch.empty(n, 3, S, S, dtype=torch.float32, device=dev)
        kind = _lib.PIX_F32_NCHW
    # mean/std are HOST float[3] (copied by value into the kernel arguments)
    mean_h = torch.tensor(list(mean), dtype=torch.float32)
    std_h = torch.tensor(list(std), dtype=torch.float32)
    ev = KernelTimer.begin()
    call("mme_preprocess_u8", imgs.data_ptr(), n, H, W, rh, rw, top, left, S, mean_h.data_ptr(), std_h.data_ptr(),
         kind, patch, kpad, out.data_ptr(), ws.data_ptr(), wsb, _stream())
    # algorithmic bytes: the u8 images in, the bf16 patches (3 p^2 of each kpad-wide row) / fp32 pixels out
    out_b = n * (S // patch) ** 2 * 3 * patch * patch * 2.0 if patch else n * 3 * S * S * 4.0
    KernelTimer.end(ev, "preprocess", 0.0, float(n * H * W * 3) + out_b)
    return out


def im2col(pixels: torch.Tensor, patch: int, kpad: int) -> torch.Tensor:
    _dev(pixels)
    if pixels.dim() != 4 or pixels.shape[1] != 3 or pixels.shape[2] != pixels.shape[3]:
        raise ValueError("im2col: expected pixel_values [n, 3, S, S]")
    if pixels.dtype not in (torch.float32, BF16):
        pixels = pixels.float()
    pixels = pixels.contiguous()
    n, _, S, _ = pixels.shape
    G = S // patch
    out = torch.empty(n * G * G, kpad, dtype=BF16, device=pixels.device)
    call("mme_im2col", pixels.data_ptr(), int(pixels.dtype == torch.float32), n, S, patch, kpad, out.data_ptr(),
         _stream())
    return out


# ---------------------------------------------------------------- retrieval
def sim_topk(q: torch.Tensor, d: torch.Tensor, k: int, col_offset: int = 0):
    """Top-k columns of q @ d.T per row: (idx int32 [nq,k], score fp32 [nq,k]), order (score desc, idx asc)."""
    _dev(q, d)
    nq, D = q.shape
    nd = d.shape[0]
    if D % 64:  # the kernel's K loop takes 64-deep steps: zero columns leave every dot product unchanged
        Dp = -(-D // 64) * 64
        q = torch.nn.functional.pad(q, (0, Dp - D))
        d = torch.nn.functional.pad(d, (0, Dp - D))
        D = Dp
    idx = torch.empty(nq, k, dtype=torch.int32, device=q.device)
    sc = torch.empty(nq, k, dtype=torch.float32, device=q.device)
    wsb = query("mme_sim_topk_workspace_bytes", nq, nd, k)
    ws = _ws.get(wsb, q.device)
    call("mme_sim_topk", q.data_ptr(), _rowmajor(q, "q"), d.data_ptr(), _rowmajor(d, "d"), nq, nd, D, k, col_offset,
         idx.data_ptr(), sc.data_ptr(), ws.data_ptr(), ws.numel(), _stream())
    return idx, sc


def topk_merge(idx: torch.Tensor, score: torch.Tensor, parts: int, k: int):
    """Merge `parts` top-k lists per row: inputs [rows, parts*k]."""
    _dev(idx, score)
    rows = idx.shape[0]
    idx = idx.contiguous()
    score = score.contiguous()
    oi = torch.empty(rows, k, dtype=torch.int32, device=idx.device)
    os_ = torch.empty(rows, k, dtype=torch.float32, device=idx.device)
    call("mme_topk_merge", idx.data_ptr(), score.data_ptr(), rows, parts, k, oi.data_ptr(), os_.data_ptr(),
         _stream())
    return oi, os_


def topk_rows(scores: torch.Tensor, k: int, col_offset: int = 0):
    """Row top-k of an fp32 score matrix: (idx int32 [rows,k], score fp32 [rows,k]), order (score desc, idx asc)."""
    _dev(scores)
    if scores.dtype != torch.float32:
        raise ValueError("topk_rows: scores must be fp32")
    rows, cols = scores.shape
    idx = torch.empty(rows, k, dtype=torch.int32, device=scores.device)
    sc = torch.empty(rows, k, dtype=torch.float32, device=scores.device)
    call("mme_topk_rows", scores.data_ptr(), _rowmajor(scores, "scores"), rows, cols, k, col_offset, idx.data_ptr(),
         sc.data_ptr(), _stream())
    return idx, sc


def topk_rows_torch(scores: torch.Tensor, k: int, col_offset: int = 0):
    """Row top-k in torch.topk's CPU order (main.py:335,365,375): (idx int32 [rows,k], score fp32
    [rows,k]). Exact ties come out as torch's libstdc++ partial_sort / nth_element leaves them."""
    _dev(scores)
    if scores.dtype != torch.float32:
        raise ValueError("topk_rows_torch: scores must be fp32")
    rows, cols = scores.shape
    idx = torch.empty(rows, k, dtype=torch.int32, device=scores.device)
    sc = torch.empty(rows, k, dtype=torch.float32, device=scores.device)
    ws_bytes = query("mme_topk_rows_torch_workspace_bytes", rows, cols, k)
    ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=scores.device)
    call("mme_topk_rows_torch", scores.data_ptr(), _rowmajor(scores, "scores"), rows, cols, k, col_offset,
         idx.data_ptr(), sc.data_ptr(), ws.data_ptr(), ws_bytes, _stream())
    return idx, sc


def recall_hits_torch(scores: torch.Tensor, tgt_count: int, ks: Sequence[int], row_offset: int = 0) -> torch.Tensor:
    """int64 [len(ks)]: rows whose torch.topk(row, min(k, cols)) holds a target column -- one selection
    per k, as compute_metrics_detailed calls torch.topk (main.py:331-378)."""
    cols = scores.shape[1]
    hits = torch.zeros(len(ks), dtype=torch.int64, device=scores.device)
    for j, k in enumerate(ks):
        kk = min(k, cols)
        idx, _ = topk_rows_torch(scores, kk)
        hits[j:j + 1] = recall_hits(idx, tgt_count, [kk], row_offset=row_offset)
    return hits


def gather_scores(S: torch.Tensor, rows: torch.Tensor, cols: torch.Tensor, g: int = 1,
                  out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """out[b*R + i, p] = S[rows[b, i], g*cols[b, p // g] + p % g]  (fp32 [B*R, C*g])."""
    _dev(S, rows, cols, out)
    if S.dtype != torch.float32 or rows.dtype != torch.int32 or cols.dtype != torch.int32:
        raise ValueError("gather_scores: S fp32, rows / cols int32")
    B, R = rows.shape
    C = cols.shape[1]
    if cols.shape[0] != B:
        raise ValueError("gather_scores: rows / cols batch mismatch")
    if out is None:
        out = torch.empty(B * R, C * g, dtype=torch.float32, device=S.device)
    call("mme_gather_scores", S.data_ptr(), _rowmajor(S, "S"), rows.contiguous().data_ptr(),
         cols.contiguous().data_ptr(), B, R, C, g, out.data_ptr(), _stream())
    return out


def recall_hits_groups(topk_idx: torch.Tensor, R: int, tgt_count: int, ks: Sequence[int]) -> torch.Tensor:
    """int64 [rows // R, len(ks)]: per group of R rows, rows whose first ks[j] indices hold a target."""
    _dev(topk_idx)
    rows, k = topk_idx.shape
    kk = torch.tensor(list(ks), dtype=torch.int32, device=topk_idx.device)
    hits = torch.zeros(rows // R, len(ks), dtype=torch.int64, device=topk_idx.device)
    call("mme_recall_hits_groups", topk_idx.contiguous().data_ptr(), rows, k, R, tgt_count, kk.data_ptr(), len(ks),
         hits.data_ptr(), _stream())
    return hits


def winoground(text: torch.Tensor, image: torch.Tensor):
    """(scores fp32 [n, 4] = bf16 <t_a, i_b> for ab = 00,01,10,11, counts int64 [3] text/image/group)."""
    _dev(text, image)
    if text.shape != image.shape or text.dim() != 3 or text.shape[1] != 2:
        raise ValueError("winoground: text / image must both be [n, 2, D]")
    n, _, D = text.shape
    text, image = text.to(BF16).contiguous(), image.to(BF16).contiguous()
    scores = torch.empty(n, 4, dtype=torch.float32, device=text.device)
    counts = torch.zeros(3, dtype=torch.int64, device=text.device)
    call("mme_winoground", text.data_ptr(), image.data_ptr(), n, D, scores.data_ptr(), counts.data_ptr(), _stream())
    return scores, counts


def recall_hits(topk_idx: torch.Tensor, tgt_count: int, ks: Sequence[int], *, tgt_start: Optional[torch.Tensor] = None,
                row_offset: int = 0, hits: Optional[torch.Tensor] = None,
                skip: Optional[torch.Tensor] = None) -> torch.Tensor:
    """int64 [len(ks)] counts of rows whose first ks[j] indices contain a target column (rows with
    skip[r] != 0 not counted)."""
    _dev(topk_idx, tgt_start, hits, skip)
    rows, k = topk_idx.shape
    if tgt_start is not None and (tgt_start.dtype != torch.int32 or tgt_start.numel() != rows):
        raise ValueError("recall_hits: tgt_start must be int32 [rows]")
    if skip is not None and (skip.dtype != torch.uint8 or skip.numel() != rows):
        raise ValueError("recall_hits: skip must be uint8 [rows]")
    kk = torch.tensor(list(ks), dtype=torch.int32, device=topk_idx.device)
    if hits is None:
        hits = torch.zeros(len(ks), dtype=torch.int64, device=topk_idx.device)
    call("mme_recall_hits", topk_idx.contiguous().data_ptr(), rows, k, _ptr(tgt_start), tgt_count, row_offset,
         kk.data_ptr(), len(ks), _ptr(skip), hits.data_ptr(), _stream())
    return hits


def tie_rows(scores: torch.Tensor) -> torch.Tensor:
    """uint8 [rows]: 1 where a sorted top-k score row holds two exactly equal neighbours."""
    _dev(scores)
    if scores.dtype != torch.float32 or not scores.is_contiguous():
        raise ValueError("tie_rows: scores must be contiguous fp32 [rows, k]")
    rows, k = scores.shape
    flags = torch.empty(rows, dtype=torch.uint8, device=scores.device)
    call("mme_tie_rows", scores.data_ptr(), rows, k, flags.data_ptr(), _stream())
    return flags


def sim_scores(q: torch.Tensor, d: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """fp32 [nq, nd] = q @ d.T through mme_sim_topk's own main loop (scores bit-identical to the ones
    sim_topk ranks)."""
    _dev(q, d, out)
    nq, D = q.shape
    nd = d.shape[0]
    if d.shape[1] != D:
        raise ValueError("sim_scores: width mismatch")
    if D % 64:
        Dp = -(-D // 64) * 64
        q = torch.nn.functional.pad(q, (0, Dp - D))
        d = torch.nn.functional.pad(d, (0, Dp - D))
        D = Dp
    if out is None:
        out = torch.empty(nq, nd, dtype=torch.float32, device=q.device)
    if out.dtype != torch.float32 or tuple(out.shape) != (nq, nd):
        raise ValueError("sim_scores: out must be fp32 [nq, nd]")
    call("mme_sim_scores", q.data_ptr(), _rowmajor(q, "q"), d.data_ptr(), _rowmajor(d, "d"), nq, nd, D,
         out.data_ptr(), _rowmajor(out, "out"), _stream())
    return out


def maxsim(Q: torch.Tensor, q_lens: torch.Tensor, D: torch.Tensor, d_lens: torch.Tensor,
           d_zero: Optional[torch.Tensor] = None, max_ws_bytes: int = 4 << 30) -> torch.Tensor:
    """ColPali MaxSim scores fp32 [nq, nd] from zero-padded Q [nq,Lq,128], D [nd,Ld,128] (Ld % 16 == 0)."""
    _dev(Q, q_lens, D, d_lens, d_zero)
    nq, Lq, dim = Q.shape
    nd, Ld, _ = D.shape
    Q = Q.contiguous()
    D = D.contiguous()
    out = torch.empty(nq, nd, dtype=torch.float32, device=Q.device)
    per_q = query("mme_maxsim_workspace_bytes", 1, Lq, nd)
    chunk = max(1, min(nq, max_ws_bytes // max(per_q, 1)))
    for q0 in range(0, nq, chunk):
        q1 = min(nq, q0 + chunk)
        wsb = query("mme_maxsim_workspace_bytes", q1 - q0, Lq, nd)
        ws = _ws.get(wsb, Q.device)
        call("mme_maxsim", Q[q0:q1].data_ptr(), q_lens[q0:q1].data_ptr(), q1 - q0, Lq, D.data_ptr(), d_lens.data_ptr(),
             _ptr(d_zero), nd, Ld, dim, out[q0:q1].data_ptr(), ws.data_ptr(), ws.numel(), _stream())
    return out


def round_up(x: int, m: int) -> int:
    return int(math.ceil(x / m) * m)
