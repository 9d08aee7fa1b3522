"""Dual-encoder models behind the reference's HF duck type.

``SiglipModel`` / ``CLIPModel`` expose exactly what main.py consumes:
  * get_image_features(pixel_values=[B,3,S,S]) -> Tensor[B, D]   (main.py:408-409)
  * get_text_features(input_ids=[B,L], attention_mask=None) -> Tensor[B, D] (main.py:428-429)
  * eval() / to() returning self (main.py:812-819)
returning plain tensors (transformers-4 semantics), plus the
fast device paths encode_images(u8 images) / encode_texts(ids) and score().

Every arithmetic step runs in libmme (mme.ops); this module only sequences
kernels and sizes buffers. The tower structure follows
TF:models/siglip/modeling_siglip.py:325-357,553-644 and
TF:models/clip/modeling_clip.py:494-656.
"""
from __future__ import annotations

import os
from typing import List, Optional, Sequence, Tuple

import torch

from . import mx, ops
from .config import ACTS, ModelSpec, TowerConfig, get_spec
from .weights import LayerW, ModelW, TextW, VisionW, from_hf_state_dict, random_state_dict

BF16 = torch.bfloat16
# LayerNorm -> Linear pairs run as mme_rowstats + mme_gemm_lnfold (the normalised rows are
# never written); MME_LN_FOLD=0 restores mme_layernorm + mme_gemm
LN_FOLD = os.environ.get("MME_LN_FOLD", "1") != "0"
# the o_proj / fc2 residual GEMMs leave the next LayerNorm's row statistics
# (mme_gemm_res_stats) instead of a separate mme_rowstats pass over the residual stream
FUSED_STATS = os.environ.get("MME_FUSED_STATS", "1") != "0"
# The pooled towers read the last layer's output at one row per item (CLIP image CLS, text EOS /
# argmax / last token): that layer's o_proj, layer_norm2 and MLP are row-wise, so they run on the
# pooled rows alone (every row's dead computation skipped; the kept rows' arithmetic unchanged).
# MME_PRUNE_LAST=0 runs them on every row.
PRUNE_LAST = os.environ.get("MME_PRUNE_LAST", "1") != "0"
# SigLIP's MAP head with the probe query absorbed into the key projection (mme_map_pool):
# no [B*T, 2d] K / V projection; MME_MAP_ABSORB=0 runs the K / V GEMM + mme_probe_attention.
MAP_ABSORB = os.environ.get("MME_MAP_ABSORB", "1") != "0"
# Head dims 72 / 80 with T > 128 (the vision towers; round 6): the attention's scale * log2(e) folded
# into the Q rows of the QKV projection, attention through mme_attention_qs (kinds 98 / 100 / 101: the
# softmax's exp2 argument straight out of the QK^T MFMA). MME_Q_PRESCALE=0 keeps the plain entry.
Q_PRESCALE = os.environ.get("MME_Q_PRESCALE", "1") != "0"


def q_prescale(cfg: TowerConfig, T: int) -> Optional[float]:
    """The factor folded into a tower's Q projection (None: the plain attention entry)."""
    return ops.attention_q_scale(cfg.head_dim) if Q_PRESCALE and cfg.head_dim in (72, 80) and T > 128 else None


class _Bufs:
    """Per-forward activation buffers: x (residual stream), h (LN / attention
    output) and one wide buffer shared by QKV and the MLP hidden."""

    def __init__(self, rows: int, cfg: TowerConfig, device, fp8: bool = False):
        d = cfg.hidden
        wide = max(3 * d, cfg.inter_pad)
        self.h = torch.empty(rows, d, dtype=BF16, device=device)
        self.wide = torch.empty(rows, wide, dtype=BF16, device=device)
        # fp8 mode: mx8 LayerNorm output and mx8 MLP hidden (fc1 -> fc2 operand)
        self.hq = mx.MXTensor.empty(rows, d, device) if fp8 else None
        self.midq = mx.MXTensor.empty(rows, cfg.inter_pad, device) if fp8 else None
        self.stats = torch.empty(rows, 2, dtype=torch.float32, device=device)
        # per-64-column (mean, M2) slices of the residual GEMMs' output rows (mme_gemm_res_stats)
        self.part = torch.empty(rows, max(1, d // 64), 2, dtype=torch.float32, device=device) \
            if FUSED_STATS and d % 64 == 0 else None


def _pooled(a: torch.Tensor, x: torch.Tensor, rows: Optional[torch.Tensor]):
    """The attention output and residual stream at the pooled rows only (a row gather: data
    movement), or both unchanged without `rows`."""
    if rows is None:
        return a, x
    return a.index_select(0, rows), x.index_select(0, rows)


def encoder_layer(x: torch.Tensor, L: LayerW, cfg: TowerConfig, B: int, T: int, bufs: _Bufs, *,
                  seq_lens: Optional[torch.Tensor] = None, causal: bool = False, stats_in: bool = False,
                  stats_out: bool = False, rows: Optional[torch.Tensor] = None) -> Tuple[bool, torch.Tensor]:
    """Pre-LN transformer block, in place on x (SiglipEncoderLayer.forward, TF:…siglip.py:341-357).

    LayerNorm-folded path: stats_in = bufs.stats already holds x's row statistics (left by
    the previous layer's fc2); stats_out = leave the statistics of the output x there for
    the next layer. Returns (whether it did — mme_gemm_res_stats on the fc2 residual GEMM —,
    the output rows).

    rows (int32 [n], the last layer of a pooled tower): only these rows of the output are
    read by the pooling head, so after the attention (which every token's K / V feed) the
    row-wise rest — o_proj + residual, layer_norm2, fc1, fc2 — runs on the gathered rows and
    the layer returns them as a new [n, d] tensor (x is left as the attention input)."""
    d, H, hd = cfg.hidden, cfg.heads, cfg.head_dim
    act = ACTS[cfg.act]
    if L.mx is not None:  # fp8 mode: QKV / fc1 / fc2 on the block-scaled fp8 MFMA (mme/mx.py)
        hq = mx.layernorm(x, L.ln1_g, L.ln1_b, cfg.eps, out=bufs.hq)
        qkv = mx.gemm(hq, L.mx.qkv, L.qkv_b if L.mx.qkv_b is None else L.mx.qkv_b, out=bufs.wide[:, : 3 * d])
        a = ops.attention(qkv, B, T, H, hd, seq_lens=seq_lens, causal=causal, out=bufs.h,
                          q_prescaled=L.mx.qkv_b is not None)
        a, x = _pooled(a, x, rows)
        n = x.shape[0]
        mlp_flops = 2.0 * n * d * cfg.intermediate
        if L.mx.o is not None:  # MME_FP8_OPROJ=1 drift experiment: o_proj on mx8 too
            mx.gemm(mx.quantize(a, out=bufs.hq), L.mx.o, L.o_b, residual=x, out=x)
        else:
            ops.gemm(a, L.o_w, L.o_b, residual=x, out=x)
        hq = mx.layernorm(x, L.ln2_g, L.ln2_b, cfg.eps, out=bufs.hq)
        midq = mx.gemm(hq, L.mx.fc1, L.fc1_b, act=act, out_mx=bufs.midq, algo_flops=mlp_flops)
        mx.gemm(midq, L.mx.fc2, L.fc2_b, residual=x, out=x, algo_flops=mlp_flops)
        return False, x
    if LN_FOLD:  # layer_norm1 -> qkv and layer_norm2 -> fc1 folded (mme.h mme_gemm_lnfold)
        if L.fold is None:
            qs, c = None, q_prescale(cfg, T)
            if c is not None:  # Q rows carry the attention's scale * log2(e)
                qs = torch.ones(3 * d, dtype=torch.float32)
                qs[:d] = c
            L.fold = (ops.LNFolded(L.qkv_w, L.qkv_b, L.ln1_g, L.ln1_b, row_scale=qs),
                      ops.LNFolded(L.fc1_w, L.fc1_b, L.ln2_g, L.ln2_b))
            L.q_prescaled = qs is not None
        fused = bufs.part is not None
        st = bufs.stats if (stats_in and fused) else ops.rowstats(x, cfg.eps, d=d, out=bufs.stats)
        qkv = ops.gemm_lnfold(x, L.fold[0], st, out=bufs.wide[:, : 3 * d])
        a = ops.attention(qkv, B, T, H, hd, seq_lens=seq_lens, causal=causal, out=bufs.h,
                          q_prescaled=L.q_prescaled)
        a, x = _pooled(a, x, rows)
        n = x.shape[0]
        mlp_flops = 2.0 * n * d * cfg.intermediate  # unpadded intermediate width
        if fused:  # o_proj + residual, with layer_norm2's statistics from the epilogue
            ops.gemm_res_stats(a, L.o_w, L.o_b, x, cfg.eps, bufs.stats, bufs.part, out=x)
            st = bufs.stats
        else:
            ops.gemm(a, L.o_w, L.o_b, residual=x, out=x)
            st = ops.rowstats(x, cfg.eps, d=d, out=bufs.stats)
        mid = ops.gemm_lnfold(x, L.fold[1], st, act=act, out=bufs.wide[:n, : cfg.inter_pad], algo_flops=mlp_flops)
        if fused and stats_out:
            ops.gemm_res_stats(mid, L.fc2_w, L.fc2_b, x, cfg.eps, bufs.stats, bufs.part, out=x, algo_flops=mlp_flops)
            return True, x
        ops.gemm(mid, L.fc2_w, L.fc2_b, residual=x, out=x, algo_flops=mlp_flops)
        return False, x
    h = ops.layernorm(x, L.ln1_g, L.ln1_b, cfg.eps, out=bufs.h)
    qkv = ops.gemm(h, L.qkv_w, L.qkv_b, out=bufs.wide[:, : 3 * d])
    a = ops.attention(qkv, B, T, H, hd, seq_lens=seq_lens, causal=causal, out=bufs.h)
    a, x = _pooled(a, x, rows)
    n = x.shape[0]
    mlp_flops = 2.0 * n * d * cfg.intermediate
    ops.gemm(a, L.o_w, L.o_b, residual=x, out=x)
    h = ops.layernorm(x, L.ln2_g, L.ln2_b, cfg.eps, out=bufs.h[:n])
    mid = ops.gemm(h, L.fc1_w, L.fc1_b, act=act, out=bufs.wide[:n, : cfg.inter_pad], algo_flops=mlp_flops)
    ops.gemm(mid, L.fc2_w, L.fc2_b, residual=x, out=x, algo_flops=mlp_flops)
    return False, x


class VisionTower:
    def __init__(self, spec: ModelSpec, w: VisionW):
        self.spec, self.cfg, self.w = spec, spec.vision, w

    def forward_patches(self, patches: torch.Tensor, B: int) -> torch.Tensor:
        """patches: bf16 [B*P, kpad] im2col image -> pooled features [B, D] (bf16)."""
        cfg, w = self.cfg, self.w
        P, d = cfg.num_patches, cfg.hidden
        dev = patches.device
        if self.spec.family == "siglip":
            T = P
            x = ops.gemm(patches, w.patch_w, w.patch_b, residual=w.pos, res_period=P,  # conv + bias + pos
                         algo_flops=2.0 * B * P * d * 3 * cfg.patch ** 2)
        else:
            T = P + 1
            pe = ops.gemm(patches, w.patch_w, algo_flops=2.0 * B * P * d * 3 * cfg.patch ** 2)
            x = ops.clip_embed_ln(pe, w.cls, w.pos, w.pre_ln_g, w.pre_ln_b, cfg.eps, B, P)
            del pe
        bufs = _Bufs(B * T, cfg, dev, fp8=w.layers[0].mx is not None)
        if self.spec.family == "siglip":  # the MAP head attends over every token
            run_layers(x, w.layers, cfg, B, T, bufs)
            return self._map_head(x, B, T, bufs)
        cls = torch.arange(B, device=dev, dtype=torch.int32) * T  # CLS rows
        y, rows = run_layers(x, w.layers, cfg, B, T, bufs, pooled_rows=cls)
        pooled = ops.layernorm(y, w.post_ln_g, w.post_ln_b, cfg.eps, rows_idx=rows)
        return ops.gemm(pooled, w.proj_w)

    def forward_tokens(self, patches: torch.Tensor, B: int) -> torch.Tensor:
        """SigLIP tower without pooling head (PaliGemma's vision_tower, vision_use_head=False,
        TF:models/siglip/modeling_siglip.py:597-619): post-LN hidden states [B*P, d] bf16."""
        cfg, w = self.cfg, self.w
        P, d = cfg.num_patches, cfg.hidden
        x = ops.gemm(patches, w.patch_w, w.patch_b, residual=w.pos, res_period=P,
                     algo_flops=2.0 * B * P * d * 3 * cfg.patch ** 2)
        bufs = _Bufs(B * P, cfg, patches.device)
        run_layers(x, w.layers, cfg, B, P, bufs)
        return ops.layernorm(x, w.post_ln_g, w.post_ln_b, cfg.eps, out=bufs.h)

    def _map_head(self, x, B, T, bufs) -> torch.Tensor:
        """post_layernorm + SiglipMultiheadAttentionPoolingHead (TF:…siglip.py:611-644)."""
        cfg, w, hw = self.cfg, self.w, self.w.head
        d = cfg.hidden
        H, hd = cfg.heads, cfg.head_dim
        h = ops.layernorm(x, w.post_ln_g, w.post_ln_b, cfg.eps, out=bufs.h)
        if MAP_ABSORB and hw.u is not None and H <= 16 and T <= 1024 and d <= 1152 and d % 2 == 0:
            # probe query absorbed into the key projection (attention.hip map_pool_kernel): scores
            # x . U_h, softmax-weighted token sums per head, then W_v on the B*H pooled rows
            S = ops.gemm(h, hw.u, out_f32=True, out=bufs.wide.view(torch.float32)[:, : 2 * H])
            pooled = ops.map_pool(S, h, B, T, H)
            g = ops.gemm(pooled, hw.v_w, hw.v_b)  # [B*H, d]: row b*H + h holds head h's block
            a = g.view(B, H, H, hd).diagonal(dim1=1, dim2=2).permute(0, 2, 1).reshape(B, d)
        else:
            kv = ops.gemm(h, hw.kv_w, hw.kv_b, out=bufs.wide[:, : 2 * d])
            a = ops.probe_attention(hw.q, kv, B, T, H, hd)
        y = ops.gemm(a, hw.out_w, hw.out_b)
        z = ops.layernorm(y, hw.ln_g, hw.ln_b, cfg.eps)
        m = ops.gemm(z, hw.fc1_w, hw.fc1_b, act=ACTS[cfg.act])
        return ops.gemm(m, hw.fc2_w, hw.fc2_b, residual=y)


class TextTower:
    def __init__(self, spec: ModelSpec, w: TextW):
        self.spec, self.cfg, self.w = spec, spec.text, w

    def forward_ids(self, ids: torch.Tensor, seq_lens: Optional[torch.Tensor]) -> torch.Tensor:
        """ids: int64 [B, L] on device -> pooled features [B, D] (bf16)."""
        cfg, w = self.cfg, self.w
        B, L = ids.shape
        x = ops.token_embed(ids, w.tok, w.pos)
        bufs = _Bufs(B * L, cfg, ids.device, fp8=self.w.layers[0].mx is not None)
        mode = {"eos": 0, "argmax": 1, "last": 2}[cfg.pool]
        pool = ops.text_pool_rows(ids, cfg.eos_id, mode)
        y, rows = run_layers(x, w.layers, cfg, B, L, bufs, pooled_rows=pool, seq_lens=seq_lens, causal=cfg.causal)
        pooled = ops.layernorm(y, w.final_ln_g, w.final_ln_b, cfg.eps, rows_idx=rows)
        return ops.gemm(pooled, w.head_w, w.head_b)


def balanced(n: int, batch: int) -> int:
    """Largest execution batch <= `batch` that splits n items into equal-sized batches
    (ceil(n / batch) batches): 625 images at 256 -> 3 x 209 instead of 256 + 256 + 113,
    so no launch runs a small, tile-starved tail batch (results do not depend on it)."""
    if n <= 0:
        return max(1, batch)
    nb = -(-n // batch)
    return -(-n // nb)


def _gemm_tiles(M: int, N: int) -> int:
    """Workgroups of one mme_gemm launch (gemm.hip dispatch): 256 x 256 tiles; when N = 256k + 128
    the last 128 columns run as 512 x 128 tiles (split grid)."""
    R = -(-M // 256)
    full, rem = divmod(N, 256)
    if rem == 0:
        return R * full
    if rem == 128:
        return R * full + -(-R // 2)
    return R * (full + 1)


def tail_aware_batch(n: int, batch: int, rows_per_item: int, cfg: Optional[TowerConfig] = None,
                     cus: int = 256) -> int:
    """Execution batch (<= `batch`) for n items of `rows_per_item` GEMM rows each.

    Each encoder layer runs four GEMMs (QKV, o_proj, fc1, fc2) whose 256 x 256 tiles fill
    the `cus` CUs one workgroup each; the last, partial wave of a launch leaves CUs idle.
    Among splits into ceil(n / batch) .. + 3 equal batches this picks the one with the
    least modelled time (sum over launches of waves x K; ties -> fewer batches).
    SigLIP-400M at the round-3 defaults (`mme.config.EXEC_*_BATCH`): 5 000 images ->
    12 x 417 (cap 512), 25 000 captions -> 5 x 5 000 (cap 8 192); at 256 / 2 048 it picked 21 x 239 (o_proj / fc2
    in 12.0 waves) instead of 20 x 250 (12.5 -> 13 waves).
    Without `cfg` it is `balanced` (equal batches, no tail model). Items never interact, but the
    batch picks the GEMM kernel (the pipelined one from M·N >= 2^20, the generic one below), so
    the fp32 summation order, and with it the output bits, may change with the batch: results
    agree within tolerance (cos >= 0.9999, tests/test_gpu_encoders.py), not bit for bit.
    With `cfg`, a batch is also capped so that the widest GEMM operand (the [rows, max(3d, I_pad)]
    activation buffer, fc2's A) stays below 4 GiB: the pipelined GEMMs address operands with 32-bit
    offsets and would otherwise fall back to the slower generic kernel (SigLIP text, L = 64:
    7 710 captions)."""
    if cfg is not None:
        widest = rows_per_item * max(3 * cfg.hidden, cfg.inter_pad) * 2
        batch = max(1, min(batch, ((1 << 32) - 1) // widest))
    if cfg is None or n <= 0 or os.environ.get("MME_TAIL_AWARE_BATCH", "1") == "0":
        return balanced(n, batch)
    d, ff = cfg.hidden, cfg.inter_pad
    shapes = ((3 * d, d), (d, d), (ff, d), (d, ff))
    nb0 = -(-n // batch)
    best = None
    for nb in range(nb0, nb0 + 4):
        bb = -(-n // nb)
        if bb < 1:
            break
        cost = 0
        for i in range(0, n, bb):
            m = min(bb, n - i) * rows_per_item
            cost += sum(-(-_gemm_tiles(m, N) // cus) * K for N, K in shapes)
        if best is None or cost < best[0] * 0.998:
            best = (cost, bb)
    return best[1]


def _num_cus(device) -> int:
    try:
        return torch.cuda.get_device_properties(device).multi_processor_count
    except (RuntimeError, AssertionError, ValueError):
        return 256


def plan_text_batches(n: int, Lmax: int, lens: Optional[List[int]], ref_batch: int, exec_batch: int,
                      cfg: Optional[TowerConfig] = None, cus: int = 256):
    """Execution plan reproducing processor(padding=True) per reference batch.

    The reference pads each batch of `ref_batch` captions (main.py:420-427) to
    its longest caption, and SigLIP pools position L_b - 1 of that padded
    batch, so a caption's embedding depends on its batch's padded length L_b.
    Captions are therefore grouped by L_b (caption order preserved) and each
    group is cut into execution batches of <= exec_batch rows.
    Yields (L_b, rows) with rows a range (contiguous) or a list of indices.
    """
    if lens is None:
        exec_batch = tail_aware_batch(n, exec_batch, Lmax, cfg, cus)
        for s in range(0, n, exec_batch):
            yield Lmax, range(s, min(n, s + exec_batch))
        return
    groups = {}
    for s in range(0, n, ref_batch):
        e = min(n, s + ref_batch)
        groups.setdefault(max(lens[s:e]), []).extend(range(s, e))
    for Lb, rows in groups.items():
        eb = tail_aware_batch(len(rows), exec_batch, Lb, cfg, cus)
        for j in range(0, len(rows), eb):
            part = rows[j:j + eb]
            yield Lb, (range(part[0], part[-1] + 1) if part[-1] - part[0] + 1 == len(part) else part)


def _seq_lens(attention_mask: Optional[torch.Tensor], B: int, L: int, device) -> Optional[torch.Tensor]:
    """Right-padded attention_mask -> int32 valid lengths (None if no padding)."""
    if attention_mask is None:
        return None
    m = attention_mask.to(device=device)
    lens = m.sum(dim=1).to(torch.int32)
    # the kernels mask keys >= len: require the mask to be a prefix mask
    ar = torch.arange(L, device=device).unsqueeze(0)
    if not torch.equal(m.bool(), ar < lens.unsqueeze(1)):
        raise ValueError("attention_mask must be right-padded (a prefix of ones per row)")
    if int(lens.min()) == L:
        return None
    return lens


def run_layers(x: torch.Tensor, layers, cfg: TowerConfig, B: int, T: int, bufs: _Bufs, *,
               pooled_rows: Optional[torch.Tensor] = None, **kw) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    """The encoder stack; each layer's fc2 hands the next layer its LayerNorm statistics.

    pooled_rows (int32): the rows the tower's pooling head reads (CLIP CLS, text EOS / argmax /
    last token). With PRUNE_LAST the last layer's row-wise half runs on those rows alone and
    this returns ([n, d] pooled output, None); otherwise (x, pooled_rows) — either way the
    head reads `out[rows]` (rows None = every row in order)."""
    have = False
    last = len(layers) - 1
    for i, L in enumerate(layers):
        rows = pooled_rows if (PRUNE_LAST and i == last) else None
        have, y = encoder_layer(x, L, cfg, B, T, bufs, stats_in=have, stats_out=i < last, rows=rows, **kw)
        if rows is not None:
            return y, None
    return x, pooled_rows


class DualEncoder:
    """Shared implementation of the SigLIP / CLIP duck type."""

    family = "?"

    def __init__(self, spec: ModelSpec, weights: ModelW, device="cuda"):
        self.spec = spec
        self.config = spec
        self.device = torch.device(device)
        self.weights = weights
        self.vision = VisionTower(spec, weights.vision)
        self.text = TextTower(spec, weights.text)
        self.dtype = BF16
        self.precision = "bf16"

    # ---- construction
    @classmethod
    def from_spec(cls, spec, seed: int = 0, device="cuda", state_dict=None) -> "DualEncoder":
        spec = get_spec(spec) if isinstance(spec, str) else spec
        sd = state_dict if state_dict is not None else random_state_dict(spec, seed, device)
        return cls(spec, from_hf_state_dict(spec, sd, device), device)

    def enable_fp8(self) -> "DualEncoder":
        """Opt-in fp8 precision mode (BASELINE configs[4]): quantise every encoder
        layer's QKV / fc1 / fc2 weights to mx8 once; forward passes then run those
        products on the block-scaled fp8 MFMA (mme/mx.py)."""
        vc = self.spec.vision
        tv = vc.num_patches + (0 if self.spec.family == "siglip" else 1)
        for tower, c in ((self.weights.vision, q_prescale(vc, tv)), (self.weights.text, None)):
            for L in tower.layers:
                if L.mx is None:
                    L.mx = mx.quantize_layer(L, q_scale=c)
        self.precision = "fp8"
        return self

    # ---- HF-style surface
    def eval(self):
        return self

    def to(self, *args, **kwargs):
        return self

    @torch.no_grad()
    def get_image_features(self, pixel_values: torch.Tensor, **_) -> torch.Tensor:
        """pixel_values [B,3,S,S] (fp32 or bf16) -> pooled image features [B, D] bf16."""
        v = self.spec.vision
        if pixel_values.shape[-1] != v.image_size:
            raise ValueError(f"pixel_values size {tuple(pixel_values.shape)} != model image size {v.image_size}")
        pv = pixel_values.to(self.device)
        B = pv.shape[0]
        patches = ops.im2col(pv, v.patch, v.kpad)
        return self.vision.forward_patches(patches, B)

    @torch.no_grad()
    def get_text_features(self, input_ids: torch.Tensor, attention_mask: Optional[torch.Tensor] = None,
                          **_) -> torch.Tensor:
        ids = input_ids.to(self.device, dtype=torch.int64)
        B, L = ids.shape
        return self.text.forward_ids(ids, _seq_lens(attention_mask, B, L, self.device))

    def __call__(self, *args, **kwargs):
        raise TypeError("use get_image_features / get_text_features (main.py:408-431)")

    # ---- fast device paths (u8 images / token ids resident in HBM)
    @torch.no_grad()
    def encode_images(self, images_u8: torch.Tensor, batch: int = 256, out: Optional[torch.Tensor] = None
                      ) -> torch.Tensor:
        """u8 [n,H,W,3] images -> L2-normalised bf16 embeddings [n, D].

        Fuses the processor (PIL-exact bicubic + normalise) into an im2col
        kernel feeding the patch GEMM. Images never interact; the batch size only
        selects GEMM kernels (see tail_aware_batch), so results agree across batch sizes
        within tolerance. Images in host memory (the
        reference's loader hands over host buffers) are streamed: batch i+1 is
        copied host -> HBM on a side stream (pinned staging, two device buffers)
        while batch i is encoded, so the PCIe transfer hides under the encoder."""
        from .processor import image_geometry
        v, ip = self.spec.vision, self.spec.image_proc
        n, H, W, _ = images_u8.shape
        rh, rw, top, left = image_geometry(H, W, ip)
        if out is None:
            out = torch.empty(n, self.spec.proj_dim, dtype=BF16, device=self.device)
        T = v.num_patches + (0 if self.spec.family == "siglip" else 1)
        batch = tail_aware_batch(n, batch, T, v, _num_cus(self.device))
        stream_in = not images_u8.is_cuda
        if stream_in:
            src = images_u8 if images_u8.is_pinned() else images_u8.pin_memory()
            copy_stream = torch.cuda.Stream(device=self.device)
            bufs = [torch.empty((batch, H, W, 3), dtype=torch.uint8, device=self.device) for _ in range(2)]
            done = [torch.cuda.Event(), torch.cuda.Event()]   # copy into buffer j finished
            free = [torch.cuda.Event(), torch.cuda.Event()]   # compute stopped reading buffer j

            def prefetch(i, j):
                b = min(batch, n - i)
                with torch.cuda.stream(copy_stream):
                    copy_stream.wait_event(free[j])
                    bufs[j][:b].copy_(src[i:i + b], non_blocking=True)
                    done[j].record(copy_stream)
            for j in range(2):
                free[j].record()
            prefetch(0, 0)
        for i in range(0, n, batch):
            if stream_in:
                j = (i // batch) & 1
                if i + batch < n:
                    prefetch(i + batch, j ^ 1)
                torch.cuda.current_stream().wait_event(done[j])
                chunk = bufs[j][:min(batch, n - i)]
            else:
                chunk = images_u8[i:i + batch]
            b = chunk.shape[0]
            patches = ops.preprocess_u8(chunk, resize=(rh, rw), crop=(top, left), size=ip.size, mean=ip.mean,
                                        std=ip.std, patch=v.patch, kpad=v.kpad)
            if stream_in:
                free[j].record()  # the preprocess kernel (the buffer's only reader) is enqueued
            feats = self.vision.forward_patches(patches, b)
            ops.l2norm(feats, out=out[i:i + b])
        return out

    @torch.no_grad()
    def encode_texts(self, ids: torch.Tensor, lens: Optional[torch.Tensor] = None, ref_batch: Optional[int] = None,
                     exec_batch: int = 2048, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Token ids -> L2-normalised bf16 embeddings, reproducing the reference's
        batch-padding semantics exactly: each reference batch of `ref_batch`
        captions (main.py:420) is padded to its own longest caption (processor
        padding=True); reference batches with equal padded length are fused into
        one execution batch of up to `exec_batch` rows.

        ids: int64 [n, Lmax] (right-padded, on device), lens: int [n] (None = all Lmax).
        """
        ref_batch = ref_batch or self.spec.batch_size
        n, Lmax = ids.shape
        if out is None:
            out = torch.empty(n, self.spec.proj_dim, dtype=BF16, device=self.device)
        if n == 0:
            return out
        lens_h = None if lens is None else lens.to("cpu", torch.int64).tolist()
        lens_d = None if lens is None else lens.to(self.device, torch.int32)
        for Lb, rows in plan_text_batches(n, Lmax, lens_h, ref_batch, exec_batch, self.spec.text,
                                          _num_cus(self.device)):
            if isinstance(rows, range):  # contiguous run: slice, no gather
                sel = slice(rows.start, rows.stop)
                bids, dst = ids[sel, :Lb], out[sel]
                sl = None if lens_d is None else lens_d[sel]
            else:
                r = torch.tensor(rows, device=self.device)
                bids, dst = ids.index_select(0, r)[:, :Lb], None
                sl = lens_d.index_select(0, r)
            if sl is not None and all(lens_h[i] == Lb for i in rows):
                sl = None
            feats = self.text.forward_ids(bids.contiguous(), sl)
            if dst is not None:
                ops.l2norm(feats, out=dst)
            else:
                out.index_copy_(0, r, ops.l2norm(feats))
        return out

    def score(self, query_emb: torch.Tensor, doc_emb: torch.Tensor) -> torch.Tensor:
        """Cosine score matrix fp32 [nq, nd] (compute_similarity_scores, main.py:473)."""
        return ops.gemm(query_emb, doc_emb, out_f32=True)


class SiglipModel(DualEncoder):
    family = "siglip"


class CLIPModel(DualEncoder):
    family = "clip"


def load_model(name: str, seed: int = 0, device="cuda", state_dict=None, batch_size: Optional[int] = None,
               fp8: bool = False, tokenizer=None, allow_hash_tokenizer: bool = False) -> Tuple[DualEncoder, "object"]:
    """(model, processor) for a registry name — the offline counterpart of
    from_pretrained(m_info['id']) (main.py:808-820). fp8=True: the mx8 encoder
    GEMM mode of BASELINE configs[4] (DualEncoder.enable_fp8). tokenizer: the
    checkpoint's HF tokenizer for caption strings (main.py:427); without it strings
    raise unless allow_hash_tokenizer=True (mme.processor)."""
    from .processor import Processor
    spec = get_spec(name)
    if batch_size is not None:
        spec = spec.with_batch_size(batch_size)
    cls = SiglipModel if spec.family == "siglip" else CLIPModel
    model = cls.from_spec(spec, seed=seed, device=device, state_dict=state_dict)
    if fp8:
        model.enable_fp8()
    return model, Processor(spec, device=device, tokenizer=tokenizer, allow_hash_tokenizer=allow_hash_tokenizer)
