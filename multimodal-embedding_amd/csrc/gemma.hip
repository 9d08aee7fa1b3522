// ColPali encoder kernels (PaliGemma-3B language side, gfx950).
//
// The ColPali branch of encode_data (main.py:402-405,422-425) runs
// ColPali(PaliGemma) = SigLIP-448 vision tower -> multi_modal_projector ->
// Gemma-2B decoder stack (bidirectional over the prefix) -> final RMSNorm ->
// 128-d projection -> per-token L2 normalise x attention_mask
// (TF:models/colpali/modeling_colpali.py:107-146,
//  TF:models/paligemma/modeling_paligemma.py:177-285,
//  TF:models/gemma/modeling_gemma.py:50-335).
// The GEMMs run on mme_gemm (GeGLU fused into its epilogue, MME_ACT_GEGLU_TANH);
// this file holds the Gemma-specific pieces:
//   * rmsnorm_kernel       GemmaRMSNorm: fp32 x*rsqrt(mean x^2 + eps)*(1 + w)  (HBM-bound)
//   * rope_kernel          rotary embedding in place on the packed q|k heads   (HBM-bound)
//   * gemma_embed_kernel   scaled token embedding + image-feature scatter     (HBM-bound)
//   * attn_mqa_kernel      flash attention, head dim 256, ONE shared K/V head  (MFMA)
//   * l2norm_masked_kernel embeddings / ||embeddings|| * attention_mask        (HBM-bound)
#include "common.h"

namespace {

template <int N>
__device__ __forceinline__ void vm_wait() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

constexpr int MAXC = 4;  // 16-B chunks per lane: d <= 2048

// GemmaRMSNorm.forward (TF:models/gemma/modeling_gemma.py:64-78): the row is
// upcast to fp32, y = x * rsqrt(mean(x^2) + eps) * (1 + w) (Gemma; unit = 1)
// or * w (unit = 0), one rounding to bf16 at the end (type_as(x)).
__global__ __launch_bounds__(256) void rmsnorm_kernel(const bf16* __restrict__ x, int ldx,
                                                      const bf16* __restrict__ w, bf16* __restrict__ y, int ldy,
                                                      int rows, int d, float eps, float unit,
                                                      const int32_t* __restrict__ idx) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= rows) return;
    const long src = idx ? idx[row] : row;
    const int nch = d >> 3;
    const bf16* xr = x + src * ldx;
    float v[MAXC][8];
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
        const int ch = lane + c * 64;
        if (ch < nch) {
            const u16x8 u = *reinterpret_cast<const u16x8*>(xr + ch * 8);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                v[c][e] = bits2f(u[e]);
                s += v[c][e] * v[c][e];
            }
        }
    }
    const float r = rsqrtf(wave_sum(s) / d + eps);
    bf16* yr = y + (long)row * ldy;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
        const int ch = lane + c * 64;
        if (ch < nch) {
            const u16x8 wu = *reinterpret_cast<const u16x8*>(w + ch * 8);
            bf16x8 o;
#pragma unroll
            for (int e = 0; e < 8; ++e) o[e] = f2bf((v[c][e] * r) * (unit + bits2f(wu[e])));
            *reinterpret_cast<bf16x8*>(yr + ch * 8) = o;
        }
    }
}

// GemmaRotaryEmbedding + apply_rotary_pos_emb (TF:models/gemma/modeling_gemma.py:100-187),
// in place on heads [0, nheads) of each packed row (the q heads, then the k head):
//   inv_freq[j] = 1 / theta^(2j/hd) (fp32), f = inv_freq[j] * pos (fp32),
//   c = bf16(cos f), s = bf16(sin f)   (cos/sin in fp32, cast to the activation dtype),
//   y[j]      = bf16( bf16(x[j] * c)      + bf16(-x[j+hd/2] * s) )
//   y[j+hd/2] = bf16( bf16(x[j+hd/2] * c) + bf16( x[j] * s) )
// pos = (row % T) + pos_offset (PaliGemma positions are 1-indexed and independent of
// the attention mask, TF:models/paligemma/modeling_paligemma.py:234-237).
// One thread per (row, head, 8 rotation pairs).
__global__ __launch_bounds__(256) void rope_kernel(bf16* __restrict__ qkv, int ld, int rows, int T, int nheads,
                                                   int hd, int pos_offset, float theta) {
    const int half = hd >> 1, cph = half >> 3;  // 8-element chunks per half head
    const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const long total = (long)rows * nheads * cph;
    if (gid >= total) return;
    const int c = gid % cph;
    const int h = (gid / cph) % nheads;
    const long row = gid / ((long)cph * nheads);
    const float pos = (float)((int)(row % T) + pos_offset);
    bf16* p1 = qkv + row * ld + (long)h * hd + c * 8;
    bf16* p2 = p1 + half;
    const u16x8 a = *reinterpret_cast<const u16x8*>(p1);
    const u16x8 b = *reinterpret_cast<const u16x8*>(p2);
    bf16x8 o1, o2;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const int j = c * 8 + e;
        const float inv = 1.0f / powf(theta, (float)(2 * j) / (float)hd);
        float sn, cs;
        sincosf(inv * pos, &sn, &cs);
        const float cb = bf2f(f2bf(cs)), sb = bf2f(f2bf(sn));
        const float x1 = bits2f(a[e]), x2 = bits2f(b[e]);
        o1[e] = f2bf(bf2f(f2bf(x1 * cb)) + bf2f(f2bf(-x2 * sb)));
        o2[e] = f2bf(bf2f(f2bf(x2 * cb)) + bf2f(f2bf(x1 * sb)));
    }
    *reinterpret_cast<bf16x8*>(p1) = o1;
    *reinterpret_cast<bf16x8*>(p2) = o2;
}

// Decoder input assembly (TF:models/paligemma/modeling_paligemma.py:231-246 and
// GemmaTextScaledWordEmbedding, TF:models/gemma/modeling_gemma.py:50-61):
//   t <  P : out[b*L+t] = img[b*P+t]                  (masked_scatter of the projected image
//                                                      features; ColPali puts its P <image> tokens first)
//   t >= P : out[b*L+t] = bf16(tok[ids[b,t]] * scale)  (scale = bf16(sqrt(d)), a bf16 multiply)
__global__ __launch_bounds__(256) void gemma_embed_kernel(const int64_t* __restrict__ ids, int rows, int L,
                                                          const bf16* __restrict__ tok, int d, float scale,
                                                          const bf16* __restrict__ img, int ld_img, int P,
                                                          bf16* __restrict__ out, int ldo) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (row >= rows) return;
    const int b = row / L, t = row % L;
    bf16* orow = out + (long)row * ldo;
    if (t < P) {
        const bf16* src = img + ((long)b * P + t) * ld_img;
        for (int ch = lane; ch < d / 8; ch += 64)
            *reinterpret_cast<u16x8*>(orow + ch * 8) = *reinterpret_cast<const u16x8*>(src + ch * 8);
        return;
    }
    const bf16* tr = tok + ids[row] * (long)d;
    for (int ch = lane; ch < d / 8; ch += 64) {
        const u16x8 a = *reinterpret_cast<const u16x8*>(tr + ch * 8);
        bf16x8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = f2bf(bits2f(a[e]) * scale);
        *reinterpret_cast<bf16x8*>(orow + ch * 8) = o;
    }
}

// ColPaliForRetrieval tail (TF:models/colpali/modeling_colpali.py:136-140):
//   e = bf16(x / bf16(||x||)) ; e = bf16(e * mask[row])   (mask: the int64 attention_mask)
__global__ __launch_bounds__(256) void l2norm_masked_kernel(const bf16* __restrict__ x, int ldx,
                                                            bf16* __restrict__ y, int ldy, int rows, int d,
                                                            const int64_t* __restrict__ mask) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= rows) return;
    const int nch = d >> 3;
    const bf16* xr = x + (long)row * ldx;
    float v[MAXC][8];
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
        const int ch = lane + c * 64;
        if (ch < nch) {
            const u16x8 u = *reinterpret_cast<const u16x8*>(xr + ch * 8);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                v[c][e] = bits2f(u[e]);
                s += v[c][e] * v[c][e];
            }
        }
    }
    const float nrm = bf2f(f2bf(sqrtf(wave_sum(s))));
    const float m = mask ? (float)mask[row] : 1.0f;
    bf16* yr = y + (long)row * ldy;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
        const int ch = lane + c * 64;
        if (ch < nch) {
            bf16x8 o;
#pragma unroll
            for (int e = 0; e < 8; ++e) o[e] = f2bf(bf2f(f2bf(v[c][e] / nrm)) * m);
            *reinterpret_cast<bf16x8*>(yr + ch * 8) = o;
        }
    }
}

// ---------------------------------------------------------------------------
// attn_mqa_kernel: softmax(Q K^T * scale + key mask) V for head dim 256 with
// ONE key/value head shared by all Hq query heads (Gemma-2B: Hq = 8, MQA;
// GemmaAttention + eager_attention_forward, TF:models/gemma/modeling_gemma.py:202-292;
// repeat_kv is never materialised). PaliGemma's decoder is bidirectional
// (use_bidirectional_attention, TF:models/paligemma/configuration_paligemma.py:92-95;
// a ColPali sequence is all prefix, token_type_ids == 0), so the mask is the
// key-padding range only: keys in [kstart[b], kend[b]) are valid (left-padded
// queries: kstart = pad count). kend[b] > kstart[b] is required.
//
// One workgroup = 8 waves over the SAME query rows of one sequence; wave w takes
// query head (w % Hq) for 16 queries (w / Hq picks the 16-row group), so every
// K/V tile staged in LDS feeds all heads (the MQA reuse).
//   * 32-key K/V tiles by LDS-DMA in "chunk planes" (plane c = 16-B column chunk c
//     of the tile's 32 keys = 512 B; one global_load_lds_dwordx4 moves two
//     planes), 2-deep ring, one barrier per tile; V planes with odd c store
//     key ^ 8 so the transposed reads hit distinct banks;
//   * S^T = K . Q^T on v_mfma_f32_16x16x32_bf16 (8 K32 steps): each lane owns one
//     query, softmax statistics are lane-local + 2 xor-shuffles;
//   * P stays in registers as the B operand of O^T = V^T . P^T, V^T read with
//     ds_read_b64_tr_b16; O^T accumulators: 16 d-tiles x 16 queries per wave.
// ---------------------------------------------------------------------------
struct MqaArgs {
    const bf16* qkv;
    bf16* out;
    const int32_t* kstart;
    const int32_t* kend;
    int ld, ldo, T, Hq;
    float scale_log2;
};

constexpr int MQ_HD = 256;
constexpr int MQ_NW = 8;                    // waves per workgroup
constexpr int MQ_QW = 16;                   // queries per wave
constexpr int MQ_KT = 32;                   // keys per tile
constexpr int MQ_NPL = MQ_HD / 8;           // 16-B planes per K (or V) row: 32
constexpr int MQ_PLANE = MQ_KT * 16;        // 512 B
constexpr int MQ_KB = MQ_NPL * MQ_PLANE;    // 16 KiB of K per tile
constexpr int MQ_TILE = 2 * MQ_KB;          // K + V
constexpr int MQ_NINS = MQ_TILE / 1024;     // DMA instructions per tile: 32
constexpr int MQ_IPW = MQ_NINS / MQ_NW;     // per wave: 4
constexpr int MQ_NSTG = 2;

__global__ __launch_bounds__(MQ_NW * 64) void attn_mqa_kernel(MqaArgs a) {
    __shared__ __attribute__((aligned(16))) char lds[MQ_NSTG * MQ_TILE];
    constexpr int NKS = MQ_HD / 32;  // K32 steps of the QK reduction: 8
    constexpr int NDT = MQ_HD / 16;  // output d-tiles: 16

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = lane >> 4, li = lane & 15;
    const int QB = MQ_QW * (MQ_NW / a.Hq);  // queries per workgroup
    const int nqb = (a.T + QB - 1) / QB;
    int id;
    {  // XCD-aware: consecutive query blocks of one sequence (same K/V) on one XCD
        const int bid = blockIdx.x, nwg = gridDim.x;
        const int xcd = bid & 7, loc = bid >> 3, q8 = nwg >> 3, r8 = nwg & 7;
        id = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
    }
    const int qb = id % nqb, b = id / nqb;
    const int h = wave % a.Hq, grp = wave / a.Hq;
    const int T = a.T;
    const bf16* base = a.qkv + (long)b * T * a.ld;
    const int q0 = qb * QB + grp * MQ_QW;
    const int ks = a.kstart ? a.kstart[b] : 0;
    const int ke = a.kend ? a.kend[b] : T;
    const float c = a.scale_log2;

    // Q^T fragments (B operand): lane (g, li) = query q0+li, depth s*32 + 8g .. +7
    bf16x8 qf[NKS];
    {
        const bf16* qrow = base + (long)min(q0 + li, T - 1) * a.ld + h * MQ_HD;
#pragma unroll
        for (int s = 0; s < NKS; ++s) qf[s] = *reinterpret_cast<const bf16x8*>(qrow + s * 32 + 8 * g);
    }

    const int t0 = ks / MQ_KT, t1 = (ke + MQ_KT - 1) / MQ_KT;

    // DMA of tile t: instruction idx = wave + 8*i; idx < 16 -> K planes 2idx, 2idx+1,
    // idx >= 16 -> V planes. Lane l -> plane 2*(idx&15) + (l>>5), key l&31 (odd V planes:
    // key ^ 8); rows past T are clamped to T-1 (finite data whose scores are masked).
    int keyi[MQ_IPW];
    const bf16* coli[MQ_IPW];
#pragma unroll
    for (int i = 0; i < MQ_IPW; ++i) {
        const int idx = wave + MQ_NW * i;
        const bool isV = idx >= MQ_NINS / 2;
        const int plane = 2 * (idx & 15) + (lane >> 5);
        keyi[i] = (isV && (plane & 1)) ? ((lane & 31) ^ 8) : (lane & 31);
        coli[i] = base + (isV ? (a.Hq + 1) * MQ_HD : a.Hq * MQ_HD) + plane * 8;
    }
    auto issue = [&](int t) {
        char* tb = lds + (t % MQ_NSTG) * MQ_TILE;
#pragma unroll
        for (int i = 0; i < MQ_IPW; ++i)
            glds16(coli[i] + (long)min(t * MQ_KT + keyi[i], T - 1) * a.ld, tb + (wave + MQ_NW * i) * 1024);
    };

    const unsigned lds0 = (unsigned)(uintptr_t)(LDS_AS char*)lds;
    const unsigned koff = g * MQ_PLANE + li * 16;  // K fragment: plane 4s+g, key kt*16+li
    const int r1 = 4 * g + (li >> 2);               // V^T fragment key rows r1, r1+16
    const unsigned vlo = (li & 1) * 8;
    const int vpl = (li >> 1) & 1;                  // plane 2dt+vpl; odd planes are key^8-swizzled
    const unsigned va0 = MQ_KB + vpl * MQ_PLANE + vlo + ((r1 ^ (vpl ? 8 : 0)) * 16);
    const unsigned vb0 = MQ_KB + vpl * MQ_PLANE + vlo + (((r1 + 16) ^ (vpl ? 8 : 0)) * 16);

    f32x4 o[NDT];
#pragma unroll
    for (int i = 0; i < NDT; ++i) o[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    float m = -1e30f, lsum = 0.f;

    if (t0 < t1) issue(t0);
    for (int t = t0; t < t1; ++t) {
        vm_wait<0>();
        __builtin_amdgcn_s_barrier();
        if (t + 1 < t1) issue(t + 1);
        const unsigned tb = lds0 + (t % MQ_NSTG) * MQ_TILE;

        f32x4 sc[2];
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
            f32x4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s = 0; s < NKS; ++s) {
                const bf16x8 kf =
                    *reinterpret_cast<const LDS_AS bf16x8*>((uintptr_t)(tb + koff + s * 4 * MQ_PLANE + kt * 256));
                z = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[s], z, 0, 0, 0);
            }
            sc[kt] = z;
        }
        // sc[kt][r] scores key t*32 + kt*16 + 4g + r; mask only tiles crossing the range
        const int tk0 = t * MQ_KT;
        if (ks > tk0 || ke < tk0 + MQ_KT) {
#pragma unroll
            for (int kt = 0; kt < 2; ++kt)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int key = tk0 + kt * 16 + 4 * g + r;
                    if (key < ks || key >= ke) sc[kt][r] = -INFINITY;
                }
        }

        float mloc = fmaxf(fmaxf(fmaxf(sc[0][0], sc[0][1]), fmaxf(sc[0][2], sc[0][3])),
                           fmaxf(fmaxf(sc[1][0], sc[1][1]), fmaxf(sc[1][2], sc[1][3])));
        mloc = fmaxf(mloc, __shfl_xor(mloc, 16, 64));
        mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
        const float mnew = fmaxf(m, mloc);
        const float alpha = __builtin_amdgcn_exp2f((m - mnew) * c);
        m = mnew;
        const float mc = mnew * c;
        float psum = 0.f;
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float p = __builtin_amdgcn_exp2f(sc[kt][r] * c - mc);
                sc[kt][r] = p;
                psum += p;
            }
        lsum = lsum * alpha + psum;
#pragma unroll
        for (int i = 0; i < NDT; ++i) o[i] *= alpha;

        const bf16x8 pb = __builtin_convertvector(__builtin_shufflevector(sc[0], sc[1], 0, 1, 2, 3, 4, 5, 6, 7),
                                                  bf16x8);
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) {
            const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (LDS_AS s16x4*)(uintptr_t)(tb + va0 + dt * 2 * MQ_PLANE));
            const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (LDS_AS s16x4*)(uintptr_t)(tb + vb0 + dt * 2 * MQ_PLANE));
            const bf16x8 vv = __builtin_bit_cast(bf16x8, __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7));
            o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vv, pb, o[dt], 0, 0, 0);
        }
    }

    float ltot = lsum + __shfl_xor(lsum, 16, 64);
    ltot += __shfl_xor(ltot, 32, 64);
    const float inv = 1.0f / ltot;
    const int q = q0 + li;
    if (q < T) {
        bf16* orow = a.out + ((long)b * T + q) * a.ldo + h * MQ_HD;
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) {
            bf16x4 v;
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = f2bf(o[dt][r] * inv);
            *reinterpret_cast<bf16x4*>(orow + dt * 16 + 4 * g) = v;
        }
    }
}

}  // namespace

extern "C" int mme_rmsnorm(const void* x, int ldx, const void* w, void* y, int ldy, int rows, int d, float eps,
                           int unit_offset, const int32_t* rows_idx, void* stream) {
    MME_REQUIRE(x && w && y, "mme_rmsnorm: null pointer");
    MME_REQUIRE(rows >= 0 && d > 0 && d % 8 == 0 && d <= 8 * 64 * MAXC, "mme_rmsnorm: d=%d unsupported", d);
    MME_REQUIRE(ldx % 8 == 0 && ldy % 8 == 0 && ldx >= d && ldy >= d, "mme_rmsnorm: bad leading dims");
    if (rows == 0) return MME_OK;
    hipLaunchKernelGGL(rmsnorm_kernel, dim3(cdiv(rows, 4)), dim3(256), 0, as_stream(stream), (const bf16*)x, ldx,
                       (const bf16*)w, (bf16*)y, ldy, rows, d, eps, unit_offset ? 1.0f : 0.0f, rows_idx);
    return mme_check_launch("mme_rmsnorm");
}

extern "C" int mme_rope(void* qkv, int ld, int rows, int T, int nheads, int hd, int pos_offset, float theta,
                        void* stream) {
    MME_REQUIRE(qkv, "mme_rope: null pointer");
    MME_REQUIRE(rows >= 0 && T > 0 && nheads > 0 && hd > 0 && hd % 16 == 0, "mme_rope: bad shape (hd %% 16 == 0)");
    MME_REQUIRE(ld % 8 == 0 && ld >= nheads * hd && ((uintptr_t)qkv & 15) == 0, "mme_rope: bad ld / alignment");
    MME_REQUIRE(theta > 1.0f, "mme_rope: theta must be > 1");
    if (rows == 0) return MME_OK;
    const long total = (long)rows * nheads * (hd / 16);
    hipLaunchKernelGGL(rope_kernel, dim3(cdiv(total, 256)), dim3(256), 0, as_stream(stream), (bf16*)qkv, ld, rows, T,
                       nheads, hd, pos_offset, theta);
    return mme_check_launch("mme_rope");
}

extern "C" int mme_gemma_embed(const int64_t* ids, int B, int L, const void* tok, int d, float scale, const void* img,
                               int ld_img, int P, void* out, int ld_out, void* stream) {
    MME_REQUIRE(ids && tok && out, "mme_gemma_embed: null pointer");
    MME_REQUIRE(B >= 0 && L > 0 && d % 8 == 0 && ld_out % 8 == 0 && ld_out >= d, "mme_gemma_embed: bad shape");
    MME_REQUIRE(P >= 0 && P <= L && (P == 0 || (img && ld_img % 8 == 0 && ld_img >= d)),
                "mme_gemma_embed: bad image prefix");
    if (B == 0) return MME_OK;
    const int rows = B * L;
    hipLaunchKernelGGL(gemma_embed_kernel, dim3(cdiv(rows, 4)), dim3(256), 0, as_stream(stream), ids, rows, L,
                       (const bf16*)tok, d, scale, (const bf16*)img, ld_img, P, (bf16*)out, ld_out);
    return mme_check_launch("mme_gemma_embed");
}

extern "C" int mme_l2norm_masked(const void* x, int ldx, void* y, int ldy, int rows, int d, const int64_t* mask,
                                 void* stream) {
    MME_REQUIRE(x && y, "mme_l2norm_masked: null pointer");
    MME_REQUIRE(rows >= 0 && d > 0 && d % 8 == 0 && d <= 8 * 64 * MAXC, "mme_l2norm_masked: d=%d unsupported", d);
    MME_REQUIRE(ldx % 8 == 0 && ldy % 8 == 0 && ldx >= d && ldy >= d, "mme_l2norm_masked: bad leading dims");
    if (rows == 0) return MME_OK;
    hipLaunchKernelGGL(l2norm_masked_kernel, dim3(cdiv(rows, 4)), dim3(256), 0, as_stream(stream), (const bf16*)x,
                       ldx, (bf16*)y, ldy, rows, d, mask);
    return mme_check_launch("mme_l2norm_masked");
}

extern "C" int mme_attention_mqa(const void* qkv, int ld_qkv, void* out, int ld_out, int B, int T, int Hq, int hd,
                                 const int32_t* kstart, const int32_t* kend, float scale, void* stream) {
    MME_REQUIRE(qkv && out, "mme_attention_mqa: null pointer");
    MME_REQUIRE(hd == MQ_HD, "mme_attention_mqa: head_dim %d unsupported (256)", hd);
    MME_REQUIRE(Hq == 1 || Hq == 2 || Hq == 4 || Hq == 8, "mme_attention_mqa: Hq=%d unsupported (1/2/4/8)", Hq);
    MME_REQUIRE(B >= 0 && T > 0, "mme_attention_mqa: bad shape");
    MME_REQUIRE(ld_qkv % 8 == 0 && ld_qkv >= (Hq + 2) * hd, "mme_attention_mqa: bad ld_qkv");
    MME_REQUIRE(ld_out % 4 == 0 && ld_out >= Hq * hd, "mme_attention_mqa: bad ld_out");
    MME_REQUIRE(((uintptr_t)qkv & 15) == 0 && ((uintptr_t)out & 7) == 0, "mme_attention_mqa: misaligned");
    if (B == 0) return MME_OK;
    MqaArgs a{(const bf16*)qkv, (bf16*)out, kstart, kend, ld_qkv, ld_out, T, Hq, scale * 1.4426950408889634f};
    const int QB = MQ_QW * (MQ_NW / Hq);
    hipLaunchKernelGGL(attn_mqa_kernel, dim3(cdiv(T, QB) * B), dim3(MQ_NW * 64), 0, as_stream(stream), a);
    return mme_check_launch("mme_attention_mqa");
}

