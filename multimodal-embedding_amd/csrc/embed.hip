// Embedding assembly kernels of the text / vision towers (HBM-bound, one wave
// per output row, 16-byte vector accesses).
#include "common.h"

namespace {

// out[b*L+t] = tok[ids[b,t]] + pos[t]  — SiglipTextEmbeddings / CLIPTextEmbeddings
// (TF:models/siglip/modeling_siglip.py:189-224): bf16 + bf16 rounded to bf16.
__global__ __launch_bounds__(256) void token_embed_kernel(const int64_t* __restrict__ ids, int rows, int L,
                                                          const bf16* __restrict__ tok, const bf16* __restrict__ pos,
                                                          int d, bf16* __restrict__ out, int ldo) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (row >= rows) return;
    const long id = ids[row];
    const int t = row % L;
    const bf16* tr = tok + id * d;
    const bf16* pr = pos + (long)t * d;
    bf16* orow = out + (long)row * ldo;
    for (int ch = lane; ch < d / 8; ch += 64) {
        const u16x8 a = *reinterpret_cast<const u16x8*>(tr + ch * 8);
        const u16x8 p = *reinterpret_cast<const u16x8*>(pr + ch * 8);
        bf16x8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = f2bf(bits2f(a[e]) + bits2f(p[e]));
        *reinterpret_cast<bf16x8*>(orow + ch * 8) = o;
    }
}

// CLIPVisionEmbeddings (TF:models/clip/modeling_clip.py:203-218) + pre_layrnorm (:642):
// x = cat(cls, patches) + pos (bf16 adds), y = LayerNorm(x).
constexpr int MAXC = 4;
__global__ __launch_bounds__(256) void clip_embed_ln_kernel(const bf16* __restrict__ patch, int ldp,
                                                            const bf16* __restrict__ cls,
                                                            const bf16* __restrict__ pos,
                                                            const bf16* __restrict__ gm,
                                                            const bf16* __restrict__ bt, float eps,
                                                            bf16* __restrict__ out, int ldo, int B, int P, int d) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int T = P + 1;
    if (row >= B * T) return;
    const int b = row / T, t = row % T;
    const bf16* src = t == 0 ? cls : patch + ((long)b * P + t - 1) * ldp;
    const bf16* pr = pos + (long)t * d;
    const int nch = d / 8;
    float v[MAXC][8];
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
        const int ch = lane + c * 64;
        if (ch < nch) {
            const u16x8 a = *reinterpret_cast<const u16x8*>(src + ch * 8);
            const u16x8 p = *reinterpret_cast<const u16x8*>(pr + ch * 8);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                v[c][e] = bf2f(f2bf(bits2f(a[e]) + bits2f(p[e])));
                s += v[c][e];
            }
        } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[c][e] = 0.f;
        }
    }
    const float mean = wave_sum(s) / d;
    float s2 = 0.f;
#pragma unroll
    for (int c = 0; c < MAXC; ++c)
        if (lane + c * 64 < nch)
#pragma unroll
            for (int e = 0; e < 8; ++e) s2 += (v[c][e] - mean) * (v[c][e] - mean);
    const float rstd = rsqrtf(wave_sum(s2) / d + eps);
    bf16* orow = out + (long)row * ldo;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
        const int ch = lane + c * 64;
        if (ch < nch) {
            const u16x8 gu = *reinterpret_cast<const u16x8*>(gm + ch * 8);
            const u16x8 bu = *reinterpret_cast<const u16x8*>(bt + ch * 8);
            bf16x8 o;
#pragma unroll
            for (int e = 0; e < 8; ++e) o[e] = f2bf((v[c][e] - mean) * rstd * bits2f(gu[e]) + bits2f(bu[e]));
            *reinterpret_cast<bf16x8*>(orow + ch * 8) = o;
        }
    }
}

// Pooling row per sequence (TF:models/clip/modeling_clip.py:561-581; SigLIP :539).
__global__ void text_pool_kernel(const int64_t* __restrict__ ids, int B, int L, int64_t eos, int mode,
                                 int32_t* __restrict__ rows) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const int64_t* r = ids + (long)b * L;
    int pos = 0;
    if (mode == 0) {  // first position equal to eos (argmax of the 0/1 mask -> 0 if absent)
        for (int t = 0; t < L; ++t)
            if (r[t] == eos) {
                pos = t;
                break;
            }
    } else if (mode == 1) {  // argmax of ids (first maximal position)
        int64_t best = r[0];
        for (int t = 1; t < L; ++t)
            if (r[t] > best) {
                best = r[t];
                pos = t;
            }
    } else {
        pos = L - 1;
    }
    rows[b] = b * L + pos;
}

}  // namespace

extern "C" int mme_token_embed(const int64_t* ids, int B, int L, const void* tok, const void* pos, int d, void* out,
                               int ld_out, void* stream) {
    MME_REQUIRE(ids && tok && pos && out, "mme_token_embed: null pointer");
    MME_REQUIRE(B >= 0 && L > 0 && d % 8 == 0 && ld_out % 8 == 0 && ld_out >= d, "mme_token_embed: bad shape");
    if (B == 0) return MME_OK;
    const int rows = B * L;
    hipLaunchKernelGGL(token_embed_kernel, dim3(cdiv(rows, 4)), dim3(256), 0, as_stream(stream), ids, rows, L,
                       (const bf16*)tok, (const bf16*)pos, d, (bf16*)out, ld_out);
    return mme_check_launch("mme_token_embed");
}

extern "C" int mme_clip_embed_ln(const void* patch, int ld_patch, const void* cls, const void* pos, const void* gamma,
                                 const void* beta, float eps, void* out, int ld_out, int B, int P, int d,
                                 void* stream) {
    MME_REQUIRE(patch && cls && pos && gamma && beta && out, "mme_clip_embed_ln: null pointer");
    MME_REQUIRE(B >= 0 && P > 0 && d % 8 == 0 && d <= 8 * 64 * MAXC, "mme_clip_embed_ln: bad shape");
    MME_REQUIRE(ld_patch % 8 == 0 && ld_out % 8 == 0 && ld_patch >= d && ld_out >= d, "mme_clip_embed_ln: bad ld");
    if (B == 0) return MME_OK;
    hipLaunchKernelGGL(clip_embed_ln_kernel, dim3(cdiv((long)B * (P + 1), 4)), dim3(256), 0, as_stream(stream),
                       (const bf16*)patch, ld_patch, (const bf16*)cls, (const bf16*)pos, (const bf16*)gamma,
                       (const bf16*)beta, eps, (bf16*)out, ld_out, B, P, d);
    return mme_check_launch("mme_clip_embed_ln");
}

extern "C" int mme_text_pool_rows(const int64_t* ids, int B, int L, int64_t eos_id, int mode, int32_t* rows_out,
                                  void* stream) {
    MME_REQUIRE(ids && rows_out, "mme_text_pool_rows: null pointer");
    MME_REQUIRE(B >= 0 && L > 0 && mode >= 0 && mode <= 2, "mme_text_pool_rows: bad args");
    if (B == 0) return MME_OK;
    hipLaunchKernelGGL(text_pool_kernel, dim3(cdiv(B, 64)), dim3(64), 0, as_stream(stream), ids, B, L, eos_id, mode,
                       rows_out);
    return mme_check_launch("mme_text_pool_rows");
}
