// Row normalisations: LayerNorm (encoder) and the bf16 L2-normalise of the
// pooled embeddings. HBM-bound wavefront reductions: one 64-lane wave owns a
// row, 16-byte (8 x bf16) vector loads/stores, statistics in fp32 registers.
#include "common.h"

namespace {

constexpr int ROWS_PER_BLOCK = 4;  // 4 waves, one row each
constexpr int MAXC = 4;            // 16-B chunks per lane: d <= 8*64*4 = 2048

__device__ __forceinline__ void load_row(const bf16* xr, int nch, int lane, float (&v)[MAXC][8]) {
    u16x8 u[MAXC];  // every chunk in flight before the first wait (common.h load_chunk_or_zero)
#pragma unroll
    for (int c = 0; c < MAXC; ++c) u[c] = load_chunk_or_zero(xr, lane + c * 64, nch);
#pragma unroll
    for (int c = 0; c < MAXC; ++c)
#pragma unroll
        for (int e = 0; e < 8; ++e) v[c][e] = bits2f(u[c][e]);
}

// nn.LayerNorm on a bf16 row (TF:models/siglip/modeling_siglip.py:329-331):
// fp32 mean / biased variance, y = (x - mean) * rsqrt(var + eps) * gamma + beta.
// Round 5: one row per HALF wave (common.h ln_*_half), 8 rows per 256-thread block.
constexpr int LN_ROWS_PER_BLOCK = 8;
template <int MAXC>
__global__ __launch_bounds__(256) void layernorm_kernel(const bf16* __restrict__ x, int ldx,
                                                        const bf16* __restrict__ g, const bf16* __restrict__ b,
                                                        bf16* __restrict__ y, int ldy, int rows, int d, float eps,
                                                        const int32_t* __restrict__ idx) {
    const int row = blockIdx.x * LN_ROWS_PER_BLOCK + (threadIdx.x >> 5);
    const int hl = threadIdx.x & 31;
    if (row >= rows) return;  // the half wave's 32 lanes together (its shuffles stay inside the half)
    const long src = idx ? idx[row] : row;
    const int nch = d >> 3;
    float v[MAXC][8];
    u16x8 gu[MAXC], bu[MAXC];
    ln_load_half(x + src * ldx, nch, hl, v);
    ln_load_affine_half(g, b, nch, hl, gu, bu);  // in flight with the row (round 6)
    float mean, rstd;
    ln_stats_half(v, nch, hl, d, eps, mean, rstd);
    bf16* yr = y + (long)row * ldy;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {  // computed without a branch, stored where the chunk is in the row
        const int ch = hl + 32 * c;
        bf16x8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = f2bf((v[c][e] - mean) * rstd * bits2f(gu[c][e]) + bits2f(bu[c][e]));
        if (ch < nch) *reinterpret_cast<bf16x8*>(yr + ch * 8) = o;
    }
}

// LayerNorm statistics only (mean, rstd) per row, for a GEMM with the LayerNorm folded
// into its weights (mme_gemm_lnfold): same fp32 two-pass arithmetic as layernorm_kernel,
// 8 bytes written per row instead of the normalised row.
// Rows per wave (loads of all its rows issued before any reduction). Measured on 430 MB of
// SigLIP rows (tools/rowstats_bench.py): 1 row 4.7 TB/s, 2 rows 3.8, 4 rows 2.7 -- the
// pass wants waves, not bytes per wave.
constexpr int RS_ROWS = 1;
__global__ __launch_bounds__(256) void rowstats_kernel(const bf16* __restrict__ x, int ldx, float* __restrict__ st,
                                                       int rows, int d, float eps) {
    const int row0 = (blockIdx.x * ROWS_PER_BLOCK + (threadIdx.x >> 6)) * RS_ROWS;
    const int lane = threadIdx.x & 63;
    if (row0 >= rows) return;
    const int nch = d >> 3;
    float v[RS_ROWS][MAXC][8];
#pragma unroll
    for (int k = 0; k < RS_ROWS; ++k) load_row(x + (long)min(row0 + k, rows - 1) * ldx, nch, lane, v[k]);
#pragma unroll
    for (int k = 0; k < RS_ROWS; ++k) {
        float s = 0.f;
#pragma unroll
        for (int c = 0; c < MAXC; ++c)
#pragma unroll
            for (int e = 0; e < 8; ++e) s += v[k][c][e];
        const float mean = wave_sum(s) / d;
        float s2 = 0.f;
#pragma unroll
        for (int c = 0; c < MAXC; ++c) {
            if (lane + c * 64 < nch) {
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    const float t = v[k][c][e] - mean;
                    s2 += t * t;
                }
            }
        }
        const float rstd = rsqrtf(wave_sum(s2) / d + eps);
        if (lane == 0 && row0 + k < rows) *reinterpret_cast<float2*>(st + 2 * (long)(row0 + k)) = make_float2(mean, rstd);
    }
}

// out / out.norm(dim=-1, keepdim=True) on a bf16 tensor (main.py:414,434):
// torch reduces the norm in fp32, rounds it to bf16, then divides in fp32 and
// rounds the quotient: y = bf16(x / float(bf16(sqrt(sum x^2)))).
__global__ __launch_bounds__(256) void l2norm_kernel(const bf16* __restrict__ x, int ldx, bf16* __restrict__ y,
                                                     int ldy, int rows, int d) {
    const int row = blockIdx.x * ROWS_PER_BLOCK + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= rows) return;
    const int nch = d >> 3;
    float v[MAXC][8];
    load_row(x + (long)row * ldx, nch, lane, v);
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < MAXC; ++c)
#pragma unroll
        for (int e = 0; e < 8; ++e) s += v[c][e] * v[c][e];
    const float nrm = bf2f(f2bf(sqrtf(wave_sum(s))));
    bf16* yr = y + (long)row * ldy;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
        const int ch = lane + c * 64;
        if (ch < nch) {
            bf16x8 o;
#pragma unroll
            for (int e = 0; e < 8; ++e) o[e] = f2bf(v[c][e] / nrm);
            *reinterpret_cast<bf16x8*>(yr + ch * 8) = o;
        }
    }
}

}  // namespace

extern "C" int mme_layernorm(const void* x, int ldx, const void* gamma, const void* beta, void* y, int ldy, int rows,
                             int d, float eps, const int32_t* rows_idx, void* stream) {
    MME_REQUIRE(x && gamma && beta && y, "mme_layernorm: null pointer");
    MME_REQUIRE(rows >= 0 && d > 0 && d % 8 == 0 && d <= 8 * 64 * MAXC, "mme_layernorm: d=%d unsupported", d);
    MME_REQUIRE(ldx % 8 == 0 && ldy % 8 == 0 && ldx >= d && ldy >= d, "mme_layernorm: bad leading dims");
    if (rows == 0) return MME_OK;
    const int nch = d / 8, mc = (nch + 31) / 32;  // chunks per lane of a half-wave row
    const dim3 grid(cdiv(rows, LN_ROWS_PER_BLOCK)), block(256);
    if (mc <= 3)
        hipLaunchKernelGGL(layernorm_kernel<3>, grid, block, 0, as_stream(stream), (const bf16*)x, ldx, (const bf16*)gamma,
                           (const bf16*)beta, (bf16*)y, ldy, rows, d, eps, rows_idx);
    else if (mc <= 4)
        hipLaunchKernelGGL(layernorm_kernel<4>, grid, block, 0, as_stream(stream), (const bf16*)x, ldx, (const bf16*)gamma,
                           (const bf16*)beta, (bf16*)y, ldy, rows, d, eps, rows_idx);
    else if (mc <= 5)
        hipLaunchKernelGGL(layernorm_kernel<5>, grid, block, 0, as_stream(stream), (const bf16*)x, ldx, (const bf16*)gamma,
                           (const bf16*)beta, (bf16*)y, ldy, rows, d, eps, rows_idx);
    else
        hipLaunchKernelGGL(layernorm_kernel<LNH_MAXC>, grid, block, 0, as_stream(stream), (const bf16*)x, ldx,
                           (const bf16*)gamma, (const bf16*)beta, (bf16*)y, ldy, rows, d, eps, rows_idx);
    return mme_check_launch("mme_layernorm");
}

extern "C" int mme_l2norm(const void* x, int ldx, void* y, int ldy, int rows, int d, void* stream) {
    MME_REQUIRE(x && y, "mme_l2norm: null pointer");
    MME_REQUIRE(rows >= 0 && d > 0 && d % 8 == 0 && d <= 8 * 64 * MAXC, "mme_l2norm: d=%d unsupported", d);
    MME_REQUIRE(ldx % 8 == 0 && ldy % 8 == 0 && ldx >= d && ldy >= d, "mme_l2norm: bad leading dims");
    if (rows == 0) return MME_OK;
    hipLaunchKernelGGL(l2norm_kernel, dim3(cdiv(rows, ROWS_PER_BLOCK)), dim3(256), 0, as_stream(stream),
                       (const bf16*)x, ldx, (bf16*)y, ldy, rows, d);
    return mme_check_launch("mme_l2norm");
}

extern "C" int mme_rowstats(const void* x, int ldx, int rows, int d, float eps, float* stats, void* stream) {
    MME_REQUIRE(x && stats, "mme_rowstats: null pointer");
    MME_REQUIRE(rows >= 0 && d > 0 && d % 8 == 0 && d <= 8 * 64 * MAXC, "mme_rowstats: d=%d unsupported", d);
    MME_REQUIRE(ldx % 8 == 0 && ldx >= d && ((uintptr_t)stats & 7) == 0, "mme_rowstats: bad leading dim / alignment");
    if (rows == 0) return MME_OK;
    hipLaunchKernelGGL(rowstats_kernel, dim3(cdiv(rows, ROWS_PER_BLOCK * RS_ROWS)), dim3(256), 0, as_stream(stream),
                       (const bf16*)x, ldx, stats, rows, d, eps);
    return mme_check_launch("mme_rowstats");
}
