// Shared device helpers for libmme (gfx950 / CDNA4 only).
//
// Everything here is written for 64-lane wavefronts and the gfx950 MFMA /
// LDS-DMA builtins; there is no other target.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

#include "../../include/mme.h"

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));
typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));

#define LDS_AS __attribute__((address_space(3)))
#define GLB_AS __attribute__((address_space(1)))

// ---------------------------------------------------------------------------
// host-side error plumbing (defined in capi.cpp)
// ---------------------------------------------------------------------------
int mme_set_error(int code, const char* fmt, ...);
int mme_check_launch(const char* what);

#define MME_REQUIRE(cond, ...)                                  \
    do {                                                        \
        if (!(cond)) return mme_set_error(MME_ERR_ARG, __VA_ARGS__); \
    } while (0)

static inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }
static inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }

// ---------------------------------------------------------------------------
// device helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ float bf2f(bf16 x) { return (float)x; }
__device__ __forceinline__ bf16 f2bf(float x) { return (bf16)x; }  // RNE (v_cvt_pk_bf16_f32)

__device__ __forceinline__ float bits2f(unsigned short u) {
    return __uint_as_float(((unsigned)u) << 16);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

// ---------------------------------------------------------------------------
// LayerNorm rows held by HALF a wave (round 5): lane hl = lane & 31 of half h = lane >> 5 owns the 16-B
// chunks hl + 32 c of its row, c < LNH_MAXC (d <= 2 048). At the encoder widths this fills the lanes
// where a whole wave per row left a third of them idle on the last chunk (d = 1 280: 160 chunks = 5 per
// lane, against 64 + 64 + 32 over a 64-lane wave; d = 1 152: 4.5 against 3 x 64 for 144). The bf16
// LayerNorm (norm.hip layernorm_kernel) and the LayerNorm -> mx8 kernel (mx.hip layernorm_mx_kernel)
// share these helpers, so their statistics are the same bits (tests/test_gpu_mx.py).
// ---------------------------------------------------------------------------
constexpr int LNH_MAXC = 8;  // d <= 2 048; the kernels instantiate the smallest count that holds their d

__device__ __forceinline__ float half_sum(float v) {
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// 16-B chunk ch of a row (8 bf16 as bits), or zeros when ch >= nch. The load itself is unconditional
// (clamped to chunk nch - 1, nch >= 1) and masked afterwards, so every chunk of a row is in flight before
// the first wait. Round 6: with the load inside a per-lane `if (ch < nch)`, hipcc waited for each chunk in
// its branch (s_waitcnt vmcnt(0) after every load): one memory round trip per chunk in series.
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ u16x8 load_chunk_or_zero(const bf16* __restrict__ xr, int ch, int nch) {
    const u32x4 u = *reinterpret_cast<const u32x4*>(xr + min(ch, nch - 1) * 8);
    const unsigned m = ch < nch ? 0xffffffffu : 0u;
    return __builtin_bit_cast(u16x8, u & u32x4{m, m, m, m});
}

template <int MAXC>
__device__ __forceinline__ void ln_load_half(const bf16* __restrict__ xr, int nch, int hl, float (&v)[MAXC][8]) {
    u16x8 u[MAXC];
#pragma unroll
    for (int c = 0; c < MAXC; ++c) u[c] = load_chunk_or_zero(xr, hl + 32 * c, nch);
#pragma unroll
    for (int c = 0; c < MAXC; ++c)
#pragma unroll
        for (int e = 0; e < 8; ++e) v[c][e] = bits2f(u[c][e]);
}

// gamma / beta chunks of a half-wave row's lane (zeros past the row), issued with the row's own loads
template <int MAXC>
__device__ __forceinline__ void ln_load_affine_half(const bf16* __restrict__ g, const bf16* __restrict__ b, int nch,
                                                    int hl, u16x8 (&gu)[MAXC], u16x8 (&bu)[MAXC]) {
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
        gu[c] = load_chunk_or_zero(g, hl + 32 * c, nch);
        bu[c] = load_chunk_or_zero(b, hl + 32 * c, nch);
    }
}

// fp32 mean and rsqrt(biased variance + eps), two passes over the registers (nn.LayerNorm)
template <int MAXC>
__device__ __forceinline__ void ln_stats_half(const float (&v)[MAXC][8], int nch, int hl, int d, float eps,
                                              float& mean, float& rstd) {
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < MAXC; ++c)
#pragma unroll
        for (int e = 0; e < 8; ++e) s += v[c][e];
    mean = half_sum(s) / d;
    float s2 = 0.f;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
        if (hl + 32 * c < nch) {
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const float t = v[c][e] - mean;
                s2 += t * t;
            }
        }
    }
    rstd = rsqrtf(half_sum(s2) / d + eps);
}

// async global -> LDS copy of 16 bytes per lane; LDS destination is the
// wave-uniform `lds_base` + lane*16 (gfx950 global_load_lds_dwordx4).
__device__ __forceinline__ void glds16(const void* gsrc, void* lds_base) {
    __builtin_amdgcn_global_load_lds((const GLB_AS void*)gsrc, (LDS_AS void*)lds_base, 16, 0, 0);
}

__device__ __forceinline__ void wait_vmcnt0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// glds16 issued from inline asm: the same global_load_lds_dwordx4, but invisible to hipcc's
// waitcnt pass, which otherwise drains it (vmcnt(0)) before any LDS read it cannot prove
// disjoint from the DMA's destination. The caller retires it with its own counted vmcnt
// wait + barrier before the bytes are read. `lds_base` must be wave-uniform (M0).
__device__ __forceinline__ void glds16_asm(const void* gsrc, void* lds_base) {
    const unsigned m0 = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(LDS_AS char*)lds_base);
    // s_nop 0: the M0 write -> LDS-DMA wait state (hipcc pads no hazard inside a statement)
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(gsrc), "s"(m0) : "memory", "m0");
}

typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 pk_fma(f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); }

// gelu(x) = x Phi(x) (nn.GELU(approximate="none"), the ViT-H / LAION-CLIP-H / MetaCLIP MLP) as a sigmoid:
// Phi(x) = 1 / (1 + 2^(x P(x^2))) with x P(x^2) ~= -log2(e) logit(Phi(x)), P of degree 6 in x^2
// (tools/gelu_erf_fit.py: minimax of |dPhi| on |x| <= 6.2 by linear programming; fit error 1.6e-8 in
// Phi). The error is absolute (minimax in |dPhi|): far in the negative tail, where |gelu| < 1.5e-5 and
// torch's own 0.5 x (1 + erf) loses its digits to cancellation, the relative error grows (5 % at x = -5);
// x P(x^2) is monotone, so no clamp: v_exp_f32 saturates to 0 or +inf and v_rcp_f32(inf) = 0 (gelu = x past
// x ~ 8, -0 below x ~ -8). Cost: the gelu_tanh form (one exp, one add, one rcp, three multiplies)
// plus five packed FMAs -- round 5's Numerical Recipes erfc fit (t = 1 / (1 + z / 2), nine FMAs of P(t),
// exp, select) took +19 % over bias-only on LAION's fc1, the tanh form +7 %
// (profiles/r05_v24_fc1_activation_cost.log). Accuracy in float32 (erf-equivalent absolute error
// 2 |gelu - x Phi(x)| / |x| against float64): 3.5e-7, against 3.9e-7 for the erfc fit and 2.1e-7 for
// torch's own fp32 formula 0.5 x (1 + erf(x / sqrt2)) with a correctly rounded erf
// (tests/test_host_logic.py, tests/test_gpu_kernels.py).
__device__ __forceinline__ f32x2 gelu_erf2(f32x2 x) {
    const f32x2 x2 = x * x;
    f32x2 p = pk_fma(x2, f32x2{-5.3743916e-09f, -5.3743916e-09f}, f32x2{3.93183313e-07f, 3.93183313e-07f});
    p = pk_fma(x2, p, f32x2{-1.15972562e-05f, -1.15972562e-05f});
    p = pk_fma(x2, p, f32x2{0.000160533178f, 0.000160533178f});
    p = pk_fma(x2, p, f32x2{9.14715347e-05f, 9.14715347e-05f});
    p = pk_fma(x2, p, f32x2{-0.104832388f, -0.104832388f});
    p = pk_fma(x2, p, f32x2{-2.30220985f, -2.30220985f});
    const f32x2 u = x * p;
    const f32x2 d = f32x2{__builtin_amdgcn_exp2f(u.x), __builtin_amdgcn_exp2f(u.y)} + 1.0f;
    return x * f32x2{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
}

// Activation codes shared by the GEMM epilogue and the host (mme.h MME_ACT_*).
// The sigmoid forms run on the transcendental unit (v_exp_f32 + v_rcp_f32, ~1 ulp
// each) instead of the libm tanhf / IEEE division sequences: in a GEMM epilogue the
// MFMA pipes idle while these run (fc1 with tanhf: ~780 TF/s vs ~1070 for the same
// shape without an activation). Results round to bf16, so the few-ulp fp32
// difference is below the output precision.
__device__ __forceinline__ float apply_act(float x, int act) {
    switch (act) {
        case MME_ACT_GELU_TANH: {  // gelu_pytorch_tanh: 0.5x(1 + tanh(u)) = x * sigmoid(2u)
            const float k1 = 0.044715f;
            const float c2 = -2.0f * 0.7978845608028654f * 1.4426950408889634f;  // -2 * sqrt(2/pi) * log2(e)
            const float e = __builtin_amdgcn_exp2f(c2 * x * (1.0f + k1 * x * x));
            return x * __builtin_amdgcn_rcpf(1.0f + e);
        }
        case MME_ACT_QUICK_GELU: {  // x * sigmoid(1.702 x)
            const float e = __builtin_amdgcn_exp2f(-1.702f * 1.4426950408889634f * x);
            return x * __builtin_amdgcn_rcpf(1.0f + e);
        }
        case MME_ACT_GELU_ERF:
            return gelu_erf2(f32x2{x, x}).x;
        default:
            return x;
    }
}

// The same activations on a pair of values with packed f32 math (v_pk_mul_f32 /
// v_pk_fma_f32 / v_pk_add_f32: two lanes' worth per 4-cycle issue); only the
// transcendentals stay per element. gelu_tanh argument as x * (c2 + c2 k1 x^2)
// (one multiply fewer than the scalar form; fp32 rounding differs by ~1 ulp,
// far below the bf16 output). Used by the GEMM epilogue, where these VALU
// cycles are pure overhead on the MFMA pipe (fc1: ~25 % of its epilogue time).
__device__ __forceinline__ f32x2 apply_act2(f32x2 x, int act) {
    switch (act) {
        case MME_ACT_GELU_TANH: {
            const float c2 = -2.0f * 0.7978845608028654f * 1.4426950408889634f;
            const f32x2 u = pk_fma(x * x, f32x2{c2 * 0.044715f, c2 * 0.044715f}, f32x2{c2, c2}) * x;
            const f32x2 d = f32x2{__builtin_amdgcn_exp2f(u.x), __builtin_amdgcn_exp2f(u.y)} + 1.0f;
            return x * f32x2{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
        }
        case MME_ACT_QUICK_GELU: {
            const f32x2 u = x * (-1.702f * 1.4426950408889634f);
            const f32x2 d = f32x2{__builtin_amdgcn_exp2f(u.x), __builtin_amdgcn_exp2f(u.y)} + 1.0f;
            return x * f32x2{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
        }
        case MME_ACT_GELU_ERF:
            return gelu_erf2(x);
        default:
            return x;
    }
}
