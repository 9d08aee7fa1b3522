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
    asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(gsrc), "s"(m0) : "memory", "m0");
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
            return 0.5f * x * (1.0f + erff(x * 0.7071067811865476f));
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
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 pk_fma(f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); }
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
            return f32x2{apply_act(x.x, act), apply_act(x.y, act)};
        default:
            return x;
    }
}
