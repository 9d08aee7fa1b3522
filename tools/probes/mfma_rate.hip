// MFMA throughput by instruction shape with every CU busy (dev probe).
//
// 8 waves per CU (one 512-thread block per CU, 2 waves per SIMD, like the GEMM), each
// running a dependency-free stream of bf16 MFMAs on register operands filled with
// random non-zero values: v_mfma_f32_16x16x32_bf16 (the GEMM's) vs v_mfma_f32_32x32x16_bf16
// (same MACs per cycle; twice the MACs per operand byte and per instruction). Under a
// power cap the chip clock, not the issue rate, may set the difference.
//
//   hipcc -O3 --offload-arch=gfx950 tools/probes/mfma_rate.hip -o tools/probes/mfma_rate
#include <hip/hip_runtime.h>

#include <cstdio>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ bf16x8 rnd8(unsigned s) {
    bf16x8 v;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        s = s * 1664525u + 1013904223u;
        v[e] = (__bf16)((float)((s >> 9) & 0xffff) * (1.0f / 65536.0f) - 0.5f);
    }
    return v;
}

template <bool BIG, bool ZERO>
__global__ __launch_bounds__(512) void mfma_stream(int iters, float* sink) {
    const unsigned seed = ZERO ? 0u : (blockIdx.x * 512u + threadIdx.x) * 2654435761u + 7u;
    bf16x8 a[4], b[2];
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = ZERO ? bf16x8{} : rnd8(seed + 17u * i);
#pragma unroll
    for (int j = 0; j < 2; ++j) b[j] = ZERO ? bf16x8{} : rnd8(seed + 1000u + 31u * j);
    float out = 0.f;
    if (BIG) {  // 128 x 64 wave tile as 4 x 2 tiles of 32 x 32: 8 accumulators x 16
        f32x16 acc[4][2] = {};
        for (int it = 0; it < iters; ++it) {
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b[j], a[i], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b[j ^ 1], a[i ^ 1], acc[i][j], 0, 0, 0);
                }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int e = 0; e < 16; ++e) out += acc[i][j][e];
    } else {  // the same tile as 8 x 4 tiles of 16 x 16
        f32x4 acc[8][4] = {};
        for (int it = 0; it < iters; ++it) {
#pragma unroll
            for (int i = 0; i < 8; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j & 1], a[i & 3], acc[i][j], 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int e = 0; e < 4; ++e) out += acc[i][j][e];
    }
    if (out == 1234.5f) sink[blockIdx.x] = out;
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    float* sink;
    if (hipMalloc(&sink, 4096 * sizeof(float)) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int iters = 20000;
    // MACs per iteration per wave: 16x16x32 form 32 x 8192; 32x32x16 form 16 x 16384 -- equal
    const double flops = 2.0 * 262144.0 * iters * 8 * cus;
    for (int rep = 0; rep < 3; ++rep)
        for (int form = 0; form < 4; ++form) {
            hipEventRecord(e0);
            if (form == 0) hipLaunchKernelGGL((mfma_stream<false, false>), dim3(cus), dim3(512), 0, 0, iters, sink);
            if (form == 1) hipLaunchKernelGGL((mfma_stream<true, false>), dim3(cus), dim3(512), 0, 0, iters, sink);
            if (form == 2) hipLaunchKernelGGL((mfma_stream<false, true>), dim3(cus), dim3(512), 0, 0, iters, sink);
            if (form == 3) hipLaunchKernelGGL((mfma_stream<true, true>), dim3(cus), dim3(512), 0, 0, iters, sink);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            printf("{\"rep\": %d, \"mfma\": \"%s\", \"operands\": \"%s\", \"ms\": %.3f, \"TFLOP_s\": %.1f}\n", rep,
                   (form & 1) ? "32x32x16" : "16x16x32", form >= 2 ? "zero" : "random", ms, flops / ms / 1e9);
        }
    hipFree(sink);
    return 0;
}
