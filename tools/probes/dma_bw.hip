// LDS-DMA (global_load_lds_dwordx4) throughput per CU by piece shape (dev probe).
//
// The GEMM stages a 256 x 256 tile's A and B panels (512 rows of K = 1152 bf16) through
// a 4-slot LDS ring of 32-deep stages: a 1 KiB piece (one wave-instruction) is 16 rows
// x 64 B, so every row segment is HALF a 128-B line. This probe streams the same bytes
// with the same ring, counted vmcnt waits and one barrier per stage, in two piece shapes:
//   shape 0: 16 rows x 64 B pieces, one 32-deep stage (32 KiB) per step (the GEMM's)
//   shape 1:  8 rows x 128 B pieces: a step moves 256 of the rows x 64 deep (same 32 KiB,
//             same ring and waits; two steps cover a 64-deep stage pair)
// and reports GB/s per CU, with every block reading the same 512 rows (L2-resident)
// or its own 512-row panel of a 75 MB table (Infinity-Cache-resident).
//
//   hipcc -O3 --offload-arch=gfx950 tools/probes/dma_bw.hip -o tools/probes/dma_bw
#include <hip/hip_runtime.h>

#include <cstdio>

#define GLB __attribute__((address_space(1)))
#define LDSA __attribute__((address_space(3)))

__device__ __forceinline__ void glds16(const void* g, void* l) {
    __builtin_amdgcn_global_load_lds((const GLB void*)g, (LDSA void*)l, 16, 0, 0);
}
template <int N>
__device__ __forceinline__ void vm_wait() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int SHAPE, bool BAR>
__global__ __launch_bounds__(512) void dma_stream(const unsigned short* A, int K, int rows_total, int shared,
                                                  int steps, float* sink) {
    __shared__ __attribute__((aligned(16))) char lds[4 * 32768];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int base = shared ? 0 : (blockIdx.x * 512) % (rows_total - 512);
    const unsigned short* src[4];
    if (SHAPE == 0) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int piece = wave * 4 + q, row = piece * 16 + (lane >> 2);
            src[q] = A + (size_t)(base + row) * K + (lane & 3) * 8;
        }
    } else {  // a step's 32 KiB = half the 512 rows x 64 deep; the halves alternate
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int piece = wave * 4 + q, row = piece * 8 + (lane >> 3);
            src[q] = A + (size_t)(base + row) * K + (lane & 7) * 8;
        }
    }
    const int nk = K / 32;
    for (int t = 0; t < steps; ++t) {
        char* slot = lds + (t & 3) * 32768;
        const int k = t % nk;
        // shape 0: stage k, all 512 rows x 32 deep; shape 1: rows 256 (k & 1) .. + 256, 64 deep from 64 (k >> 1)
        const size_t off = SHAPE == 0 ? (size_t)k * 32 : (size_t)(k & 1) * 256 * K + (k >> 1) * 64;
#pragma unroll
        for (int q = 0; q < 4; ++q) glds16(src[q] + off, slot + (wave * 4 + q) * 1024);
        vm_wait<12>();
        if (BAR) __builtin_amdgcn_s_barrier();
    }
    vm_wait<0>();
    __syncthreads();
    if (tid == 0) sink[blockIdx.x] = (float)lds[(blockIdx.x * 16) & 131071];
}

int main() {
    const int K = 1152, rows = 32768;
    unsigned short* A;
    float* sink;
    if (hipMalloc(&A, (size_t)rows * K * 2) != hipSuccess) return 1;
    if (hipMalloc(&sink, 4096 * sizeof(float)) != hipSuccess) return 1;
    hipMemset(A, 0, (size_t)rows * K * 2);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int steps = 1440;  // 40 passes over K = 1152 (32-deep)
    for (int shared = 1; shared >= 0; --shared)
        for (int bar = 1; bar >= 0; --bar)
            for (int shape = 0; shape < 2; ++shape)
                for (int blocks : {cus, 4 * cus}) {
                    float best = 1e30f;
                    for (int rep = 0; rep < 4; ++rep) {
                        hipEventRecord(e0);
                        if (shape == 0 && bar)
                            hipLaunchKernelGGL((dma_stream<0, true>), dim3(blocks), dim3(512), 0, 0, A, K, rows, shared, steps, sink);
                        else if (shape == 0)
                            hipLaunchKernelGGL((dma_stream<0, false>), dim3(blocks), dim3(512), 0, 0, A, K, rows, shared, steps, sink);
                        else if (bar)
                            hipLaunchKernelGGL((dma_stream<1, true>), dim3(blocks), dim3(512), 0, 0, A, K, rows, shared, steps, sink);
                        else
                            hipLaunchKernelGGL((dma_stream<1, false>), dim3(blocks), dim3(512), 0, 0, A, K, rows, shared, steps, sink);
                        hipEventRecord(e1);
                        hipEventSynchronize(e1);
                        float ms = 0;
                        hipEventElapsedTime(&ms, e0, e1);
                        if (ms < best) best = ms;
                    }
                    const double bytes = (double)blocks * steps * 32768.0;
                    printf("{\"shape\": \"%s\", \"l2_shared\": %d, \"barrier\": %d, \"blocks\": %d, \"ms\": %.3f, "
                           "\"TB_s\": %.2f, \"GB_s_per_CU\": %.1f}\n",
                           shape ? "8x128B" : "16x64B", shared, bar, blocks, best, bytes / best / 1e9,
                           bytes / best / 1e6 / cus);
                }
    hipFree(A);
    hipFree(sink);
    return 0;
}
