// Per-CU global store throughput of the GEMM epilogue's store pattern (dev probe).
//
// Each 512-thread block writes `tiles` 256 x 256 bf16 tiles (128 KiB each) the way
// gemm_epilogue_lds does: thread c of the block stores 16-B chunk c, c + 512, ... of the
// tile (32 chunks = one 512-B row segment per 32 lanes), rows `ld` elements apart, with
// non-temporal (nt = 1) or plain stores. Launch with few blocks (per-CU limit, HBM idle)
// and with one block per CU (chip limit).
//
//   hipcc -O3 --offload-arch=gfx950 tools/probes/store_bw.hip -o tools/probes/store_bw
//   tools/probes/store_bw
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));

template <bool NT>
__global__ __launch_bounds__(512) void store_tiles(unsigned short* out, int ld, int tiles, int rows_total) {
    const int tid = threadIdx.x;
    for (int t = 0; t < tiles; ++t) {
        const int tile = blockIdx.x * tiles + t;
        const int m0 = (tile * 256) % (rows_total - 256);
        u16x8 v = {(unsigned short)t, 1, 2, 3, 4, 5, 6, (unsigned short)tid};
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int c = tid + q * 512;
            const int row = c / 32, cc = c % 32;
            u16x8* p = reinterpret_cast<u16x8*>(out + (size_t)(m0 + row) * ld + cc * 8);
            if (NT)
                __builtin_nontemporal_store(v, p);
            else
                *p = v;
        }
        __syncthreads();
    }
}

int main() {
    const int ld = 4352, rows = 174080;
    unsigned short* out;
    if (hipMalloc(&out, (size_t)rows * ld * 2) != hipSuccess) return 1;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int tiles = 40;
    for (int nt = 0; nt < 2; ++nt) {
        for (int blocks : {8, 32, 64, 128, cus}) {
            float best = 1e30f;
            for (int rep = 0; rep < 4; ++rep) {
                hipEventRecord(a);
                if (nt)
                    hipLaunchKernelGGL(store_tiles<true>, dim3(blocks), dim3(512), 0, 0, out, ld, tiles, rows);
                else
                    hipLaunchKernelGGL(store_tiles<false>, dim3(blocks), dim3(512), 0, 0, out, ld, tiles, rows);
                hipEventRecord(b);
                hipEventSynchronize(b);
                float ms = 0;
                hipEventElapsedTime(&ms, a, b);
                if (ms < best) best = ms;
            }
            const double bytes = (double)blocks * tiles * 131072.0;
            printf("{\"nt\": %d, \"blocks\": %d, \"ms\": %.4f, \"GB_s_total\": %.1f, \"GB_s_per_block\": %.2f, "
                   "\"us_per_tile\": %.2f}\n",
                   nt, blocks, best, bytes / best / 1e6, bytes / best / 1e6 / blocks, best * 1e3 / tiles);
        }
    }
    hipFree(out);
    return 0;
}
