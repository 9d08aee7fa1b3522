// Shared MFMA GEMM mainloop pieces (LDS-DMA staging, swizzled LDS image,
// 16x16x32 bf16 MFMA tile) used by gemm.hip and retrieval.hip.
#pragma once
#include "common.h"

namespace gemmcore {

constexpr int BK = 64;

template <int BM_, int BN_, int WM_, int WN_>
struct Cfg {
    static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_;
    static constexpr int NW = WM * WN, NT = NW * 64;
    static constexpr int TM = BM / WM, TN = BN / WN;
    static constexpr int FM = TM / 16, FN = TN / 16;
    static constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
    static constexpr int STAGE = A_BYTES + B_BYTES;
    static constexpr int LDS = 2 * STAGE;
    static constexpr int A_LOADS = A_BYTES / 1024 / NW;
    static constexpr int B_LOADS = B_BYTES / 1024 / NW;
    static_assert(A_LOADS * 1024 * NW == A_BYTES, "A tile must split evenly into 1 KiB DMA pieces");
    static_assert(B_LOADS * 1024 * NW == B_BYTES, "B tile must split evenly into 1 KiB DMA pieces");
};

__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

// Bijective XCD remap (cdna_hip_programming.md §5, "XCD swizzle must be bijective").
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
    const int xcd = bid & 7, loc = bid >> 3;
    const int q = nwg >> 3, r = nwg & 7;
    const int start = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
    return start + loc;
}

// Tile order: XCD remap (each XCD gets a contiguous range of tile ids), then
// GROUP_M-row bands walked column-major inside the band, so the 32 tiles an
// XCD runs concurrently form a GROUP_M x (32/GROUP_M) patch that shares A row
// panels and B column panels in that XCD's L2.
template <int GROUP_M>
__device__ __forceinline__ void tile_coords(int tile, int nbm, int nbn, int& bm, int& bn) {
    if (GROUP_M <= 1) {
        bm = tile / nbn;
        bn = tile % nbn;
        return;
    }
    const int per_group = GROUP_M * nbn;
    const int gid = tile / per_group;
    const int first_m = gid * GROUP_M;
    const int gsz = min(nbm - first_m, GROUP_M);
    const int r = tile % per_group;
    bm = first_m + r % gsz;
    bn = r / gsz;
}

// Pipelined-kernel helpers: counted vmcnt / lgkmcnt waits (immediates) and
// inline-asm fragment reads (hipcc's waitcnt pass would otherwise drain
// lgkmcnt(0) at loop heads).
template <int N>
__device__ __forceinline__ void vm_wait() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
template <int N>
__device__ __forceinline__ void lgkm_wait() {
    asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
    __builtin_amdgcn_sched_barrier(0);
}
template <int OFF>
__device__ __forceinline__ void ds_read16(bf16x8& r, unsigned addr) {
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "n"(OFF));
}

template <class C>
__device__ __forceinline__ void stage_tile(const bf16* __restrict__ A, int lda, int M, int m0,
                                           const bf16* __restrict__ B, int ldb, int N, int n0, int k0,
                                           char* lds_stage, int wave, int lane) {
#pragma unroll
    for (int i = 0; i < C::A_LOADS; ++i) {
        const int c = wave * C::A_LOADS + i;
        const int row = c * 8 + (lane >> 3);
        const int grow = min(m0 + row, M - 1);
        const bf16* src = A + (size_t)grow * lda + k0 + swz(row, lane & 7) * 8;
        glds16(src, lds_stage + c * 1024);
    }
#pragma unroll
    for (int i = 0; i < C::B_LOADS; ++i) {
        const int c = wave * C::B_LOADS + i;
        const int row = c * 8 + (lane >> 3);
        const int grow = min(n0 + row, N - 1);
        const bf16* src = B + (size_t)grow * ldb + k0 + swz(row, lane & 7) * 8;
        glds16(src, lds_stage + C::A_BYTES + c * 1024);
    }
}

template <class C>
__device__ __forceinline__ void mma_tile(const char* lds_stage, f32x4 (&acc)[C::FM][C::FN], int wm, int wn,
                                         int lane) {
    const char* As = lds_stage;
    const char* Bs = lds_stage + C::A_BYTES;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
        const int chunk = ks * 4 + (lane >> 4);
        bf16x8 a[C::FM], b[C::FN];
#pragma unroll
        for (int i = 0; i < C::FM; ++i) {
            const int row = wm * C::TM + i * 16 + (lane & 15);
            a[i] = *reinterpret_cast<const bf16x8*>(As + row * 128 + (swz(row, chunk) << 4));
        }
#pragma unroll
        for (int j = 0; j < C::FN; ++j) {
            const int row = wn * C::TN + j * 16 + (lane & 15);
            b[j] = *reinterpret_cast<const bf16x8*>(Bs + row * 128 + (swz(row, chunk) << 4));
        }
#pragma unroll
        for (int i = 0; i < C::FM; ++i)
#pragma unroll
            for (int j = 0; j < C::FN; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
}


// Full K loop: acc += A[m0:m0+BM, :K] . B[n0:n0+BN, :K]^T, double-buffered
// LDS-DMA staging, one barrier per 64-deep K-tile. Leaves no DMA in flight.
template <class C>
__device__ __forceinline__ void mainloop(const bf16* __restrict__ A, int lda, int M, int m0,
                                         const bf16* __restrict__ B, int ldb, int N, int n0, int K, char* lds,
                                         f32x4 (&acc)[C::FM][C::FN], int wave, int lane) {
    const int wm = wave / C::WN, wn = wave % C::WN;
#pragma unroll
    for (int i = 0; i < C::FM; ++i)
#pragma unroll
        for (int j = 0; j < C::FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int nk = K / BK;
    stage_tile<C>(A, lda, M, m0, B, ldb, N, n0, 0, lds, wave, lane);
    for (int kt = 0; kt < nk; ++kt) {
        char* cur = lds + (kt & 1) * C::STAGE;
        wait_vmcnt0();
        __syncthreads();
        if (kt + 1 < nk)
            stage_tile<C>(A, lda, M, m0, B, ldb, N, n0, (kt + 1) * BK, lds + ((kt + 1) & 1) * C::STAGE, wave, lane);
        mma_tile<C>(cur, acc, wm, wn, lane);
    }
}
}  // namespace gemmcore
