// bf16 MFMA GEMM for the ViT / text-transformer projections (gfx950).
//
//   C[M,N] = act(A[M,K] . B[N,K]^T + bias) + residual[r(row)]
//
// Both operands are K-contiguous ("TN"): A = activations [tokens, in],
// B = nn.Linear weight [out, in] exactly as HF stores it, so no weight
// transpose is ever materialised. This is the op behind every nn.Linear /
// patch Conv2d of SiglipEncoderLayer (TF:models/siglip/modeling_siglip.py:268-322)
// and CLIPEncoderLayer (TF:models/clip/modeling_clip.py).
//
// Structure (cdna_hip_programming.md §5):
//   * block tile BM x BN x 64, 8 waves (4 x 2) or 4 waves (2 x 2), each wave a
//     64 x 64 sub-tile of 4 x 4 v_mfma_f32_16x16x32_bf16 accumulators;
//   * A/B tiles staged HBM -> LDS with global_load_lds_dwordx4 (LDS-DMA),
//     double-buffered: the DMA of K-tile t+1 is in flight while tile t feeds
//     the MFMAs, one barrier per K-tile;
//   * LDS image [row][64] (128-B rows) XOR-swizzled on 16-B chunks
//     (chunk ^ ((row>>1)&7)), applied on the per-lane SOURCE address (the
//     DMA destination is lane-linear) and on the ds_read_b128 address, which
//     makes every 16-lane ds_read_b128 group conflict-free;
//   * XCD-aware block remap so tiles that share an A row-panel run on one XCD
//     (one L2).

#include "gemm_core.h"

namespace {
using namespace gemmcore;

struct GemmArgs {
    const bf16* A;
    const bf16* B;
    void* C;
    const bf16* bias;
    const bf16* res;
    int lda, ldb, ldc, ldr;
    int M, N, K;
    int res_period, act, out_f32;
};

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

template <class C, int GROUP_M>
__global__ __launch_bounds__(C::NT) void gemm_tn_kernel(GemmArgs p) {
    __shared__ __attribute__((aligned(16))) char lds[C::LDS];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wave / C::WN, wn = wave % C::WN;

    const int nbm = (p.M + C::BM - 1) / C::BM;
    const int nbn = (p.N + C::BN - 1) / C::BN;
    const int tile = xcd_remap(blockIdx.x, gridDim.x);
    int bm, bn;
    tile_coords<GROUP_M>(tile, nbm, nbn, bm, bn);
    const int m0 = bm * C::BM;
    const int n0 = bn * C::BN;

    f32x4 acc[C::FM][C::FN];
    mainloop<C>(p.A, p.lda, p.M, m0, p.B, p.ldb, p.N, n0, p.K, lds, acc, wave, lane);

    // epilogue: fp32 acc -> +bias -> act -> +residual -> bf16 / fp32
#pragma unroll
    for (int j = 0; j < C::FN; ++j) {
        const int col = n0 + wn * C::TN + j * 16 + (lane & 15);
        if (col >= p.N) continue;
        const float bv = p.bias ? bf2f(p.bias[col]) : 0.f;
#pragma unroll
        for (int i = 0; i < C::FM; ++i) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = m0 + wm * C::TM + i * 16 + 4 * (lane >> 4) + r;
                if (row >= p.M) continue;
                float v = apply_act(acc[i][j][r] + bv, p.act);
                if (p.res) {
                    const int rr = p.res_period ? row % p.res_period : row;
                    v += bf2f(p.res[(size_t)rr * p.ldr + col]);
                }
                if (p.out_f32)
                    reinterpret_cast<float*>(p.C)[(size_t)row * p.ldc + col] = v;
                else
                    reinterpret_cast<bf16*>(p.C)[(size_t)row * p.ldc + col] = f2bf(v);
            }
        }
    }
}

template <class C, int GROUP_M>
int launch(const GemmArgs& a, hipStream_t s) {
    const int nbm = (a.M + C::BM - 1) / C::BM, nbn = (a.N + C::BN - 1) / C::BN;
    hipLaunchKernelGGL((gemm_tn_kernel<C, GROUP_M>), dim3(nbm * nbn), dim3(C::NT), 0, s, a);
    return mme_check_launch("mme_gemm");
}

using BigCfg = Cfg<256, 128, 4, 2>;
using SqCfg = Cfg<256, 256, 2, 4>;
using SmallCfg = Cfg<128, 128, 2, 2>;

int g_variant = -1;  // dev-only override (tools/gemm_bench.py)

}  // namespace

extern "C" int mme_gemm_variant(int v) {
    g_variant = v;
    return MME_OK;
}

extern "C" int mme_gemm(const void* A, int lda, const void* B, int ldb, void* Cp, int ldc, int M, int N, int K,
                        const void* bias, const void* residual, int ldr, int res_period, int act, int out_f32,
                        void* stream) {
    MME_REQUIRE(A && B && Cp, "mme_gemm: null operand");
    MME_REQUIRE(M > 0 && N > 0 && K > 0, "mme_gemm: empty shape M=%d N=%d K=%d", M, N, K);
    MME_REQUIRE(K % BK == 0, "mme_gemm: K=%d must be a multiple of %d (pad weights/activations)", K, BK);
    MME_REQUIRE(lda % 8 == 0 && ldb % 8 == 0, "mme_gemm: lda/ldb must be multiples of 8 (16-B rows)");
    MME_REQUIRE(lda >= K && ldb >= K && ldc >= N, "mme_gemm: leading dim smaller than the row");
    MME_REQUIRE(((uintptr_t)A & 15) == 0 && ((uintptr_t)B & 15) == 0, "mme_gemm: A/B must be 16-byte aligned");
    MME_REQUIRE(!residual || ldr >= N, "mme_gemm: ldr < N");
    MME_REQUIRE(res_period >= 0, "mme_gemm: res_period < 0");
    MME_REQUIRE(act >= MME_ACT_NONE && act <= MME_ACT_GELU_ERF, "mme_gemm: bad act %d", act);
    GemmArgs a{(const bf16*)A, (const bf16*)B, Cp, (const bf16*)bias, (const bf16*)residual,
               lda, ldb, ldc, ldr, M, N, K, res_period, act, out_f32};
    hipStream_t s = as_stream(stream);
    switch (g_variant) {
        case 0: return launch<BigCfg, 1>(a, s);
        case 1: return launch<BigCfg, 4>(a, s);
        case 2: return launch<BigCfg, 8>(a, s);
        case 3: return launch<SqCfg, 1>(a, s);
        case 4: return launch<SqCfg, 4>(a, s);
        case 5: return launch<SqCfg, 8>(a, s);
        case 6: return launch<SmallCfg, 8>(a, s);
        default: break;
    }
    if ((long)M * N >= 2048L * 1024) return launch<BigCfg, 1>(a, s);
    return launch<SmallCfg, 1>(a, s);
}
