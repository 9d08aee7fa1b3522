// ColPali late-interaction MaxSim (colpali_engine processor.score, main.py:467):
//   score[q,d] = bf16( sum_{i<q_len} bf16( max_{j<d_len} <Q[q,i], D[d,j]> ) )
// The reference evaluates einsum("bnd,csd->bcns") in bf16 on 10 x 10 chunks
// re-uploaded per chunk (main.py:451-470); the in-container port is
// TF:models/colpali/processing_colpali.py:256-270. max commutes with the
// monotone bf16 rounding, so the dots are accumulated in fp32 on the MFMA and
// rounded once after the max.
//
// Stage 1 (MFMA, compute-bound): for 256 query-token rows x a range of docs,
//   the doc tokens stream through LDS in 64-token tiles (LDS-DMA,
//   double-buffered, XOR-swizzled 256-B rows); S^T = Dtok . Qtok^T on
//   v_mfma_f32_16x16x32_bf16 puts one query token per lane and 4 doc tokens
//   per register, so the running max over doc tokens is lane-local.
//   Output: rowmax[d][query-token] (bf16).
// Stage 2 (bandwidth): score[q][d] = bf16(sum over the query's tokens), in a
//   fixed reduction order (deterministic).
#include "common.h"

namespace {

constexpr int MS_ROWS = 256;  // query-token rows per workgroup (8 waves x 32)
constexpr int MS_TILE = 64;   // doc tokens per LDS tile (64 x 256 B = 16 KiB)

struct MaxSimArgs {
    const bf16* Q;
    const bf16* D;
    const int32_t* d_lens;
    const uint8_t* d_zero;
    bf16* out;  // [nd][nrows]
    int nrows, nd, Ld, dpb;
};

__device__ __forceinline__ void ms_stage(const bf16* D, long tok0, long tok_end, char* buf, int wave, int lane) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int piece = wave * 2 + i;  // 4 token rows per 1 KiB piece
        const int row = piece * 4 + (lane >> 4);
        const long tok = min(tok0 + row, tok_end - 1);
        const int logical = (lane & 15) ^ (row & 15);
        glds16(D + tok * 128 + logical * 8, buf + piece * 1024);
    }
}

__global__ __launch_bounds__(512) void maxsim_rowmax_kernel(MaxSimArgs a) {
    __shared__ __attribute__((aligned(16))) char lds[2 * MS_TILE * 256];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = lane >> 4, li = lane & 15;
    const int r0 = blockIdx.x * MS_ROWS + wave * 32;
    const int d0 = blockIdx.y * a.dpb, d1 = min(a.nd, d0 + a.dpb);
    const long tok_begin = (long)d0 * a.Ld, tok_end = (long)d1 * a.Ld;
    const int ntok = (int)(tok_end - tok_begin);
    const int ntile = (ntok + MS_TILE - 1) / MS_TILE;

    bf16x8 qf[2][4];
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
        const int row = min(r0 + qb * 16 + li, a.nrows - 1);
#pragma unroll
        for (int ks = 0; ks < 4; ++ks)
            qf[qb][ks] = *reinterpret_cast<const bf16x8*>(a.Q + (long)row * 128 + ks * 32 + 8 * g);
    }
    float m[2] = {-INFINITY, -INFINITY};

    ms_stage(a.D, tok_begin, tok_end, lds, wave, lane);
    for (int t = 0; t < ntile; ++t) {
        const char* cur = lds + (t & 1) * MS_TILE * 256;
        wait_vmcnt0();
        __syncthreads();
        if (t + 1 < ntile)
            ms_stage(a.D, tok_begin + (long)(t + 1) * MS_TILE, tok_end, lds + ((t + 1) & 1) * MS_TILE * 256, wave,
                     lane);
        const int nblk = min(4, (ntok - t * MS_TILE) / 16);
        for (int blk = 0; blk < nblk; ++blk) {
            const int trel = t * MS_TILE + blk * 16;  // token offset from tok_begin
            const int doc = d0 + trel / a.Ld;
            const int tl = trel % a.Ld;
            const int len = a.d_lens[doc];
            const int row = blk * 16 + li;
            bf16x8 dv[4];
#pragma unroll
            for (int ks = 0; ks < 4; ++ks) {
                const int chunk = ks * 4 + g;
                dv[ks] = *reinterpret_cast<const bf16x8*>(cur + row * 256 + ((chunk ^ (row & 15)) << 4));
            }
#pragma unroll
            for (int qb = 0; qb < 2; ++qb) {
                f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int ks = 0; ks < 4; ++ks) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(dv[ks], qf[qb][ks], acc, 0, 0, 0);
                if (tl + 16 > len) {
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        if (tl + 4 * g + r >= len) acc[r] = -INFINITY;
                }
                m[qb] = fmaxf(m[qb], fmaxf(fmaxf(acc[0], acc[1]), fmaxf(acc[2], acc[3])));
            }
            if (tl + 16 == a.Ld) {  // end of this doc: reduce and emit
#pragma unroll
                for (int qb = 0; qb < 2; ++qb) {
                    float mm = fmaxf(m[qb], __shfl_xor(m[qb], 16, 64));
                    mm = fmaxf(mm, __shfl_xor(mm, 32, 64));
                    if (a.d_zero && a.d_zero[doc]) mm = fmaxf(mm, 0.f);
                    const int orow = r0 + qb * 16 + li;
                    if (g == 0 && orow < a.nrows) a.out[(long)doc * a.nrows + orow] = f2bf(mm);
                    m[qb] = -INFINITY;
                }
            }
        }
    }
}

// score[q][d] = bf16(sum_{i<q_len} rowmax[d][q*Lq + i]); GS lanes per (q, d).
template <int GS>
__global__ __launch_bounds__(256) void maxsim_sum_kernel(const bf16* __restrict__ rm, const int32_t* __restrict__ qlens,
                                                         int nq, int Lq, int nd, float* __restrict__ out) {
    const long pair = ((long)blockIdx.x * 256 + threadIdx.x) / GS;
    const int sub = threadIdx.x % GS;
    const bool live = pair < (long)nq * nd;
    const long pp = live ? pair : 0;
    const int q = pp / nd, d = pp % nd;
    const int ql = qlens[q];
    const bf16* src = rm + (long)d * nq * Lq + (long)q * Lq;
    float s = 0.f;
    for (int i = sub * 8; i < Lq; i += GS * 8) {
        const u16x8 u = *reinterpret_cast<const u16x8*>(src + i);
#pragma unroll
        for (int e = 0; e < 8; ++e)
            if (i + e < ql) s += bits2f(u[e]);
    }
#pragma unroll
    for (int o = GS / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if (live && sub == 0) out[(long)q * nd + d] = bf2f(f2bf(s));
}

}  // namespace

extern "C" size_t mme_maxsim_workspace_bytes(int nq, int Lq, int nd) {
    return (size_t)nq * Lq * nd * sizeof(uint16_t) + 256;
}

extern "C" int mme_maxsim(const void* Q, const int32_t* q_lens, int nq, int Lq, const void* D, const int32_t* d_lens,
                          const uint8_t* d_zero, int nd, int Ld, int dim, float* out, void* workspace, size_t ws_bytes,
                          void* stream) {
    MME_REQUIRE(Q && q_lens && D && d_lens && out && workspace, "mme_maxsim: null pointer");
    MME_REQUIRE(dim == 128, "mme_maxsim: dim=%d unsupported (ColPali projection dim 128)", dim);
    MME_REQUIRE(nq >= 0 && nd >= 0 && Lq > 0 && Ld > 0, "mme_maxsim: bad shape");
    MME_REQUIRE(Ld % 16 == 0 && Lq % 8 == 0, "mme_maxsim: Ld %% 16 and Lq %% 8 must be 0 (pad with zeros)");
    MME_REQUIRE(ws_bytes >= mme_maxsim_workspace_bytes(nq, Lq, nd), "mme_maxsim: workspace too small");
    MME_REQUIRE(((uintptr_t)Q & 15) == 0 && ((uintptr_t)D & 15) == 0, "mme_maxsim: Q/D must be 16-byte aligned");
    if (nq == 0 || nd == 0) return MME_OK;
    hipStream_t s = as_stream(stream);
    const int nrows = nq * Lq;
    // ~8k doc tokens per workgroup
    const int dpb = max(1, 8192 / Ld);
    MaxSimArgs a{(const bf16*)Q, (const bf16*)D, d_lens, d_zero, (bf16*)workspace, nrows, nd, Ld, dpb};
    hipLaunchKernelGGL(maxsim_rowmax_kernel, dim3(cdiv(nrows, MS_ROWS), cdiv(nd, dpb)), dim3(512), 0, s, a);
    int rc = mme_check_launch("mme_maxsim(rowmax)");
    if (rc) return rc;
    const long pairs = (long)nq * nd;
    const bf16* rm = (const bf16*)workspace;
    if (Lq <= 64) {
        hipLaunchKernelGGL(maxsim_sum_kernel<4>, dim3(cdiv(pairs * 4, 256)), dim3(256), 0, s, rm, q_lens, nq, Lq, nd,
                           out);
    } else {
        hipLaunchKernelGGL(maxsim_sum_kernel<64>, dim3(cdiv(pairs * 64, 256)), dim3(256), 0, s, rm, q_lens, nq, Lq,
                           nd, out);
    }
    return mme_check_launch("mme_maxsim(sum)");
}
