// Fused multi-head attention for the ViT / text encoders (flash-style, gfx950).
//
// softmax(Q K^T * scale + mask) V for one (batch, head, 128-query block) per
// workgroup, streaming 64-key K/V tiles through LDS with online softmax —
// replaces eager/SDPA attention of SiglipAttention / CLIPAttention
// (TF:models/siglip/modeling_siglip.py:228-247,273-306).
//
// Layout tricks (cdna_hip_programming.md §3, T10, T12):
//   * S^T = K . Q^T on v_mfma_f32_16x16x32_bf16 (+ one 16x16x16 step for the
//     72/80 head dims): the accumulator puts ONE query on each lane and 16 of
//     its keys in registers, so the row max / row sum are lane-local plus two
//     xor-shuffles (lanes l, l^16, l^32, l^48 share a query);
//   * those registers, packed to bf16, are directly the B operand of
//     O^T = V^T . P^T (the MFMA k-order is permuted identically on both
//     operands), so P never touches LDS;
//   * the V^T operand is read from the row-major V tile with
//     ds_read_b64_tr_b16 (hardware transpose), V rows padded to 80 elements
//     (160 B) which makes the transposed reads bank-conflict-free;
//   * head dims 72 and 80 run as 3 x K32 MFMA steps over a zero-padded 96-deep
//     reduction (same-shape accumulation chains only); the O^T accumulators
//     cover 5 d-tiles of 16 (80 columns).
//   * 4 waves x 32 query rows per workgroup: the K and V^T fragments read
//     from LDS feed two query tiles each.
//   * K/V tiles are double-buffered through registers: the global loads of
//     tile t+1 are issued before the MFMAs of tile t and written to the other
//     LDS buffer afterwards.
#include "common.h"

namespace {

template <int N>
__device__ __forceinline__ void vm_wait() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}


struct AttnArgs {
    const bf16* qkv;
    bf16* out;
    const int32_t* seq_lens;
    int ld, ldo, T, H, hd, causal;  // hd is also the kernel's template parameter
    float scale_log2;
};

template <int HD, int DIAG = 0, bool THR = false>
__global__ __launch_bounds__(256, 2) void attn_fwd_kernel(AttnArgs a) {
    // DIAG (dev builds, wrong results): 1 no K/V global loads, 2 no exp2, 3 no PV MFMA, 4 no QK MFMA
    // THR (round 4, kind 89): O and the weight sum rescaled only when a query's running max grows by
    // more than 2^8 in the exp2 domain (attn_hyb_kernel's XT 2), instead of on every tile
    // QK^T reduction depth covered by 16x16x32 steps: 64, or 96 for head dims
    // 72/80 zero-padded. Only same-shape MFMA accumulation chains are used: a
    // 16x16x16 tail step chained on a 16x16x32 result was observed to be
    // scheduled without the wait states it needs (wrong scores on gfx950).
    constexpr int HDP = HD == 64 ? 64 : 96;
    constexpr int NKS = HDP / 32;    // K32 steps
    constexpr int KS = HDP + 8;      // K LDS row stride (elements)
    constexpr int VS = 80;           // V LDS row stride (elements): conflict-free tr reads
    constexpr int NCHL = HD / 8;     // 16-B chunks loaded per K / V row
    constexpr int NDT = (HD + 15) / 16;  // output d-tiles of 16
    constexpr int QW = 32;           // query rows per wave (2 MFMA column tiles)
    __shared__ __attribute__((aligned(16))) bf16 Ks[2][64 * KS];
    __shared__ __attribute__((aligned(16))) bf16 Vs[2][64 * VS];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int g = lane >> 4, li = lane & 15;
    // 1-D grid, XCD-aware: blocks b and b+8 share an XCD (round-robin dispatch), so
    // remap ids so each XCD runs a contiguous range of (batch, head, q-block)
    // tuples -> the q-blocks of one head re-read its K/V from the same L2.
    const int nqb = (a.T + 4 * QW - 1) / (4 * QW);
    int id;
    {
        const int bid = blockIdx.x, nwg = gridDim.x;
        const int xcd = bid & 7, loc = bid >> 3, q8 = nwg >> 3, r8 = nwg & 7;
        id = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
    }
    const int qb = id % nqb, h = (id / nqb) % a.H, b = id / (nqb * a.H);
    const int T = a.T, D = a.H * HD;
    const bf16* base = a.qkv + (long)b * T * a.ld;
    const int qw0 = qb * (4 * QW) + wave * QW;  // first query row of this wave
    const int Tk = a.seq_lens ? a.seq_lens[b] : T;
    const float c = a.scale_log2;

    // zero the padding columns (K: HD..HDP, V: HD..VS) of both buffers once;
    // the tile loads below never write them
    for (int i = tid; i < 2 * 64; i += 256) {
        bf16* kr = &Ks[i >> 6][(i & 63) * KS];
        for (int col = HD; col < HDP; col += 8) *reinterpret_cast<u16x8*>(kr + col) = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
        bf16* vr = &Vs[i >> 6][(i & 63) * VS];
        for (int col = HD; col < VS; col += 8) *reinterpret_cast<u16x8*>(vr + col) = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }

    // Q^T fragments (B operand) for the wave's two 16-row query tiles; columns >= HD are zero
    bf16x8 qf[2][NKS];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const bf16* qrow = base + (long)min(qw0 + u * 16 + li, T - 1) * a.ld + h * HD;
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
            const int col = ks * 32 + 8 * g;
            if (col < HD)
                qf[u][ks] = *reinterpret_cast<const bf16x8*>(qrow + col);
            else
                qf[u][ks] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
        }
    }

    int nkt = (Tk + 63) / 64;
    if (a.causal) nkt = min(nkt, (min(T, qb * 4 * QW + 4 * QW) + 63) / 64);

    // K/V tile staging through registers; rows beyond T are clamped (finite
    // values whose scores are masked / weights are 0). K and V chunks are
    // distributed by separate loops so no lane branches on the tensor.
    constexpr int NCH = 64 * NCHL;              // chunks per K (or V) tile
    constexpr int CPT1 = (NCH + 255) / 256;
    u16x8 pk[CPT1], pv[CPT1];
    auto load_tile = [&](int t) {
        if (DIAG == 1 && t > 0) return;
#pragma unroll
        for (int i = 0; i < CPT1; ++i) {
            const int cidx = tid + i * 256;
            if (NCH % 256 == 0 || cidx < NCH) {
                const int row = cidx / NCHL, ch = cidx % NCHL;
                const bf16* r = base + (long)min(t * 64 + row, T - 1) * a.ld + h * HD + ch * 8;
                pk[i] = *reinterpret_cast<const u16x8*>(r + D);
                pv[i] = *reinterpret_cast<const u16x8*>(r + 2 * D);
            }
        }
    };
    auto store_tile = [&](int buf) {
#pragma unroll
        for (int i = 0; i < CPT1; ++i) {
            const int cidx = tid + i * 256;
            if (NCH % 256 == 0 || cidx < NCH) {
                const int row = cidx / NCHL, ch = cidx % NCHL;
                *reinterpret_cast<u16x8*>(&Ks[buf][row * KS + ch * 8]) = pk[i];
                *reinterpret_cast<u16x8*>(&Vs[buf][row * VS + ch * 8]) = pv[i];
            }
        }
    };

    f32x4 o[2][NDT];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int i = 0; i < NDT; ++i) o[u][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    float m[2] = {-1e30f, -1e30f}, lsum[2] = {0.f, 0.f};  // running max in raw-score units

    load_tile(0);
    __syncthreads();  // padding zeroes visible before the first tile overwrites its rows
    store_tile(0);
    __syncthreads();
    for (int t = 0; t < nkt; ++t) {
        const int buf = t & 1;
        if (t + 1 < nkt) load_tile(t + 1);
        const bf16* Kb = Ks[buf];
        const bf16* Vb = Vs[buf];

        // S^T[key][q] for 4 sub-tiles of 16 keys x 2 query tiles; K fragments shared
        f32x4 sc[2][4];
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) {
            const bf16* krow = Kb + (kt * 16 + li) * KS;
            bf16x8 kf[NKS];
#pragma unroll
            for (int ks = 0; ks < NKS; ++ks) kf[ks] = *reinterpret_cast<const bf16x8*>(krow + ks * 32 + 8 * g);
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                f32x4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int ks = 0; ks < NKS; ++ks) {
                    if (DIAG == 4)
                        asm volatile("" : "+v"(z) : "v"(kf[ks]), "v"(qf[u][ks]));
                    else
                        z = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[ks], qf[u][ks], z, 0, 0, 0);
                }
                sc[u][kt] = z;
            }
        }

        // masking only where the tile crosses the key length or the causal diagonal
        if ((t * 64 + 64 > Tk) || (a.causal && t * 64 + 63 > qw0)) {
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int q = qw0 + u * 16 + li;
                const int lim = a.causal ? min(Tk, q + 1) : Tk;  // valid keys: key < lim
#pragma unroll
                for (int kt = 0; kt < 4; ++kt)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        if (t * 64 + kt * 16 + 4 * g + r >= lim) sc[u][kt][r] = -INFINITY;
            }
        }

        // online softmax (log2 domain, scale folded into one FMA per score)
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            float mloc = fmaxf(fmaxf(sc[u][0][0], sc[u][0][1]), fmaxf(sc[u][0][2], sc[u][0][3]));
#pragma unroll
            for (int kt = 1; kt < 4; ++kt)
                mloc = fmaxf(mloc, fmaxf(fmaxf(sc[u][kt][0], sc[u][kt][1]), fmaxf(sc[u][kt][2], sc[u][kt][3])));
            mloc = fmaxf(mloc, __shfl_xor(mloc, 16, 64));
            mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
            const float mnew = fmaxf(m[u], mloc);
            if (THR) {
                if (__builtin_amdgcn_ballot_w64((mloc - m[u]) * c > 8.0f)) {
                    const float alpha = __builtin_amdgcn_exp2f((m[u] - mnew) * c);
                    m[u] = mnew;
                    lsum[u] *= alpha;
#pragma unroll
                    for (int i = 0; i < NDT; ++i) o[u][i] *= alpha;
                }
                const float mc = m[u] * c;
                float psum = 0.f;
#pragma unroll
                for (int kt = 0; kt < 4; ++kt)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float pv = __builtin_amdgcn_exp2f(__builtin_fmaf(sc[u][kt][r], c, -mc));
                        sc[u][kt][r] = pv;
                        psum += pv;
                    }
                lsum[u] += psum;
                continue;
            }
            const float alpha = __builtin_amdgcn_exp2f((m[u] - mnew) * c);
            m[u] = mnew;
            const float mc = mnew * c;
            float psum = 0.f;
#pragma unroll
            for (int kt = 0; kt < 4; ++kt)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float pv = DIAG == 2 ? __builtin_fmaf(sc[u][kt][r], c, -mc) : __builtin_amdgcn_exp2f(__builtin_fmaf(sc[u][kt][r], c, -mc));
                    sc[u][kt][r] = pv;
                    psum += pv;
                }
            lsum[u] = lsum[u] * alpha + psum;
#pragma unroll
            for (int i = 0; i < NDT; ++i) o[u][i] *= alpha;
        }

        // O^T[d][q] += V^T[d][key] . P^T[key][q]; V^T fragments shared by both query tiles
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
            bf16x8 pb[2];
#pragma unroll
            for (int u = 0; u < 2; ++u)
                pb[u] = __builtin_convertvector(__builtin_shufflevector(sc[u][2 * hh], sc[u][2 * hh + 1], 0, 1, 2, 3,
                                                                        4, 5, 6, 7), bf16x8);
            const int r1 = 32 * hh + 4 * g + (li >> 2);
#pragma unroll
            for (int dt = 0; dt < NDT; ++dt) {
                const int col = dt * 16 + 4 * (li & 3);
                const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(Vb + r1 * VS + col));
                const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(Vb + (r1 + 16) * VS + col));
                const bf16x8 vv = __builtin_bit_cast(bf16x8, __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    if (DIAG == 3)
                        asm volatile("" : "+v"(o[u][dt]) : "v"(vv), "v"(pb[u]));
                    else
                        o[u][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vv, pb[u], o[u][dt], 0, 0, 0);
                }
            }
        }

        if (t + 1 < nkt) store_tile(buf ^ 1);
        __syncthreads();
    }

#pragma unroll
    for (int u = 0; u < 2; ++u) {
        float ltot = lsum[u] + __shfl_xor(lsum[u], 16, 64);
        ltot += __shfl_xor(ltot, 32, 64);
        const float inv = 1.0f / ltot;
        const int q = qw0 + u * 16 + li;
        if (q < T) {
            bf16* orow = a.out + ((long)b * T + q) * a.ldo + h * HD;
#pragma unroll
            for (int dt = 0; dt < NDT; ++dt) {
                const int d0 = dt * 16 + 4 * g;
                if (d0 < HD) {
                    bf16x4 v;
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[r] = f2bf(o[u][dt][r] * inv);
                    *reinterpret_cast<bf16x4*>(orow + d0) = v;
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------
// attn_dma_kernel: the same per-wave math as attn_fwd_kernel (32 query rows
// per wave, S^T = K.Q^T, P in registers, V^T by transposed LDS reads), with
// the K/V tiles staged by LDS-DMA instead of through registers:
//   * "chunk-plane" tile layout: plane c (16-B column chunk c of all 64 keys)
//     is one 1 KiB DMA instruction, lane = key -> no register staging, no
//     ds_write, and conflict-free ds_read_b128 for the K fragments (the 16
//     lanes of a read group have distinct keys);
//   * V planes with odd c store key ^ 8 (swizzled through the per-lane DMA
//     source row) so the 32 lanes of a ds_read_b64_tr_b16 group hit 64
//     distinct banks;
//   * head-dim padding is never stored: fragment lanes past HD read plane 0
//     (finite data meeting zero Q columns / producing discarded O rows);
//   * NSTG-deep ring of tiles, tile t+NSTG-1 issued after the barrier that
//     opens tile t (WAR: every wave finished tile t-1 before that barrier;
//     RAW: each wave retires its own DMA of tile t by a counted vmcnt before it).
// ---------------------------------------------------------------------------
template <int HD, int NW, int NSTG, int DIAG = 0, int MINW = 1>
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(MINW))) void attn_dma_kernel(AttnArgs a) {
    // DIAG (dev builds, wrong results; tools/attn_bench.py): 1 no K/V DMA, 2 no exp2,
    // 3 no PV MFMA, 4 no QK MFMA, 5 no O rescale, 6 no LDS fragment reads
    constexpr int HDP = HD == 64 ? 64 : 96;
    constexpr int NKS = HDP / 32;
    constexpr int NCHL = HD / 8;             // real 16-B planes per K (or V) tile
    constexpr int NDT = (HD + 15) / 16;
    constexpr int QW = 32, QB = NW * QW;     // query rows per wave / per block
    constexpr int TILE = 2 * NCHL * 1024;    // bytes per K+V tile
    constexpr int NINS = 2 * NCHL;           // DMA instructions per tile
    constexpr int MAXI = (NINS + NW - 1) / NW;
    __shared__ __attribute__((aligned(16))) char lds[NSTG * TILE];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = lane >> 4, li = lane & 15;
    const int nqb = (a.T + QB - 1) / QB;
    int id;
    {
        const int bid = blockIdx.x, nwg = gridDim.x;
        const int xcd = bid & 7, loc = bid >> 3, q8 = nwg >> 3, r8 = nwg & 7;
        id = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
    }
    const int qb = id % nqb, h = (id / nqb) % a.H, b = id / (nqb * a.H);
    const int T = a.T, D = a.H * HD;
    const bf16* base = a.qkv + (long)b * T * a.ld;
    const int qw0 = qb * QB + wave * QW;
    const int Tk = a.seq_lens ? a.seq_lens[b] : T;
    const float c = a.scale_log2;

    bf16x8 qf[2][NKS];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const bf16* qrow = base + (long)min(qw0 + u * 16 + li, T - 1) * a.ld + h * HD;
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
            const int col = ks * 32 + 8 * g;
            if (col < HD)
                qf[u][ks] = *reinterpret_cast<const bf16x8*>(qrow + col);
            else
                qf[u][ks] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
        }
    }

    int nkt = (Tk + 63) / 64;
    if (a.causal) nkt = min(nkt, (min(T, qb * QB + QB) + 63) / 64);

    // this wave's DMA instructions: idx = wave + NW*i (K planes 0..NCHL-1, V planes after)
    const int nmine = (NINS - wave + NW - 1) / NW;
    auto issue = [&](int t) {
        char* tb = lds + (t % NSTG) * TILE;
        if (DIAG == 1) return;
#pragma unroll
        for (int i = 0; i < MAXI; ++i) {
            const int idx = wave + NW * i;
            if (i < MAXI - 1 || idx < NINS) {
                const bool isV = idx >= NCHL;
                const int plane = isV ? idx - NCHL : idx;
                const int key = isV && (plane & 1) ? lane ^ 8 : lane;
                const bf16* src = base + (long)min(t * 64 + key, T - 1) * a.ld + (isV ? 2 : 1) * D + h * HD + plane * 8;
                glds16(src, tb + idx * 1024);
            }
        }
    };
    auto wait_own = [&](int later) {  // retire own DMA except `later` (0/1) tiles after it
        if (later == 0) {
            vm_wait<0>();
        } else if (nmine == MAXI) {
            vm_wait<MAXI>();
        } else {
            vm_wait<MAXI - 1>();
        }
    };

    // fragment addresses inside a tile
    const unsigned lds0 = (unsigned)(uintptr_t)(LDS_AS char*)lds;
    unsigned koff[NKS];
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
        const int cch = ks * 4 + g;
        koff[ks] = (cch < NCHL ? cch : 0) * 1024 + li * 16;
    }
    unsigned voff[NDT];  // + key*16 added per read (key parity handled by the plane's swizzle)
    int vsw[NDT];
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
        int plane = 2 * dt + ((li >> 1) & 1);
        if (plane >= NCHL) plane = 0;
        voff[dt] = (NCHL + plane) * 1024 + (li & 1) * 8;
        vsw[dt] = (plane & 1) ? 8 : 0;
    }

    f32x4 o[2][NDT];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int i = 0; i < NDT; ++i) o[u][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    float m[2] = {-1e30f, -1e30f}, lsum[2] = {0.f, 0.f};

    static_assert(NSTG == 2 || NSTG == 3, "ring depth");
    for (int t = 0; t < NSTG - 1 && t < nkt; ++t) issue(t);
    for (int t = 0; t < nkt; ++t) {
        wait_own(NSTG == 3 && t + 1 < nkt ? 1 : 0);
        __builtin_amdgcn_s_barrier();
        if (t + NSTG - 1 < nkt) issue(t + NSTG - 1);
        const unsigned tb = lds0 + (t % NSTG) * TILE;

        f32x4 sc[2][4];
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) {
            bf16x8 kf[NKS];
#pragma unroll
            for (int ks = 0; ks < NKS; ++ks) {
                if (DIAG == 6) {
                    kf[ks] = qf[0][ks];
                    asm volatile("" : "+v"(kf[ks]));
                } else {
                    kf[ks] = *reinterpret_cast<const LDS_AS bf16x8*>((uintptr_t)(tb + koff[ks] + kt * 256));
                }
            }
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                f32x4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int ks = 0; ks < NKS; ++ks) {
                    if (DIAG == 4)
                        asm volatile("" : "+v"(z) : "v"(kf[ks]), "v"(qf[u][ks]));
                    else
                        z = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[ks], qf[u][ks], z, 0, 0, 0);
                }
                sc[u][kt] = z;
            }
        }

        if ((t * 64 + 64 > Tk) || (a.causal && t * 64 + 63 > qw0)) {
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int q = qw0 + u * 16 + li;
                const int lim = a.causal ? min(Tk, q + 1) : Tk;
#pragma unroll
                for (int kt = 0; kt < 4; ++kt)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        if (t * 64 + kt * 16 + 4 * g + r >= lim) sc[u][kt][r] = -INFINITY;
            }
        }

#pragma unroll
        for (int u = 0; u < 2; ++u) {
            float mloc = fmaxf(fmaxf(sc[u][0][0], sc[u][0][1]), fmaxf(sc[u][0][2], sc[u][0][3]));
#pragma unroll
            for (int kt = 1; kt < 4; ++kt)
                mloc = fmaxf(mloc, fmaxf(fmaxf(sc[u][kt][0], sc[u][kt][1]), fmaxf(sc[u][kt][2], sc[u][kt][3])));
            mloc = fmaxf(mloc, __shfl_xor(mloc, 16, 64));
            mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
            const float mnew = fmaxf(m[u], mloc);
            const float alpha = __builtin_amdgcn_exp2f((m[u] - mnew) * c);
            m[u] = mnew;
            const float mc = mnew * c;
            float psum = 0.f;
#pragma unroll
            for (int kt = 0; kt < 4; ++kt)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float pv = DIAG == 2 ? __builtin_fmaf(sc[u][kt][r], c, -mc)
                                               : __builtin_amdgcn_exp2f(__builtin_fmaf(sc[u][kt][r], c, -mc));
                    sc[u][kt][r] = pv;
                    psum += pv;
                }
            lsum[u] = lsum[u] * alpha + psum;
            if (DIAG != 5) {
#pragma unroll
                for (int i = 0; i < NDT; ++i) o[u][i] *= alpha;
            }
        }

#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
            bf16x8 pb[2];
#pragma unroll
            for (int u = 0; u < 2; ++u)
                pb[u] = __builtin_convertvector(__builtin_shufflevector(sc[u][2 * hh], sc[u][2 * hh + 1], 0, 1, 2, 3,
                                                                        4, 5, 6, 7), bf16x8);
            const int r1 = 32 * hh + 4 * g + (li >> 2);
#pragma unroll
            for (int dt = 0; dt < NDT; ++dt) {
                bf16x8 vv;
                if (DIAG == 6) {
                    vv = pb[0];
                    asm volatile("" : "+v"(vv));
                } else {
                    const unsigned va = tb + voff[dt] + ((r1 ^ vsw[dt]) * 16);
                    const unsigned vb2 = tb + voff[dt] + (((r1 + 16) ^ vsw[dt]) * 16);
                    const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(uintptr_t)va);
                    const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(uintptr_t)vb2);
                    vv = __builtin_bit_cast(bf16x8, __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7));
                }
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    if (DIAG == 3)
                        asm volatile("" : "+v"(o[u][dt]) : "v"(vv), "v"(pb[u]));
                    else
                        o[u][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vv, pb[u], o[u][dt], 0, 0, 0);
                }
            }
        }
    }

#pragma unroll
    for (int u = 0; u < 2; ++u) {
        float ltot = lsum[u] + __shfl_xor(lsum[u], 16, 64);
        ltot += __shfl_xor(ltot, 32, 64);
        const float inv = 1.0f / ltot;
        const int q = qw0 + u * 16 + li;
        if (q < T) {
            bf16* orow = a.out + ((long)b * T + q) * a.ldo + h * HD;
#pragma unroll
            for (int dt = 0; dt < NDT; ++dt) {
                const int d0 = dt * 16 + 4 * g;
                if (d0 < HD) {
                    bf16x4 v;
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[r] = f2bf(o[u][dt][r] * inv);
                    *reinterpret_cast<bf16x4*>(orow + d0) = v;
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------
// attn_pipe_kernel: attn_dma_kernel's per-wave math, software-pipelined across
// key tiles. attn_dma_kernel runs QK^T(t) -> softmax(t) -> PV(t) as one dependent
// chain per tile, so with two waves per SIMD the MFMA pipe idles whenever both
// sit in their softmax (tools/attn_bench.py ablations: latency-bound, no single
// part > 14 %). Here iteration t computes S(t+1) = K(t+1).Q^T right after the
// barrier and only then the softmax and PV of tile t, so tile t's VALU work has
// independent MFMAs beside it. Needs K(t+1) resident one iteration earlier ->
// 3-deep tile ring (tile t+2 in flight). Also:
//   * row max / row sum cross-lane steps with v_permlane16/32_swap (VALU) instead
//     of ds_bpermute round trips through the LDS;
//   * per-lane fragment addresses computed once; per tile only the ring slot
//     offset is added (the swizzled V row r ^ 8 commutes with +16 / +32 rows).
// Ordering: tile t+2 overwrites the slot of tile t-1, whose last reads (PV(t-1))
// every wave finished before the barrier of iteration t; K(t+1) is read after
// that barrier, which follows every wave's own vmcnt wait for tile t+1.
// ---------------------------------------------------------------------------
__device__ __forceinline__ float xmax16(float v) {  // max over lanes l, l^16
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xmax32(float v) {  // max over lanes l, l^32
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xsum16(float v) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float xsum32(float v) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// XF (dev extras, bit mask): 1 = K/V DMA from inline asm (ADMA), 2 = exp arguments as packed
// FMAs (v_pk_fma_f32, half the issues; same per-element fma, bit-identical), 4 = s_setprio 1
// for the second half of the waves before the tile loop (static priority)
template <int HD, int NW, int NSTG, bool PIPE, bool ONES, bool LAZY, bool PING = false, int MINW = 1, bool UNR = false,
          int XF = 0>
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(MINW))) void attn_pipe_kernel(AttnArgs a) {
    constexpr bool ADMA = XF & 1, PKX = XF & 2, PRIO = XF & 4, NODMA = XF & 8;  // 8: diagnostic, no K/V DMA (wrong results)
    constexpr bool WIDE = XF & 16;  // 16: O stored as 16-B rows (v_permlane16_swap pairs of d-tiles)
    constexpr bool PAIR = XF & 32;  // 32: 4-tile ring, one barrier per PAIR of key tiles (UNR, NSTG 4)
    static_assert(!PAIR || (UNR && NSTG == 4 && !PIPE && !PING), "paired tiles: unrolled 4-slot ring");
    static_assert(!PIPE || NSTG == 3, "the pipelined loop keeps tile t+1 resident while t+2 lands");
    static_assert(!PING || (!PIPE && NSTG == 4), "ping-pong: two tiles resident beside the one landing");
    static_assert(!ONES || HD == 72, "the ones column lives in the padding of the 80-wide V^T tiles");
    constexpr int HDP = HD == 64 ? 64 : 96;
    constexpr int NKS = HDP / 32;
    constexpr int NCHL = HD / 8;
    constexpr int NDT = (HD + 15) / 16;
    constexpr int QW = 32, QB = NW * QW;
    constexpr int TILE = (2 * NCHL + (ONES ? 1 : 0)) * 1024;  // K planes, V planes (+ a plane of ones)
    constexpr int NINS = 2 * NCHL;
    constexpr int MAXI = (NINS + NW - 1) / NW;
    __shared__ __attribute__((aligned(16))) char lds[NSTG * TILE];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = lane >> 4, li = lane & 15;
    const int nqb = (a.T + QB - 1) / QB;
    int id;
    {
        const int bid = blockIdx.x, nwg = gridDim.x;
        const int xcd = bid & 7, loc = bid >> 3, q8 = nwg >> 3, r8 = nwg & 7;
        id = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
    }
    const int qb = id % nqb, h = (id / nqb) % a.H, b = id / (nqb * a.H);
    const int T = a.T, D = a.H * HD;
    const bf16* base = a.qkv + (long)b * T * a.ld;
    const int qw0 = qb * QB + wave * QW;
    const int Tk = a.seq_lens ? a.seq_lens[b] : T;
    const float c = a.scale_log2;

    if (ONES) {  // V^T column HD (inside the 80-wide padding) = 1: the PV MFMAs then also sum the weights
        for (int i = tid; i < NSTG * 64; i += NW * 64)
            *reinterpret_cast<u16x8*>(lds + (i >> 6) * TILE + 2 * NCHL * 1024 + (i & 63) * 16) =
                u16x8{0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80};
    }

    bf16x8 qf[2][NKS];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const bf16* qrow = base + (long)min(qw0 + u * 16 + li, T - 1) * a.ld + h * HD;
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
            const int col = ks * 32 + 8 * g;
            if (col < HD)
                qf[u][ks] = *reinterpret_cast<const bf16x8*>(qrow + col);
            else
                qf[u][ks] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
        }
    }

    int nkt = (Tk + 63) / 64;
    if (a.causal) nkt = min(nkt, (min(T, qb * QB + QB) + 63) / 64);
    if (ADMA) {  // Q landed before the tile loop: hipcc then never waits inside it (it cannot count the asm DMA)
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int ks = 0; ks < NKS; ++ks) asm volatile("" ::"v"(qf[u][ks]));
    }

    const int nmine = (NINS - wave + NW - 1) / NW;
    auto issue = [&](int t) {
        if (NODMA && t > 0) return;
        char* tb = lds + (t % NSTG) * TILE;
#pragma unroll
        for (int i = 0; i < MAXI; ++i) {
            const int idx = wave + NW * i;
            if (i < MAXI - 1 || idx < NINS) {
                const bool isV = idx >= NCHL;
                const int plane = isV ? idx - NCHL : idx;
                const int key = isV && (plane & 1) ? lane ^ 8 : lane;
                const bf16* src = base + (long)min(t * 64 + key, T - 1) * a.ld + (isV ? 2 : 1) * D + h * HD + plane * 8;
                if (ADMA)
                    glds16_asm(src, tb + idx * 1024);
                else
                    glds16(src, tb + idx * 1024);
            }
        }
    };
    auto wait_own = [&](int later) {  // retire own DMA except `later` (0/1) tiles after it
        if (later == 0) {
            vm_wait<0>();
        } else if (nmine == MAXI) {
            vm_wait<MAXI>();
        } else {
            vm_wait<MAXI - 1>();
        }
    };

    const unsigned lds0 = (unsigned)(uintptr_t)(LDS_AS char*)lds;
    // K fragment of step ks = plane 4 ks + g; lanes past HD read planes beyond the K planes
    // (V planes of the same tile: finite, landed with it) against zero Q columns, so every
    // step is the lane base + an immediate (no per-step address registers).
    const unsigned kb0 = lds0 + g * 1024 + li * 16;
    // V^T fragment of d-tile dt = plane 2 dt + ((li >> 1) & 1): the lane base + dt * 2 KiB,
    // except at head dim 72 without the ones plane, where plane 9 does not exist (clamped)
    constexpr bool VLIN = !(HD == 72 && !ONES);
    unsigned vb[NDT];
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
        int plane = 2 * dt + ((li >> 1) & 1);
        if (plane >= NCHL) plane = ONES ? NCHL : 0;  // ONES: plane 2*NCHL of the tile (all ones)
        const int vsw = (plane & 1) ? 8 : 0;
        vb[dt] = lds0 + (NCHL + plane) * 1024 + (li & 1) * 8 + (((4 * g + (li >> 2)) ^ vsw) * 16);
    }

    f32x4 o[2][NDT];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int i = 0; i < NDT; ++i) o[u][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    float m[2] = {-1e30f, -1e30f}, lsum[2] = {0.f, 0.f};

    auto qk_at = [&](int t, const unsigned so, f32x4(&sc)[2][4]) {
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) {
            bf16x8 kf[NKS];
#pragma unroll
            for (int ks = 0; ks < NKS; ++ks)
                kf[ks] = *reinterpret_cast<const LDS_AS bf16x8*>((uintptr_t)(kb0 + so + kt * 256 + ks * 4096));
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                f32x4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int ks = 0; ks < NKS; ++ks) z = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[ks], qf[u][ks], z, 0, 0, 0);
                sc[u][kt] = z;
            }
        }
        if ((t * 64 + 64 > Tk) || (a.causal && t * 64 + 63 > qw0)) {
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int q = qw0 + u * 16 + li;
                const int lim = a.causal ? min(Tk, q + 1) : Tk;
#pragma unroll
                for (int kt = 0; kt < 4; ++kt)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        if (t * 64 + kt * 16 + 4 * g + r >= lim) sc[u][kt][r] = -INFINITY;
            }
        }
    };
    auto qk = [&](int t, f32x4(&sc)[2][4]) { qk_at(t, (t % NSTG) * TILE, sc); };
    auto softmax_pv_at = [&](int t, const unsigned so, f32x4(&sc)[2][4], auto&& before_pv) {
        float mnew[2];
        bool grew = false;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            float mloc = fmaxf(fmaxf(sc[u][0][0], sc[u][0][1]), fmaxf(sc[u][0][2], sc[u][0][3]));
#pragma unroll
            for (int kt = 1; kt < 4; ++kt)
                mloc = fmaxf(mloc, fmaxf(fmaxf(sc[u][kt][0], sc[u][kt][1]), fmaxf(sc[u][kt][2], sc[u][kt][3])));
            mloc = xmax32(xmax16(mloc));
            mnew[u] = fmaxf(m[u], mloc);
            grew |= mnew[u] != m[u];
        }
        // LAZY: alpha == 1 exactly when no row max of the wave grew -> skip the rescale
        if (!LAZY || __builtin_amdgcn_ballot_w64(grew)) {
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const float alpha = __builtin_amdgcn_exp2f((m[u] - mnew[u]) * c);
                if (!ONES) lsum[u] *= alpha;
#pragma unroll
                for (int i = 0; i < NDT; ++i) o[u][i] *= alpha;
            }
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            m[u] = mnew[u];
            const float mc = mnew[u] * c;
            float psum = 0.f;
            if (PKX) {
#pragma unroll
                for (int kt = 0; kt < 4; ++kt)
#pragma unroll
                    for (int r = 0; r < 4; r += 2) {
                        const f32x2 x = pk_fma(f32x2{sc[u][kt][r], sc[u][kt][r + 1]}, f32x2{c, c}, f32x2{-mc, -mc});
                        sc[u][kt][r] = __builtin_amdgcn_exp2f(x.x);
                        sc[u][kt][r + 1] = __builtin_amdgcn_exp2f(x.y);
                        if (!ONES) {
                            psum += sc[u][kt][r];
                            psum += sc[u][kt][r + 1];
                        }
                    }
            } else {
#pragma unroll
                for (int kt = 0; kt < 4; ++kt)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float pv = __builtin_amdgcn_exp2f(__builtin_fmaf(sc[u][kt][r], c, -mc));
                        sc[u][kt][r] = pv;
                        if (!ONES) psum += pv;
                    }
            }
            if (!ONES) lsum[u] += psum;
        }
        before_pv();
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
            bf16x8 pb[2];
#pragma unroll
            for (int u = 0; u < 2; ++u)
                pb[u] = __builtin_convertvector(__builtin_shufflevector(sc[u][2 * hh], sc[u][2 * hh + 1], 0, 1, 2, 3,
                                                                        4, 5, 6, 7), bf16x8);
#pragma unroll
            for (int dt = 0; dt < NDT; ++dt) {
                const unsigned va = (VLIN ? vb[0] + dt * 2048 : vb[dt]) + so + hh * 512;
                const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(uintptr_t)va);
                const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(uintptr_t)(va + 256));
                const bf16x8 vv = __builtin_bit_cast(bf16x8, __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
                for (int u = 0; u < 2; ++u)
                    o[u][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vv, pb[u], o[u][dt], 0, 0, 0);
            }
        }
    };

    auto softmax_pv = [&](int t, f32x4(&sc)[2][4], auto&& before_pv) {
        softmax_pv_at(t, (t % NSTG) * TILE, sc, before_pv);
    };

    f32x4 sA[2][4], sB[2][4];
    if (PRIO && wave >= NW / 2) __builtin_amdgcn_s_setprio(1);
    if (PAIR) {
        // two key tiles per barrier: tiles t, t+1 landed -> barrier -> issue t+2, t+3 into the
        // slots of t-2, t-1 (read before this barrier) -> QK / softmax / PV of t, then t+1;
        // waves drift within a pair instead of meeting at every tile, and each tile has two
        // tiles of compute to land. Unrolled by the ring (slot offsets are immediates).
        if (nkt > 0) issue(0);
        if (nkt > 1) issue(1);
        for (int t = 0; t < nkt; t += 4) {
            vm_wait<0>();
            __builtin_amdgcn_s_barrier();
            if (t + 2 < nkt) issue(t + 2);
            if (t + 3 < nkt) issue(t + 3);
            qk_at(t, 0, sA);
            softmax_pv_at(t, 0, sA, [] {});
            if (t + 1 < nkt) {
                qk_at(t + 1, TILE, sA);
                softmax_pv_at(t + 1, TILE, sA, [] {});
            }
            if (t + 2 < nkt) {
                vm_wait<0>();
                __builtin_amdgcn_s_barrier();
                if (t + 4 < nkt) issue(t + 4);
                if (t + 5 < nkt) issue(t + 5);
                qk_at(t + 2, 2 * TILE, sA);
                softmax_pv_at(t + 2, 2 * TILE, sA, [] {});
                if (t + 3 < nkt) {
                    qk_at(t + 3, 3 * TILE, sA);
                    softmax_pv_at(t + 3, 3 * TILE, sA, [] {});
                }
            }
        }
    } else if (UNR && !PIPE && !PING && NSTG == 2) {
        // unrolled by the ring depth: the ring slot of every LDS access is a compile-time
        // constant (immediate ds_read offsets, no per-tile address VALU)
        if (nkt > 0) issue(0);
        for (int t = 0; t < nkt; t += 2) {
            vm_wait<0>();
            __builtin_amdgcn_s_barrier();
            if (t + 1 < nkt) issue(t + 1);
            qk_at(t, 0, sA);
            softmax_pv_at(t, 0, sA, [] {});
            if (t + 1 < nkt) {
                vm_wait<0>();
                __builtin_amdgcn_s_barrier();
                if (t + 2 < nkt) issue(t + 2);
                qk_at(t + 1, TILE, sA);
                softmax_pv_at(t + 1, TILE, sA, [] {});
            }
        }
    } else if (PIPE) {
        // iteration t: [tile t+1 landed, barrier, issue t+2, S(t+1)] then softmax + PV of tile t
        auto iter = [&](int t, f32x4(&cur)[2][4], f32x4(&nxt)[2][4]) {
            if (t + 1 < nkt) {
                wait_own(0);
                __builtin_amdgcn_s_barrier();
                if (t + 2 < nkt) issue(t + 2);
                qk(t + 1, nxt);
            }
            softmax_pv(t, cur, [] {});
        };
        issue(0);
        if (nkt > 1) issue(1);
        wait_own(nkt > 1 ? 1 : 0);
        __builtin_amdgcn_s_barrier();
        qk(0, sA);
        for (int t = 0; t < nkt; t += 2) {
            iter(t, sA, sB);
            if (t + 1 < nkt) iter(t + 1, sB, sA);
        }
    } else if (PING) {
        // Ping-pong (two barriers per tile: S(t) before QK, H(t) before PV): waves NW/2.. run
        // one barrier behind, so on every SIMD one wave's exp / max VALU meets the other's PV
        // or QK MFMAs instead of both waves hitting the softmax together. Tile t+2 goes into
        // the slot of tile t-2, whose last reads (the late half's PV(t-2)) end two barriers
        // earlier. Every wave's own pieces of tile t+1 land before the barrier after which the
        // early half reads it: early waves wait at S(t+1), late waves before their H(t).
        const bool late = wave >= NW / 2;
        issue(0);
        if (nkt > 1) issue(1);
        if (late) {
            wait_own(nkt > 1 ? 1 : 0);
            __builtin_amdgcn_s_barrier();
        }
        for (int t = 0; t < nkt; ++t) {
            if (!late) wait_own(t + 1 < nkt ? 1 : 0);
            __builtin_amdgcn_s_barrier();
            if (t + 2 < nkt) issue(t + 2);
            qk(t, sA);
            softmax_pv(t, sA, [&] {
                if (late) wait_own(t + 2 < nkt ? 1 : 0);
                __builtin_amdgcn_s_barrier();
            });
        }
        if (!late) __builtin_amdgcn_s_barrier();
    } else {
        for (int t = 0; t < NSTG - 1 && t < nkt; ++t) issue(t);
        for (int t = 0; t < nkt; ++t) {
            wait_own(NSTG == 3 && t + 1 < nkt ? 1 : 0);
            __builtin_amdgcn_s_barrier();
            if (t + NSTG - 1 < nkt) issue(t + NSTG - 1);
            qk(t, sA);
            softmax_pv(t, sA, [] {});
        }
    }

#pragma unroll
    for (int u = 0; u < 2; ++u) {
        float ltot;
        if (ONES)  // the weight sums sit in O^T row HD = 64 + 4*2 + 0: lanes 32..47, element 0
            ltot = __shfl(o[u][NDT - 1][0], 32 + li, 64);
        else
            ltot = xsum32(xsum16(lsum[u]));
        const float inv = 1.0f / ltot;
        const int q = qw0 + u * 16 + li;
        if (WIDE) {
            // d-tile pairs (dt, dt + 1): after v_permlane16_swap of the packed halves, the lanes
            // of lane-row g hold 8 consecutive columns 16 (dt + (g & 1)) + 8 (g >> 1) .. + 7
            // (same values and addresses as the 8-B stores, half the store instructions)
            bf16* orow = a.out + ((long)b * T + min(q, T - 1)) * a.ldo + h * HD;
#pragma unroll
            for (int dt = 0; dt + 1 < NDT && (dt + 2) * 16 <= HD; dt += 2) {
                bf16x4 v0, v1;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    v0[r] = f2bf(o[u][dt][r] * inv);
                    v1[r] = f2bf(o[u][dt + 1][r] * inv);
                }
                uint2 x = __builtin_bit_cast(uint2, v0), y = __builtin_bit_cast(uint2, v1);
                const auto sx = __builtin_amdgcn_permlane16_swap(x.x, y.x, false, false);
                const auto sy = __builtin_amdgcn_permlane16_swap(x.y, y.y, false, false);
                if (q < T)
                    *reinterpret_cast<uint4*>(orow + 16 * (dt + (g & 1)) + 8 * (g >> 1)) =
                        make_uint4(sx[0], sy[0], sx[1], sy[1]);
            }
            constexpr int DT0 = (HD / 32) * 2;  // first d-tile not covered by a whole pair
#pragma unroll
            for (int dt = DT0; dt < NDT; ++dt) {
                const int d0 = dt * 16 + 4 * g;
                if (q < T && d0 < HD) {
                    bf16x4 v;
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[r] = f2bf(o[u][dt][r] * inv);
                    *reinterpret_cast<bf16x4*>(orow + d0) = v;
                }
            }
        } else if (q < T) {
            bf16* orow = a.out + ((long)b * T + q) * a.ldo + h * HD;
#pragma unroll
            for (int dt = 0; dt < NDT; ++dt) {
                const int d0 = dt * 16 + 4 * g;
                if (d0 < HD) {
                    bf16x4 v;
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[r] = f2bf(o[u][dt][r] * inv);
                    *reinterpret_cast<bf16x4*>(orow + d0) = v;
                }
            }
        }
    }
}

// attn_short_kernel: sequences of at most 64 tokens (SigLIP text, L = 64) — the
// whole key range is ONE 64-key tile, so there is no online softmax and no tile
// ring. attn_fwd_kernel's 128-query blocks computed 64 clamped duplicate query
// rows there (half its MFMA / exp work wasted: ~125 TF/s on the text towers).
// Here a workgroup = 4 waves = TWO (batch, head) units: waves 2s, 2s+1 take the
// 32-query halves of unit s, whose K and V tiles sit in LDS slot s (the two
// buffers attn_fwd_kernel rings through). Same per-wave math (S^T = K.Q^T, P in
// registers as the B operand of O^T = V^T.P^T, V^T by ds_read_b64_tr_b16).
// COMPACT (head dims 72/80): K rows at the V pitch of 80 elements, so one block holds
// 40 KiB of LDS and four blocks share a CU (three at the padded 104-element K pitch).
// The zero-padded 96-deep QK^T reduction then reads past a K row's 80 elements into
// the next row (or, for the last row, into the V tile behind it): finite values
// against zero Q columns; only the K padding columns HD..80 are zeroed.
template <int HD, bool COMPACT = false>
__global__ __launch_bounds__(256, 3) void attn_short_kernel(AttnArgs a, int units) {
    constexpr int HDP = HD == 64 ? 64 : 96;
    constexpr int NKS = HDP / 32;
    constexpr int KS = COMPACT && HD != 64 ? 80 : HDP + 8;  // K LDS row stride (elements)
    constexpr int KZ = COMPACT && HD != 64 ? KS : HDP;      // K columns HD..KZ zeroed
    constexpr int VS = 80;       // V LDS row stride: conflict-free tr reads
    constexpr int NCHL = HD / 8;
    constexpr int NDT = (HD + 15) / 16;
    constexpr int NCH = 64 * NCHL;  // 16-B chunks per K (or V) tile
    static_assert((4 * NCH) % 256 == 0, "K + V tiles of both slots split evenly over 256 threads");
    __shared__ __attribute__((aligned(16))) bf16 sm[2 * 64 * KS + 2 * 64 * VS];  // K slots, then V slots
    bf16 (*Ks)[64 * KS] = reinterpret_cast<bf16 (*)[64 * KS]>(sm);
    bf16 (*Vs)[64 * VS] = reinterpret_cast<bf16 (*)[64 * VS]>(sm + 2 * 64 * KS);

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int g = lane >> 4, li = lane & 15;
    const int T = a.T, D = a.H * HD;
    // XCD-aware: consecutive unit pairs (neighbouring heads of one sequence, whose
    // 2*HD-byte row segments share cache lines) run on the same XCD / L2
    int pair;
    {
        const int bid = blockIdx.x, nwg = gridDim.x;
        const int xcd = bid & 7, loc = bid >> 3, q8 = nwg >> 3, r8 = nwg & 7;
        pair = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
    }

    const int slot = wave >> 1;
    const int unit = pair * 2 + slot;
    const int uc = min(unit, units - 1);
    const int b = uc / a.H, h = uc % a.H;
    const bf16* base = a.qkv + (long)b * T * a.ld;
    const int qw0 = (wave & 1) * 32;
    const int Tk = a.seq_lens ? a.seq_lens[b] : T;
    const float c = a.scale_log2;

    // Q fragments, loaded unconditionally and zeroed past HD by a mask: the padding columns HD..HDP of
    // the reduction read the next head's (or K's) columns of the same row, in bounds since
    // h * HD + HDP <= 3 * H * HD <= ld. Round 6: the per-lane `if (col < HD)` load this replaces made
    // hipcc copy the loaded value inside the branch, i.e. wait for it (s_waitcnt vmcnt(0)) before the
    // first K / V load below was issued -- one HBM round trip in series per block.
    typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
    bf16x8 qf[2][NKS];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const bf16* qrow = base + (long)min(qw0 + u * 16 + li, T - 1) * a.ld + h * HD;
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
            const int col = ks * 32 + 8 * g;
            const unsigned keep = col < HD ? 0xffffffffu : 0u;
            const u32x4_t v = *reinterpret_cast<const u32x4_t*>(qrow + col);
            qf[u][ks] = __builtin_bit_cast(bf16x8, v & u32x4_t{keep, keep, keep, keep});
        }
    }
    // stage K and V of both units (rows past T clamped: finite, masked below): every load issued before the
    // first LDS write, the units' K bases computed once (the per-chunk run-time division by H cost ~40
    // instructions in front of each load)
    constexpr int NLD = 4 * NCH / 256;
    long kb[2];  // element offsets (not pointers: a pointer array indexed per lane became flat loads)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        const int un = min(pair * 2 + s, units - 1);
        kb[s] = (long)(un / a.H) * T * a.ld + D + (un % a.H) * HD;
    }
    u16x8 kv[NLD];
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
        const int ci = tid + i * 256;
        const int s = ci / (2 * NCH), r = ci % (2 * NCH);
        const bool isV = r >= NCH;
        const int row = (r % NCH) / NCHL, ch = (r % NCH) % NCHL;
        kv[i] = *reinterpret_cast<const u16x8*>(a.qkv + (s ? kb[1] : kb[0]) + (long)min(row, T - 1) * a.ld +
                                                (isV ? D : 0) + ch * 8);
    }
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
        const int ci = tid + i * 256;
        const int s = ci / (2 * NCH), r = ci % (2 * NCH);
        const bool isV = r >= NCH;
        const int row = (r % NCH) / NCHL, ch = (r % NCH) % NCHL;
        if (isV)
            *reinterpret_cast<u16x8*>(&Vs[s][row * VS + ch * 8]) = kv[i];
        else
            *reinterpret_cast<u16x8*>(&Ks[s][row * KS + ch * 8]) = kv[i];
    }
    if (KZ > HD || VS > HD) {  // zero the padding columns (disjoint from the tile bytes)
        for (int i = tid; i < 2 * 64; i += 256) {
            bf16* kr = &Ks[i >> 6][(i & 63) * KS];
            for (int col = HD; col < KZ; col += 8) *reinterpret_cast<u16x8*>(kr + col) = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
            bf16* vr = &Vs[i >> 6][(i & 63) * VS];
            for (int col = HD; col < VS; col += 8) *reinterpret_cast<u16x8*>(vr + col) = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
        }
    }

    __syncthreads();

    const bf16* Kb = Ks[slot];
    const bf16* Vb = Vs[slot];
    f32x4 sc[2][4];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
        const bf16* krow = Kb + (kt * 16 + li) * KS;
        bf16x8 kf[NKS];
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) kf[ks] = *reinterpret_cast<const bf16x8*>(krow + ks * 32 + 8 * g);
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            f32x4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int ks = 0; ks < NKS; ++ks) z = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[ks], qf[u][ks], z, 0, 0, 0);
            sc[u][kt] = z;
        }
    }
    if (Tk < 64 || a.causal) {
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int q = qw0 + u * 16 + li;
            const int lim = a.causal ? min(Tk, q + 1) : Tk;
#pragma unroll
            for (int kt = 0; kt < 4; ++kt)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    if (kt * 16 + 4 * g + r >= lim) sc[u][kt][r] = -INFINITY;
        }
    }

    float lsum[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        float mloc = -1e30f;
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
            mloc = fmaxf(mloc, fmaxf(fmaxf(sc[u][kt][0], sc[u][kt][1]), fmaxf(sc[u][kt][2], sc[u][kt][3])));
        mloc = xmax32(xmax16(mloc));
        const float mc = mloc * c;
        float psum = 0.f;
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float pv = __builtin_amdgcn_exp2f(__builtin_fmaf(sc[u][kt][r], c, -mc));
                sc[u][kt][r] = pv;
                psum += pv;
            }
        lsum[u] = xsum32(xsum16(psum));
    }

    f32x4 o[2][NDT];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int i = 0; i < NDT; ++i) o[u][i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
        bf16x8 pb[2];
#pragma unroll
        for (int u = 0; u < 2; ++u)
            pb[u] = __builtin_convertvector(__builtin_shufflevector(sc[u][2 * hh], sc[u][2 * hh + 1], 0, 1, 2, 3, 4, 5,
                                                                    6, 7), bf16x8);
        const int r1 = 32 * hh + 4 * g + (li >> 2);
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) {
            const int col = dt * 16 + 4 * (li & 3);
            const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(Vb + r1 * VS + col));
            const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(Vb + (r1 + 16) * VS + col));
            const bf16x8 vv = __builtin_bit_cast(bf16x8, __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
            for (int u = 0; u < 2; ++u) o[u][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vv, pb[u], o[u][dt], 0, 0, 0);
        }
    }

    if (unit >= units) return;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const float inv = 1.0f / lsum[u];
        const int q = qw0 + u * 16 + li;
        if (q < T) {
            bf16* orow = a.out + ((long)b * T + q) * a.ldo + h * HD;
#pragma unroll
            for (int dt = 0; dt < NDT; ++dt) {
                const int d0 = dt * 16 + 4 * g;
                if (d0 < HD) {
                    bf16x4 v;
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[r] = f2bf(o[u][dt][r] * inv);
                    *reinterpret_cast<bf16x4*>(orow + d0) = v;
                }
            }
        }
    }
}

// attn_short2_kernel (round 6, kind 102): sequences of 65..128 tokens at head dim 64 -- the CLIP
// causal text towers (T 77: OpenAI-CLIP-L, LAION-CLIP-H, MetaCLIP, DFN5B-H). attn_fwd_kernel (kind 89)
// runs them as a two-tile flash loop: Q and key tile 0 loaded, then tile 1 loaded while tile 0
// computes -- two HBM round trips in series per block for a kernel that is HBM-bound (3.9 TB/s).
// Here a block = one (batch, head) unit and 4 waves of 32 queries; Q, and K / V of all 128 key rows
// (rows past T clamped: finite, masked), are loaded in one burst (8 + 4 loads per lane) before the
// first LDS write; the scores of all 128 keys stay in registers, so the softmax is one pass (no
// running max, no rescale). Waves whose 32 queries all lie past T only help load. Per-wave math is
// attn_short_kernel's (S^T = K.Q^T, P in registers as the B operand of O^T = V^T.P^T, V^T by
// ds_read_b64_tr_b16), over 8 key sub-tiles instead of 4.
template <int HD>
__global__ __launch_bounds__(256, 4) void attn_short2_kernel(AttnArgs a, int units) {
    static_assert(HD == 64, "attn_short2_kernel: head dim 64 (the CLIP text towers)");
    constexpr int NKS = HD / 32;
    constexpr int KS = HD + 8;   // K LDS row stride (elements)
    constexpr int VS = 80;       // V LDS row stride: conflict-free tr reads
    constexpr int NCHL = HD / 8;
    constexpr int NDT = HD / 16;
    constexpr int NCH = 128 * NCHL;          // 16-B chunks per K (or V) image
    constexpr int NLD = 2 * NCH / 256;       // K + V chunks per thread
    __shared__ __attribute__((aligned(16))) bf16 Ks[128 * KS];
    __shared__ __attribute__((aligned(16))) bf16 Vs[128 * VS];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int g = lane >> 4, li = lane & 15;
    const int T = a.T, D = a.H * HD;
    int unit;  // XCD-aware: consecutive units (neighbouring heads of one sequence) on one XCD / L2
    {
        const int bid = blockIdx.x, nwg = gridDim.x;
        const int xcd = bid & 7, loc = bid >> 3, q8 = nwg >> 3, r8 = nwg & 7;
        unit = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
    }
    if (unit >= units) return;  // uniform over the block
    const int b = unit / a.H, h = unit % a.H;
    const bf16* base = a.qkv + (long)b * T * a.ld + h * HD;
    const int qw0 = wave * 32;
    const int Tk = a.seq_lens ? a.seq_lens[b] : T;
    const float c = a.scale_log2;

    bf16x8 qf[2][NKS];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const bf16* qrow = base + (long)min(qw0 + u * 16 + li, T - 1) * a.ld;
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) qf[u][ks] = *reinterpret_cast<const bf16x8*>(qrow + ks * 32 + 8 * g);
    }
    u16x8 kv[NLD];
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
        const int ci = tid + i * 256;
        const bool isV = ci >= NCH;
        const int r = ci % NCH, row = r / NCHL, ch = r % NCHL;
        kv[i] = *reinterpret_cast<const u16x8*>(base + (long)min(row, T - 1) * a.ld + (isV ? 2 * D : D) + ch * 8);
    }
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
        const int ci = tid + i * 256;
        const bool isV = ci >= NCH;
        const int r = ci % NCH, row = r / NCHL, ch = r % NCHL;
        if (isV)
            *reinterpret_cast<u16x8*>(&Vs[row * VS + ch * 8]) = kv[i];
        else
            *reinterpret_cast<u16x8*>(&Ks[row * KS + ch * 8]) = kv[i];
    }
    __syncthreads();
    if (qw0 >= T) return;  // wave-uniform; no barrier follows

    f32x4 sc[2][8];
#pragma unroll
    for (int kt = 0; kt < 8; ++kt) {
        const bf16* krow = Ks + (kt * 16 + li) * KS;
        bf16x8 kf[NKS];
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) kf[ks] = *reinterpret_cast<const bf16x8*>(krow + ks * 32 + 8 * g);
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            f32x4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int ks = 0; ks < NKS; ++ks) z = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[ks], qf[u][ks], z, 0, 0, 0);
            sc[u][kt] = z;
        }
    }
    // keys past the sequence (T < 128: clamped duplicate rows), past its length or the causal diagonal
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const int q = qw0 + u * 16 + li;
        const int lim = a.causal ? min(Tk, q + 1) : Tk;  // valid keys: key < lim (<= T)
#pragma unroll
        for (int kt = 0; kt < 8; ++kt)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                if (kt * 16 + 4 * g + r >= lim) sc[u][kt][r] = -INFINITY;
    }

    float lsum[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        float mloc = -1e30f;
#pragma unroll
        for (int kt = 0; kt < 8; ++kt)
            mloc = fmaxf(mloc, fmaxf(fmaxf(sc[u][kt][0], sc[u][kt][1]), fmaxf(sc[u][kt][2], sc[u][kt][3])));
        mloc = xmax32(xmax16(mloc));
        const float mc = mloc * c;
        float psum = 0.f;
#pragma unroll
        for (int kt = 0; kt < 8; ++kt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float pv = __builtin_amdgcn_exp2f(__builtin_fmaf(sc[u][kt][r], c, -mc));
                sc[u][kt][r] = pv;
                psum += pv;
            }
        lsum[u] = xsum32(xsum16(psum));
    }

    f32x4 o[2][NDT];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int i = 0; i < NDT; ++i) o[u][i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int hh = 0; hh < 4; ++hh) {
        bf16x8 pb[2];
#pragma unroll
        for (int u = 0; u < 2; ++u)
            pb[u] = __builtin_convertvector(__builtin_shufflevector(sc[u][2 * hh], sc[u][2 * hh + 1], 0, 1, 2, 3, 4, 5,
                                                                    6, 7), bf16x8);
        const int r1 = 32 * hh + 4 * g + (li >> 2);
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) {
            const int col = dt * 16 + 4 * (li & 3);
            const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(Vs + r1 * VS + col));
            const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(Vs + (r1 + 16) * VS + col));
            const bf16x8 vv = __builtin_bit_cast(bf16x8, __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
            for (int u = 0; u < 2; ++u) o[u][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vv, pb[u], o[u][dt], 0, 0, 0);
        }
    }

#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const float inv = 1.0f / lsum[u];
        const int q = qw0 + u * 16 + li;
        if (q < T) {
            bf16* orow = a.out + ((long)b * T + q) * a.ldo + h * HD;
#pragma unroll
            for (int dt = 0; dt < NDT; ++dt) {
                bf16x4 v;
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] = f2bf(o[u][dt][r] * inv);
                *reinterpret_cast<bf16x4*>(orow + dt * 16 + 4 * g) = v;
            }
        }
    }
}

#ifdef MME_DEV
// attn_short_pf_kernel (dev, round 3): attn_short_kernel as a persistent loop over unit pairs
// whose next pair's Q fragments and K / V chunks are loaded into registers while the current
// pair computes (the short kernel's workgroups each load, then compute, then store, with no
// loads in flight across those phases). Same per-pair math, so bit-identical to kind 16.
template <int HD>
__global__ __launch_bounds__(256, 2) void attn_short_pf_kernel(AttnArgs a, int units, int npairs) {
    constexpr int HDP = HD == 64 ? 64 : 96;
    constexpr int NKS = HDP / 32;
    constexpr int KS = HDP + 8;
    constexpr int VS = 80;
    constexpr int NCHL = HD / 8;
    constexpr int NDT = (HD + 15) / 16;
    constexpr int NCH = 64 * NCHL;
    constexpr int NLD = 4 * NCH / 256;  // 16-B K / V chunks per thread and pair
    static_assert((4 * NCH) % 256 == 0, "K + V tiles of both slots split evenly over 256 threads");
    __shared__ __attribute__((aligned(16))) bf16 sm[2 * 64 * KS + 2 * 64 * VS];
    bf16 (*Ks)[64 * KS] = reinterpret_cast<bf16 (*)[64 * KS]>(sm);
    bf16 (*Vs)[64 * VS] = reinterpret_cast<bf16 (*)[64 * VS]>(sm + 2 * 64 * KS);

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int g = lane >> 4, li = lane & 15;
    const int T = a.T, D = a.H * HD;
    const int slot = wave >> 1, qw0 = (wave & 1) * 32;
    const float c = a.scale_log2;
    // XCD-aware pair order: the block's XCD owns a contiguous range of pairs (neighbouring heads
    // of one sequence share 128-B lines), walked by the blocks of that XCD in turn
    const int bid = blockIdx.x, nwg = gridDim.x;
    const int xcd = bid & 7, loc = bid >> 3, q8 = nwg >> 3, r8 = nwg & 7;
    const int nblk = xcd < r8 ? q8 + 1 : q8;  // blocks on this XCD
    const int p8 = npairs >> 3, pr8 = npairs & 7;
    const int pbeg = xcd < pr8 ? xcd * (p8 + 1) : pr8 * (p8 + 1) + (xcd - pr8) * p8;
    const int pend = pbeg + (xcd < pr8 ? p8 + 1 : p8);

    if (KS > HD || VS > HD) {  // padding columns: zeroed once, never overwritten by the tiles
        for (int i = tid; i < 2 * 64; i += 256) {
            bf16* kr = &Ks[i >> 6][(i & 63) * KS];
            for (int col = HD; col < KS; col += 8) *reinterpret_cast<u16x8*>(kr + col) = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
            bf16* vr = &Vs[i >> 6][(i & 63) * VS];
            for (int col = HD; col < VS; col += 8) *reinterpret_cast<u16x8*>(vr + col) = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
        }
    }
    bf16x8 qf[2][NKS];
    u16x8 kvn[NLD];
    auto load_q = [&](int pair) {  // Q fragments of this wave's unit (dead after QK^T: reloaded there)
        const int uc = min(pair * 2 + slot, units - 1);
        const int b = uc / a.H, h = uc % a.H;
        const bf16* base = a.qkv + (long)b * T * a.ld;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const bf16* qrow = base + (long)min(qw0 + u * 16 + li, T - 1) * a.ld + h * HD;
#pragma unroll
            for (int ks = 0; ks < NKS; ++ks) {
                const int col = ks * 32 + 8 * g;
                qf[u][ks] = col < HD ? *reinterpret_cast<const bf16x8*>(qrow + col) : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
            }
        }
    };
    // per-thread chunk offsets within a unit's rows (pair-invariant; slot s of chunk i is
    // compile-time: NCH * 2 chunks per slot, 256 threads, so i < NLD / 2 is slot 0 when NLD is even)
    int koff[NLD];
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
        const int ci = tid + i * 256;
        const int r = ci % (2 * NCH);
        const bool isV = r >= NCH;
        const int row = (r % NCH) / NCHL, ch = (r % NCH) % NCHL;
        koff[i] = min(row, T - 1) * a.ld + (isV ? 2 : 1) * D + ch * 8;
    }
    auto load = [&](int pair) {  // K / V chunks of both units into registers
        const int u0 = min(pair * 2, units - 1), u1 = min(pair * 2 + 1, units - 1);
        const bf16* b0 = a.qkv + (long)(u0 / a.H) * T * a.ld + (u0 % a.H) * HD;
        const bf16* b1 = a.qkv + (long)(u1 / a.H) * T * a.ld + (u1 % a.H) * HD;
#pragma unroll
        for (int i = 0; i < NLD; ++i) {
            const int s = (tid + i * 256) / (2 * NCH);
            kvn[i] = *reinterpret_cast<const u16x8*>((s ? b1 : b0) + koff[i]);
        }
    };
    int pair = pbeg + loc;
    if (pair < pend) {
        load_q(pair);
        load(pair);
    }
    for (; pair < pend; pair += nblk) {
        // the prefetched pair -> LDS / fragments (every wave is past the previous pair's LDS reads)
#pragma unroll
        for (int i = 0; i < NLD; ++i) {
            const int ci = tid + i * 256;
            const int s = ci / (2 * NCH), r = ci % (2 * NCH);
            const bool isV = r >= NCH;
            const int row = (r % NCH) / NCHL, ch = (r % NCH) % NCHL;
            if (isV)
                *reinterpret_cast<u16x8*>(&Vs[s][row * VS + ch * 8]) = kvn[i];
            else
                *reinterpret_cast<u16x8*>(&Ks[s][row * KS + ch * 8]) = kvn[i];
        }
        __syncthreads();
        const int unit = pair * 2 + slot;
        const int uc = min(unit, units - 1);
        const int b = uc / a.H, h = uc % a.H;
        const int Tk = a.seq_lens ? a.seq_lens[b] : T;
        if (pair + nblk < pend) load(pair + nblk);  // next pair's loads fly under this pair's math

        const bf16* Kb = Ks[slot];
        const bf16* Vb = Vs[slot];
        f32x4 sc[2][4];
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) {
            const bf16* krow = Kb + (kt * 16 + li) * KS;
            bf16x8 kf[NKS];
#pragma unroll
            for (int ks = 0; ks < NKS; ++ks) kf[ks] = *reinterpret_cast<const bf16x8*>(krow + ks * 32 + 8 * g);
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                f32x4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int ks = 0; ks < NKS; ++ks) z = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[ks], qf[u][ks], z, 0, 0, 0);
                sc[u][kt] = z;
            }
        }
        if (pair + nblk < pend) load_q(pair + nblk);
        if (Tk < 64 || a.causal) {
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int q = qw0 + u * 16 + li;
                const int lim = a.causal ? min(Tk, q + 1) : Tk;
#pragma unroll
                for (int kt = 0; kt < 4; ++kt)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        if (kt * 16 + 4 * g + r >= lim) sc[u][kt][r] = -INFINITY;
            }
        }
        float lsum[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            float mloc = -1e30f;
#pragma unroll
            for (int kt = 0; kt < 4; ++kt)
                mloc = fmaxf(mloc, fmaxf(fmaxf(sc[u][kt][0], sc[u][kt][1]), fmaxf(sc[u][kt][2], sc[u][kt][3])));
            mloc = xmax32(xmax16(mloc));
            const float mc = mloc * c;
            float psum = 0.f;
#pragma unroll
            for (int kt = 0; kt < 4; ++kt)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float pv = __builtin_amdgcn_exp2f(__builtin_fmaf(sc[u][kt][r], c, -mc));
                    sc[u][kt][r] = pv;
                    psum += pv;
                }
            lsum[u] = xsum32(xsum16(psum));
        }
        f32x4 o[2][NDT];
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int i = 0; i < NDT; ++i) o[u][i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
            bf16x8 pb[2];
#pragma unroll
            for (int u = 0; u < 2; ++u)
                pb[u] = __builtin_convertvector(__builtin_shufflevector(sc[u][2 * hh], sc[u][2 * hh + 1], 0, 1, 2, 3, 4,
                                                                        5, 6, 7), bf16x8);
            const int r1 = 32 * hh + 4 * g + (li >> 2);
#pragma unroll
            for (int dt = 0; dt < NDT; ++dt) {
                const int col = dt * 16 + 4 * (li & 3);
                const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(Vb + r1 * VS + col));
                const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(Vb + (r1 + 16) * VS + col));
                const bf16x8 vv = __builtin_bit_cast(bf16x8, __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7));
#pragma unroll
                for (int u = 0; u < 2; ++u) o[u][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vv, pb[u], o[u][dt], 0, 0, 0);
            }
        }
        if (unit < units) {
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const float inv = 1.0f / lsum[u];
                const int q = qw0 + u * 16 + li;
                if (q < T) {
                    bf16* orow = a.out + ((long)b * T + q) * a.ldo + h * HD;
#pragma unroll
                    for (int dt = 0; dt < NDT; ++dt) {
                        const int d0 = dt * 16 + 4 * g;
                        if (d0 < HD) {
                            bf16x4 v;
#pragma unroll
                            for (int r = 0; r < 4; ++r) v[r] = f2bf(o[u][dt][r] * inv);
                            *reinterpret_cast<bf16x4*>(orow + d0) = v;
                        }
                    }
                }
            }
        }
        __syncthreads();  // every wave is done reading this pair's K / V before the next overwrite
    }
}
#endif

// ---------------------------------------------------------------------------
// attn_m32_kernel: the LDS-DMA flash loop on v_mfma_f32_32x32x16_bf16 (round 2).
// attn_pipe_kernel's counters (profiles/r02_pmc_attn_siglip_vision.json) put the
// hd-72 loop at the SIMD's vector-issue limit: per wave and 64-key tile 44
// 16x16x32 MFMAs hold the issue port 8 cycles each (352) beside ~600 cycles of
// softmax VALU, against 704 cycles of MFMA pipe work. A 32x32x16 MFMA does twice
// the work per issue (8 of its 32 cycles), so the same tile takes 22 MFMAs and
// 176 issue cycles, and the reduction depth is 16: head dim 72 / 80 runs the
// QK^T product 80 deep (5 steps) instead of 96.
//   * S^T = K . Q^T (A = K rows, B = Q^T): lane (r, h) = (lane & 31, lane >> 5)
//     holds query r and keys (reg & 3) + 8 (reg >> 2) + 4 h of each 32-key block,
//     so the row max is lane-local plus one v_permlane32_swap;
//   * registers 8 s' .. 8 s' + 7 of a key block, packed to bf16, are directly the
//     B operand (P^T) of O^T = V^T . P^T for the keys 16 s' .. 16 s' + 15 of that
//     block (cdna_hip_programming.md §3 'accumulator tile as the next operand');
//     the V^T operand takes the same permuted key order from two
//     ds_read_b64_tr_b16 (keys +4h + 0..3 and +8 + 4h + 0..3);
//   * K / V tiles of 64 keys land by LDS-DMA as "chunk planes" (plane c = 16-B
//     column chunk c of all 64 keys, 1 KiB, lane = key). V plane c stores key k
//     in slot k ^ (4 (c & 3)) (through the per-lane DMA source row), which makes
//     the transposed reads of a 32-lane half (4 planes x 4 keys) hit 64
//     distinct banks; the K reads (512 contiguous bytes per half) are
//     conflict-free unswizzled;
//   * O^T covers ceil((HD + 1) / 32) d-blocks of 32: at head dims 72 / 80 the
//     V^T row HD (inside the padding) is a plane of ones, so O^T row HD is the
//     softmax weight sum Σ bf16(p) and the per-tile sums disappear (HD 64: f32 adds);
//   * lazy rescale (alpha == 1 exactly when no row max of the wave grew), static
//     priority for the second half of the waves, tile loop unrolled by the 2-deep
//     ring (every LDS address a lane base + immediate), 16-B O stores after a
//     v_permlane32_swap of the two lane halves.
// ---------------------------------------------------------------------------
// SKIP (round 3, kind 65): a tile whose second 32-key block lies wholly past the keys skips
// that block's QK^T and PV MFMAs, as attn_hyb_kernel's kind 62 does at hd 72 -- ViT-H
// (T = 257 = 4 x 64 + 1) ends in such a tile (1/10 of the key blocks). Its P is 0, and an MFMA
// with an all-zero operand leaves its accumulator bit-identical (tools/mfma_zero_probe.hip, round 4),
// so the skip is exact; yet 0-18 of 0.1-3.7 M outputs differ from the unskipped kernel by one bf16
// ulp, a deterministic code-generation effect of these compiled loops (printf instrumentation of the
// unskipped kernel alone moves outputs the same way; DESIGN.md §4 round 4, test_attention_skip_vs_
// unskipped). The same skip in 8-wave blocks (DFN5B,
// T = 730) measured 18 % slower than kind 38 (0.59 vs 0.50 ms, profiles/r03_v11_attn_dfn5b_ab.log)
// and is not built.
// THR (round 4, kinds 86-88): rescale O only when a query's running max grows by more than 2^8 in the
// exp2 domain (attn_hyb_kernel's XT 2; P <= 256 otherwise, the weight sums share the stale max).
template <int HD, int NW, int MINW, bool PRIO, bool DPV = false, bool PF = false, bool SKIP = false, bool THR = false,
          bool BIAS = false>
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(MINW))) void attn_m32_kernel(AttnArgs a) {
    constexpr int NSTG = DPV ? 3 : 2;
    constexpr bool ONES = HD % 32 != 0;
    constexpr int NCHL = HD / 8;                    // K / V planes with data
    // BIAS (round 6, with THR; Q pre-scaled by the caller, mme_attention_qs): attn_hyb_kernel's XT 4 --
    // Q^T row HD holds -M (the running max as a bf16 value) against a ones row of K, so the QK^T MFMAs
    // return c s - M. Row HD lies in the zero padding of the last k-step at hd 72; hd 80 adds a k-step.
    static_assert(!BIAS || (THR && !DPV && !PF && HD % 32 != 0), "BIAS: threshold rescale, plain loop, hd 72 / 80");
    constexpr int NKS = (HD + 15) / 16 + (BIAS && HD % 16 == 0 ? 1 : 0);  // QK^T k-steps of 16
    constexpr int KSB = HD / 16, HHB = (HD % 16) / 8;  // BIAS: Q^T row HD = k-step KSB, lane half HHB, element 0
    constexpr int NDB = (HD + (ONES ? 1 : 0) + 31) / 32;  // O^T d-blocks of 32
    constexpr int NVP = 4 * NDB;                    // V planes read (data, ones, zero padding)
    constexpr int TILE = (NCHL + NVP) * 1024;
    constexpr int NINS = 2 * NCHL;
    constexpr int MAXI = (NINS + NW - 1) / NW;
    constexpr int QB = NW * 32;
    static_assert(2 * NKS <= NCHL + NVP, "K reads past the head dim stay inside the tile");
    __shared__ __attribute__((aligned(16))) char lds[NSTG * TILE];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 31, hh = lane >> 5;
    float mb = 0.f;  // BIAS: the running max M that Q^T row HD holds as -M
    const int nqb = (a.T + QB - 1) / QB;
    int id;
    {
        const int bid = blockIdx.x, nwg = gridDim.x;
        const int xcd = bid & 7, loc = bid >> 3, q8 = nwg >> 3, r8 = nwg & 7;
        id = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
    }
    const int qb = id % nqb, h = (id / nqb) % a.H, b = id / (nqb * a.H);
    const int T = a.T, D = a.H * HD;
    const bf16* base = a.qkv + (long)b * T * a.ld;
    const int qw0 = qb * QB + wave * 32;
    const int Tk = a.seq_lens ? a.seq_lens[b] : T;
    const float c = a.scale_log2;

    // V planes past the data: the ones plane (ONES) and zero padding, in both ring slots
    constexpr int NPAD = NVP > NCHL ? NVP - NCHL : 1;
    for (int i = tid; i < NSTG * (NVP - NCHL) * 64; i += NW * 64) {
        const int slot = i / (NPAD * 64), rem = i % (NPAD * 64);
        const int pl = NCHL + rem / 64;
        const unsigned short v = (ONES && pl == NCHL) ? 0x3F80 : 0;
        *reinterpret_cast<u16x8*>(lds + slot * TILE + (NCHL + pl) * 1024 + (rem & 63) * 16) =
            u16x8{v, v, v, v, v, v, v, v};
    }

    bf16x8 qf[NKS];  // B operand: Q^T[d = 16 ks + 8 hh + j][query r]
    {
        const bf16* qrow = base + (long)min(qw0 + r, T - 1) * a.ld + h * HD;
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
            const int col = ks * 16 + 8 * hh;
            if (col < HD)
                qf[ks] = *reinterpret_cast<const bf16x8*>(qrow + col);
            else
                qf[ks] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
        }
    }

    int nkt = (Tk + 63) / 64;
    if (a.causal) nkt = min(nkt, (min(T, qb * QB + QB) + 63) / 64);

    auto issue = [&](int t) {
        char* tb = lds + (t % NSTG) * TILE;
#pragma unroll
        for (int i = 0; i < MAXI; ++i) {
            const int idx = wave + NW * i;
            if (i < MAXI - 1 || idx < NINS) {
                const bool isV = idx >= NCHL;
                const int plane = isV ? idx - NCHL : idx;
                const int key = isV ? lane ^ (4 * (plane & 3)) : lane;
                const bf16* src = base + (long)min(t * 64 + key, T - 1) * a.ld + (isV ? 2 : 1) * D + h * HD + plane * 8;
                glds16(src, tb + idx * 1024);
            }
        }
    };

    const unsigned lds0 = (unsigned)(uintptr_t)(LDS_AS char*)lds;
    // K fragment (A operand) of k-step ks, key block kb: plane 2 ks + hh, key 32 kb + r
    const unsigned kb0 = lds0 + hh * 1024 + r * 16;
    // BIAS: k-step KSB's lanes past the head dim read the ones plane (V plane NCHL = tile plane 2 NCHL)
    const unsigned kbb = (HD % 16 == 0 || hh == HHB) ? lds0 + 2 * NCHL * 1024 + r * 16 : kb0 + KSB * 2048;
    auto kaddr = [&](int ks) { return (BIAS && ks == KSB) ? kbb : kb0 + ks * 2048; };
    // V^T fragment (A operand) of d-block db, key step (kb, s'): two transposed reads,
    // keys 32 kb + 16 s' + 8 j + 4 hh + q (j = 0, 1) at d = 32 db + 16 half + 4 p .. + 3
    unsigned vbj[2];
    {
        const int i16 = lane & 15, q = i16 >> 2, p = i16 & 3, half = (lane >> 4) & 1;
        const int cc = 2 * half + (p >> 1);
#pragma unroll
        for (int j = 0; j < 2; ++j)
            vbj[j] = lds0 + (NCHL + cc) * 1024 + (((8 * j + 4 * hh + q) ^ (4 * cc)) * 16) + (p & 1) * 8;
    }

    f32x16 o[NDB];
#pragma unroll
    for (int i = 0; i < NDB; ++i)
#pragma unroll
        for (int e = 0; e < 16; ++e) o[i][e] = 0.f;
    float m = -1e30f, lsum = 0.f;

    // PF: every LDS fragment a product needs is read ahead of its MFMAs (the 10 K fragments
    // before QK^T, the 24 transposed V reads before the softmax, whose VALU covers their
    // latency); without it the register-capped build re-uses one fragment register and waits
    // lgkmcnt(0) in front of every MFMA.
    auto qk_pf = [&](int t, const unsigned so, f32x16(&sc)[2]) __attribute__((always_inline)) {
        bf16x8 kf[2][NKS];
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int ks = 0; ks < NKS; ++ks)
                kf[kb][ks] = *reinterpret_cast<const LDS_AS bf16x8*>((uintptr_t)(kb0 + so + kb * 512 + ks * 2048));
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
            f32x16 z;
#pragma unroll
            for (int e = 0; e < 16; ++e) z[e] = 0.f;
#pragma unroll
            for (int ks = 0; ks < NKS; ++ks) z = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf[kb][ks], qf[ks], z, 0, 0, 0);
            sc[kb] = z;
        }
    };
    auto qk = [&](int t, const unsigned so, f32x16(&sc)[2]) __attribute__((always_inline)) {
        const bool half = SKIP && t * 64 + 32 >= Tk;
        if constexpr (PF) {
            qk_pf(t, so, sc);
        } else {
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
            f32x16 z;
#pragma unroll
            for (int e = 0; e < 16; ++e) z[e] = kb == 1 && half ? -INFINITY : 0.f;
            if (kb == 1 && half) {
                sc[kb] = z;
                continue;
            }
#pragma unroll
            for (int ks = 0; ks < NKS; ++ks) {
                const bf16x8 kf = *reinterpret_cast<const LDS_AS bf16x8*>((uintptr_t)(kaddr(ks) + so + kb * 512));
                z = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[ks], z, 0, 0, 0);
            }
            sc[kb] = z;
        }
        }
        if ((t * 64 + 64 > Tk) || (a.causal && t * 64 + 63 > qw0)) {
            const int q = qw0 + r;
            const int lim = a.causal ? min(Tk, q + 1) : Tk;
#pragma unroll
            for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                for (int e = 0; e < 16; ++e)
                    if (t * 64 + kb * 32 + (e & 3) + 8 * (e >> 2) + 4 * hh >= lim) sc[kb][e] = -INFINITY;
        }
    };
    // online softmax of one tile's scores: running max, lazy O rescale, P packed to bf16
    // (pk[2 kb + s'] = registers 8 s' .. 8 s' + 7 of key block kb)
    auto softmax = [&](f32x16(&sc)[2], bf16x8(&pk)[4], int t = 0) {
        float mloc = fmaxf(sc[0][0], sc[0][1]);
#pragma unroll
        for (int e = 2; e < 16; ++e) mloc = fmaxf(mloc, sc[0][e]);
#pragma unroll
        for (int e = 0; e < 16; ++e) mloc = fmaxf(mloc, sc[1][e]);
        if constexpr (BIAS) {  // scores are c s - M: attn_hyb_kernel's XT 4 rescale
            if (t == 0 || __builtin_amdgcn_ballot_w64(mloc > 8.0f)) {
                const float mq = xmax32(mloc);
                const float mn = bf2f(f2bf(mb + (t == 0 ? mq : fmaxf(mq, 0.f))));
                const float d = mn - mb;  // exact: both bf16 values
                if (t > 0) {
                    const float alpha = __builtin_amdgcn_exp2f(-d);
#pragma unroll
                    for (int i = 0; i < NDB; ++i) o[i] *= alpha;
                }
#pragma unroll
                for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                    for (int e = 0; e < 16; ++e) sc[kb][e] -= d;
                mb = mn;
                uint4 w = __builtin_bit_cast(uint4, qf[KSB]);
                const unsigned nb = __builtin_bit_cast(unsigned short, f2bf(-mn));
                w.x = hh == HHB ? nb : w.x;  // Q^T row HD (row HD + 1 stays 0)
                qf[KSB] = __builtin_bit_cast(bf16x8, w);
            }
#pragma unroll
            for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                for (int e = 0; e < 16; ++e) sc[kb][e] = __builtin_amdgcn_exp2f(sc[kb][e]);
#pragma unroll
            for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                for (int sp = 0; sp < 2; ++sp)
#pragma unroll
                    for (int j = 0; j < 8; ++j) pk[2 * kb + sp][j] = f2bf(sc[kb][8 * sp + j]);
            return;
        }
        mloc = xmax32(mloc);
        const float mnew = fmaxf(m, mloc);
        if (__builtin_amdgcn_ballot_w64(THR ? (mloc - m) * c > 8.0f : mnew != m)) {
            const float alpha = __builtin_amdgcn_exp2f((m - mnew) * c);
            if (!ONES) lsum *= alpha;
#pragma unroll
            for (int i = 0; i < NDB; ++i) o[i] *= alpha;
            if (THR) m = mnew;
        }
        if (!THR) m = mnew;
        const float mc = m * c;
        float psum = 0.f;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const float pv = __builtin_amdgcn_exp2f(__builtin_fmaf(sc[kb][e], c, -mc));
                sc[kb][e] = pv;
                if (!ONES) psum += pv;
            }
        if (!ONES) lsum += psum;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int sp = 0; sp < 2; ++sp)
#pragma unroll
                for (int j = 0; j < 8; ++j) pk[2 * kb + sp][j] = f2bf(sc[kb][8 * sp + j]);
    };
    auto pv = [&](const unsigned so, const bf16x8(&pk)[4], bool half = false) {
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
            if (SKIP && kb == 1 && half) break;
#pragma unroll
            for (int sp = 0; sp < 2; ++sp)
#pragma unroll
                for (int db = 0; db < NDB; ++db) {
                    const unsigned off = so + db * 4096 + kb * 512 + sp * 256;
                    const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(uintptr_t)(vbj[0] + off));
                    const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(uintptr_t)(vbj[1] + off));
                    const bf16x8 vv = __builtin_bit_cast(bf16x8, __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7));
                    o[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vv, pk[2 * kb + sp], o[db], 0, 0, 0);
                }
        }
    };
    // PF: V^T fragments read before the softmax, MFMAs after it
    auto vread = [&](const unsigned so, bf16x8(&vf)[4][NDB]) __attribute__((always_inline)) {
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int sp = 0; sp < 2; ++sp)
#pragma unroll
                for (int db = 0; db < NDB; ++db) {
                    const unsigned off = so + db * 4096 + kb * 512 + sp * 256;
                    const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(uintptr_t)(vbj[0] + off));
                    const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(uintptr_t)(vbj[1] + off));
                    vf[2 * kb + sp][db] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7));
                }
    };
    auto pv_pf = [&](const bf16x8(&vf)[4][NDB], const bf16x8(&pk)[4]) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int db = 0; db < NDB; ++db) o[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf[i][db], pk[i], o[db], 0, 0, 0);
    };
    auto tile_pf = [&](int t, const unsigned so, f32x16(&sc)[2], bf16x8(&pk)[4]) __attribute__((always_inline)) {
        bf16x8 vf[4][NDB];
        qk(t, so, sc);
        vread(so, vf);
        __builtin_amdgcn_sched_barrier(0);
        softmax(sc, pk);
        pv_pf(vf, pk);
    };

    if (PRIO && wave >= NW / 2) __builtin_amdgcn_s_setprio(1);
    if (nkt > 0) issue(0);
    f32x16 sc[2];
    bf16x8 pk[4];
    if constexpr (PF) {
        for (int t = 0; t < nkt; t += 2) {
            vm_wait<0>();
            __builtin_amdgcn_s_barrier();
            if (t + 1 < nkt) issue(t + 1);
            tile_pf(t, 0, sc, pk);
            if (t + 1 < nkt) {
                vm_wait<0>();
                __builtin_amdgcn_s_barrier();
                if (t + 2 < nkt) issue(t + 2);
                tile_pf(t + 1, TILE, sc, pk);
            }
        }
    } else if constexpr (!DPV) {
        for (int t = 0; t < nkt; t += 2) {
            vm_wait<0>();
            __builtin_amdgcn_s_barrier();
            if (t + 1 < nkt) issue(t + 1);
            qk(t, 0, sc);
            softmax(sc, pk, t);
            pv(0, pk, SKIP && t * 64 + 32 >= Tk);
            if (t + 1 < nkt) {
                vm_wait<0>();
                __builtin_amdgcn_s_barrier();
                if (t + 2 < nkt) issue(t + 2);
                qk(t + 1, TILE, sc);
                softmax(sc, pk, t + 1);
                pv(TILE, pk, SKIP && (t + 1) * 64 + 32 >= Tk);
            }
        }
    } else {
        // delayed PV: iteration t runs QK(t), then PV(t - 1) -- MFMAs independent of tile t's
        // softmax, which the wave issues beside them -- then softmax(t) (its O rescale after
        // PV(t - 1) in program order). 3-slot ring: tile t + 1 lands in the slot of t - 2, whose
        // last reads (PV(t - 2), iteration t - 1) precede this iteration's barrier.
        for (int t = 0; t < nkt; t += 3) {
#pragma unroll
            for (int u = 0; u < 3; ++u) {
                const int tt = t + u;
                if (tt < nkt) {
                    vm_wait<0>();
                    __builtin_amdgcn_s_barrier();
                    if (tt + 1 < nkt) issue(tt + 1);
                    qk(tt, u * TILE, sc);
                    if (tt > 0) pv(((u + 2) % 3) * TILE, pk);
                    softmax(sc, pk);
                }
            }
        }
        if (nkt > 0) pv(((nkt - 1) % 3) * TILE, pk);
    }

    float ltot;
    if (ONES) {
        // register 4 (HD % 32) / 8 of d-block HD / 32 is O^T row HD + 4 hh: both rows lie in
        // the ones plane (columns HD .. HD + 7), so every lane holds its query's weight sum
        constexpr int DB1 = HD / 32, REG1 = 4 * ((HD % 32) / 8);
        ltot = o[DB1][REG1];
    } else {
        ltot = xsum32(lsum);
    }
    const float inv = 1.0f / ltot;
    const int q = qw0 + r;
    bf16* orow = a.out + ((long)b * T + min(q, T - 1)) * a.ldo + h * HD;
    // registers 4 mm .. 4 mm + 3 of d-block db = columns 32 db + 8 mm + 4 hh .. + 3; a
    // permlane32 swap of the pair (mm, mm + 1) gives lane half hh the 8 columns 32 db + 8 (mm + hh) ..
#pragma unroll
    for (int db = 0; db < NDB; ++db)
#pragma unroll
        for (int mm = 0; mm < 4; mm += 2) {
            if (32 * db + 8 * mm >= HD) continue;
            bf16x4 v0, v1;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                v0[e] = f2bf(o[db][4 * mm + e] * inv);
                v1[e] = f2bf(o[db][4 * mm + 4 + e] * inv);
            }
            const uint2 x = __builtin_bit_cast(uint2, v0), y = __builtin_bit_cast(uint2, v1);
            const auto sx = __builtin_amdgcn_permlane32_swap(x.x, y.x, false, false);
            const auto sy = __builtin_amdgcn_permlane32_swap(x.y, y.y, false, false);
            const int d0 = 32 * db + 8 * (mm + hh);
            if (q < T && d0 + 8 <= HD) *reinterpret_cast<uint4*>(orow + d0) = make_uint4(sx[0], sy[0], sx[1], sy[1]);
        }
}

// ---------------------------------------------------------------------------
// attn_m32x2_kernel: attn_m32_kernel with TWO 32-query sub-blocks per wave. The hd-72 loop
// reads ~22 KiB of K / V fragments from LDS per wave and tile (10 K reads of 1 KiB, 24
// transposed V reads of 512 B); at 4 waves per SIMD that is ~80 % of the LDS array's
// 256 B/clk over the measured tile time, i.e. the loop is bound by the LDS reads, which
// neither the MFMA shape nor the issue order changes. Here every K / V fragment read
// feeds the MFMAs of both sub-blocks (64 queries), halving the LDS read bytes per FLOP.
// Registers: Q^T fragments, O^T accumulators, running max / sum per sub-block (~220
// VGPRs: 2 waves per SIMD); NW = 4 waves = 256 queries per block, two blocks per CU.
// Sub-block math, LDS layout, DMA and output are attn_m32_kernel's.
// ---------------------------------------------------------------------------
template <int V>
struct IC {
    static constexpr int value = V;
};

template <int HD, int NW, bool PRIO, bool ILV = false>
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(2))) void attn_m32x2_kernel(AttnArgs a) {
    constexpr bool ONES = HD % 32 != 0;
    constexpr int NCHL = HD / 8;
    constexpr int NKS = (HD + 15) / 16;
    constexpr int NDB = (HD + (ONES ? 1 : 0) + 31) / 32;
    constexpr int NVP = 4 * NDB;
    constexpr int TILE = (NCHL + NVP) * 1024;
    constexpr int NINS = 2 * NCHL;
    constexpr int MAXI = (NINS + NW - 1) / NW;
    constexpr int QB = NW * 64;
    static_assert(2 * NKS <= NCHL + NVP, "K reads past the head dim stay inside the tile");
    __shared__ __attribute__((aligned(16))) char lds[2 * TILE];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 31, hh = lane >> 5;
    const int nqb = (a.T + QB - 1) / QB;
    int id;
    {
        const int bid = blockIdx.x, nwg = gridDim.x;
        const int xcd = bid & 7, loc = bid >> 3, q8 = nwg >> 3, r8 = nwg & 7;
        id = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
    }
    const int qb = id % nqb, h = (id / nqb) % a.H, b = id / (nqb * a.H);
    const int T = a.T, D = a.H * HD;
    const bf16* base = a.qkv + (long)b * T * a.ld;
    const int qw0 = qb * QB + wave * 64;  // sub-block u: queries qw0 + 32 u + r
    const int Tk = a.seq_lens ? a.seq_lens[b] : T;
    const float c = a.scale_log2;

    constexpr int NPAD = NVP > NCHL ? NVP - NCHL : 1;
    for (int i = tid; i < 2 * (NVP - NCHL) * 64; i += NW * 64) {
        const int slot = i / (NPAD * 64), rem = i % (NPAD * 64);
        const int pl = NCHL + rem / 64;
        const unsigned short v = (ONES && pl == NCHL) ? 0x3F80 : 0;
        *reinterpret_cast<u16x8*>(lds + slot * TILE + (NCHL + pl) * 1024 + (rem & 63) * 16) =
            u16x8{v, v, v, v, v, v, v, v};
    }

    bf16x8 qf[2][NKS];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const bf16* qrow = base + (long)min(qw0 + 32 * u + r, T - 1) * a.ld + h * HD;
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
            const int col = ks * 16 + 8 * hh;
            if (col < HD)
                qf[u][ks] = *reinterpret_cast<const bf16x8*>(qrow + col);
            else
                qf[u][ks] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
        }
    }

    int nkt = (Tk + 63) / 64;
    if (a.causal) nkt = min(nkt, (min(T, qb * QB + QB) + 63) / 64);

    auto issue = [&](int t) {
        char* tb = lds + (t & 1) * TILE;
#pragma unroll
        for (int i = 0; i < MAXI; ++i) {
            const int idx = wave + NW * i;
            if (i < MAXI - 1 || idx < NINS) {
                const bool isV = idx >= NCHL;
                const int plane = isV ? idx - NCHL : idx;
                const int key = isV ? lane ^ (4 * (plane & 3)) : lane;
                const bf16* src = base + (long)min(t * 64 + key, T - 1) * a.ld + (isV ? 2 : 1) * D + h * HD + plane * 8;
                glds16(src, tb + idx * 1024);
            }
        }
    };

    const unsigned lds0 = (unsigned)(uintptr_t)(LDS_AS char*)lds;
    const unsigned kb0 = lds0 + hh * 1024 + r * 16;
    unsigned vbj[2];
    {
        const int i16 = lane & 15, q = i16 >> 2, p = i16 & 3, half = (lane >> 4) & 1;
        const int cc = 2 * half + (p >> 1);
#pragma unroll
        for (int j = 0; j < 2; ++j)
            vbj[j] = lds0 + (NCHL + cc) * 1024 + (((8 * j + 4 * hh + q) ^ (4 * cc)) * 16) + (p & 1) * 8;
    }

    f32x16 o[2][NDB];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int i = 0; i < NDB; ++i)
#pragma unroll
            for (int e = 0; e < 16; ++e) o[u][i][e] = 0.f;
    float m[2] = {-1e30f, -1e30f}, lsum[2] = {0.f, 0.f};

    // ILV: each wave's own MFMA and VALU streams interleaved in program order (the counters put
    // MFMA busy + VALU busy ~ the tile time: the two barely overlap). Per tile, four segments:
    // QK(u0) | QK(u1) + softmax(u0) | PV(u0) + softmax(u1) | PV(u1), the MFMA / VALU / LDS-read
    // placement inside the two mixed segments fixed by sched_group_barrier; the masking and the
    // lazy rescale branches sit on the segment boundaries.
    auto qk_u = [&](auto U, const unsigned so, f32x16(&s2)[2]) {
        constexpr int u = decltype(U)::value;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
            f32x16 z;
#pragma unroll
            for (int e = 0; e < 16; ++e) z[e] = 0.f;
#pragma unroll
            for (int ks = 0; ks < NKS; ++ks) {
                const bf16x8 kf = *reinterpret_cast<const LDS_AS bf16x8*>((uintptr_t)(kb0 + so + kb * 512 + ks * 2048));
                z = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[u][ks], z, 0, 0, 0);
            }
            s2[kb] = z;
        }
    };
    auto mask_u = [&](auto U, int t, f32x16(&s2)[2]) {
        constexpr int u = decltype(U)::value;
        if ((t * 64 + 64 > Tk) || (a.causal && t * 64 + 63 > qw0 + 32 * u)) {
            const int q = qw0 + 32 * u + r;
            const int lim = a.causal ? min(Tk, q + 1) : Tk;
#pragma unroll
            for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                for (int e = 0; e < 16; ++e)
                    if (t * 64 + kb * 32 + (e & 3) + 8 * (e >> 2) + 4 * hh >= lim) s2[kb][e] = -INFINITY;
        }
    };
    // max + exp + pack (no branch): returns the new max; the caller rescales O on the boundary
    auto sm_u = [&](auto U, f32x16(&s2)[2], bf16x8(&p4)[4]) {
        constexpr int u = decltype(U)::value;
        float mloc = fmaxf(s2[0][0], s2[0][1]);
#pragma unroll
        for (int e = 2; e < 16; ++e) mloc = fmaxf(mloc, s2[0][e]);
#pragma unroll
        for (int e = 0; e < 16; ++e) mloc = fmaxf(mloc, s2[1][e]);
        mloc = xmax32(mloc);
        const float mnew = fmaxf(m[u], mloc);
        const float mc = mnew * c;
        float psum = 0.f;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const float pv = __builtin_amdgcn_exp2f(__builtin_fmaf(s2[kb][e], c, -mc));
                s2[kb][e] = pv;
                if (!ONES) psum += pv;
            }
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int sp = 0; sp < 2; ++sp)
#pragma unroll
                for (int j = 0; j < 8; ++j) p4[2 * kb + sp][j] = f2bf(s2[kb][8 * sp + j]);
        return make_float2(mnew, psum);
    };
    auto rescale_u = [&](auto U, float2 mp) __attribute__((always_inline)) {
        constexpr int u = decltype(U)::value;
        const float mnew = mp.x;
        if (__builtin_amdgcn_ballot_w64(mnew != m[u])) {
            const float alpha = __builtin_amdgcn_exp2f((m[u] - mnew) * c);
            if (!ONES) lsum[u] *= alpha;
#pragma unroll
            for (int i = 0; i < NDB; ++i) o[u][i] *= alpha;
        }
        m[u] = mnew;
        if (!ONES) lsum[u] += mp.y;
    };
    auto pv_u = [&](auto U, const unsigned so, const bf16x8(&p4)[4]) {
        constexpr int u = decltype(U)::value;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int sp = 0; sp < 2; ++sp)
#pragma unroll
                for (int db = 0; db < NDB; ++db) {
                    const unsigned off = so + db * 4096 + kb * 512 + sp * 256;
                    const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(uintptr_t)(vbj[0] + off));
                    const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(uintptr_t)(vbj[1] + off));
                    const bf16x8 vv = __builtin_bit_cast(bf16x8, __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7));
                    o[u][db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vv, p4[2 * kb + sp], o[u][db], 0, 0, 0);
                }
    };
    auto tile_ilv = [&](int t, const unsigned so) __attribute__((always_inline)) {
        f32x16 s0[2], s1[2];
        bf16x8 p0[4], p1[4];
        qk_u(IC<0>{}, so, s0);
        mask_u(IC<0>{}, t, s0);
        __builtin_amdgcn_sched_barrier(0);
        qk_u(IC<1>{}, so, s1);
        const float2 mp0 = sm_u(IC<0>{}, s0, p0);
#pragma unroll
        for (int i = 0; i < 2 * NKS; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 1);  // K fragment read
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 1);  // QK(u1) MFMA
            __builtin_amdgcn_sched_group_barrier(0x402, 9, 1);  // softmax(u0) VALU / exp
        }
        __builtin_amdgcn_sched_barrier(0);
        rescale_u(IC<0>{}, mp0);
        mask_u(IC<1>{}, t, s1);
        __builtin_amdgcn_sched_barrier(0);
        pv_u(IC<0>{}, so, p0);
        const float2 mp1 = sm_u(IC<1>{}, s1, p1);
#pragma unroll
        for (int i = 0; i < 4 * NDB; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x100, 2, 2);  // V^T transposed reads
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 2);  // PV(u0) MFMA
            __builtin_amdgcn_sched_group_barrier(0x402, 8, 2);  // softmax(u1) VALU / exp
        }
        __builtin_amdgcn_sched_barrier(0);
        rescale_u(IC<1>{}, mp1);
        __builtin_amdgcn_sched_barrier(0);
        pv_u(IC<1>{}, so, p1);
    };

    auto tile_step = [&](int t, const unsigned so) __attribute__((always_inline)) {
        if constexpr (ILV) {
            tile_ilv(t, so);
            return;
        }
        f32x16 sc[2][2];
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
            f32x16 z0, z1;
#pragma unroll
            for (int e = 0; e < 16; ++e) z0[e] = z1[e] = 0.f;
#pragma unroll
            for (int ks = 0; ks < NKS; ++ks) {
                const bf16x8 kf = *reinterpret_cast<const LDS_AS bf16x8*>((uintptr_t)(kb0 + so + kb * 512 + ks * 2048));
                z0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[0][ks], z0, 0, 0, 0);
                z1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[1][ks], z1, 0, 0, 0);
            }
            sc[0][kb] = z0;
            sc[1][kb] = z1;
        }
        if ((t * 64 + 64 > Tk) || (a.causal && t * 64 + 63 > qw0)) {
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int q = qw0 + 32 * u + r;
                const int lim = a.causal ? min(Tk, q + 1) : Tk;
#pragma unroll
                for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                    for (int e = 0; e < 16; ++e)
                        if (t * 64 + kb * 32 + (e & 3) + 8 * (e >> 2) + 4 * hh >= lim) sc[u][kb][e] = -INFINITY;
            }
        }
        bf16x8 pk[2][4];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            float mloc = fmaxf(sc[u][0][0], sc[u][0][1]);
#pragma unroll
            for (int e = 2; e < 16; ++e) mloc = fmaxf(mloc, sc[u][0][e]);
#pragma unroll
            for (int e = 0; e < 16; ++e) mloc = fmaxf(mloc, sc[u][1][e]);
            mloc = xmax32(mloc);
            const float mnew = fmaxf(m[u], mloc);
            if (__builtin_amdgcn_ballot_w64(mnew != m[u])) {
                const float alpha = __builtin_amdgcn_exp2f((m[u] - mnew) * c);
                if (!ONES) lsum[u] *= alpha;
#pragma unroll
                for (int i = 0; i < NDB; ++i) o[u][i] *= alpha;
            }
            m[u] = mnew;
            const float mc = mnew * c;
            float psum = 0.f;
#pragma unroll
            for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                for (int e = 0; e < 16; ++e) {
                    const float pv = __builtin_amdgcn_exp2f(__builtin_fmaf(sc[u][kb][e], c, -mc));
                    sc[u][kb][e] = pv;
                    if (!ONES) psum += pv;
                }
            if (!ONES) lsum[u] += psum;
#pragma unroll
            for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                for (int sp = 0; sp < 2; ++sp)
#pragma unroll
                    for (int j = 0; j < 8; ++j) pk[u][2 * kb + sp][j] = f2bf(sc[u][kb][8 * sp + j]);
        }
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int sp = 0; sp < 2; ++sp)
#pragma unroll
                for (int db = 0; db < NDB; ++db) {
                    const unsigned off = so + db * 4096 + kb * 512 + sp * 256;
                    const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(uintptr_t)(vbj[0] + off));
                    const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(uintptr_t)(vbj[1] + off));
                    const bf16x8 vv = __builtin_bit_cast(bf16x8, __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7));
                    o[0][db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vv, pk[0][2 * kb + sp], o[0][db], 0, 0, 0);
                    o[1][db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vv, pk[1][2 * kb + sp], o[1][db], 0, 0, 0);
                }
    };

    if (PRIO && wave >= NW / 2) __builtin_amdgcn_s_setprio(1);
    if (nkt > 0) issue(0);
    for (int t = 0; t < nkt; t += 2) {
        vm_wait<0>();
        __builtin_amdgcn_s_barrier();
        if (t + 1 < nkt) issue(t + 1);
        tile_step(t, 0);
        if (t + 1 < nkt) {
            vm_wait<0>();
            __builtin_amdgcn_s_barrier();
            if (t + 2 < nkt) issue(t + 2);
            tile_step(t + 1, TILE);
        }
    }

#pragma unroll
    for (int u = 0; u < 2; ++u) {
        float ltot;
        if (ONES) {
            constexpr int DB1 = HD / 32, REG1 = 4 * ((HD % 32) / 8);
            ltot = o[u][DB1][REG1];
        } else {
            ltot = xsum32(lsum[u]);
        }
        const float inv = 1.0f / ltot;
        const int q = qw0 + 32 * u + r;
        bf16* orow = a.out + ((long)b * T + min(q, T - 1)) * a.ldo + h * HD;
#pragma unroll
        for (int db = 0; db < NDB; ++db)
#pragma unroll
            for (int mm = 0; mm < 4; mm += 2) {
                if (32 * db + 8 * mm >= HD) continue;
                bf16x4 v0, v1;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    v0[e] = f2bf(o[u][db][4 * mm + e] * inv);
                    v1[e] = f2bf(o[u][db][4 * mm + 4 + e] * inv);
                }
                const uint2 x = __builtin_bit_cast(uint2, v0), y = __builtin_bit_cast(uint2, v1);
                const auto sx = __builtin_amdgcn_permlane32_swap(x.x, y.x, false, false);
                const auto sy = __builtin_amdgcn_permlane32_swap(x.y, y.y, false, false);
                const int d0 = 32 * db + 8 * (mm + hh);
                if (q < T && d0 + 8 <= HD)
                    *reinterpret_cast<uint4*>(orow + d0) = make_uint4(sx[0], sy[0], sx[1], sy[1]);
            }
    }
}

// ---------------------------------------------------------------------------
// attn_hyb_kernel (head dim 72): QK^T on v_mfma_f32_32x32x16_bf16 (80 deep, as attn_m32_kernel)
// and PV on v_mfma_f32_16x16x32_bf16 (80 output rows: 5 d-tiles of 16, the ones row at d = 72),
// i.e. 160 MFMA rows per 144 useful instead of 176 for either single-shape kernel. The
// hd-72 kernels run against the power cap (profiles/r02_pmc_attn_kind30_vs_m32.json), so
// the MFMA work they skip is what can pay.
//   P layout change: the 32x32 S^T accumulator gives lane (r, h) query r and keys
//   (e & 3) + 8 (e >> 2) + 4 h of a 32-key block (e = 0..15). One v_permlane16_swap per
//   packed register pair (x = e 0..7, y = e 8..15) turns them into the two 16x16x32 B
//   operands: x' (queries 0..15) and y' (queries 16..31), where lane l of 16-lane group
//   g = l >> 4 holds keys base_g + (j & 3) + 8 (j >> 2), base = {0, 16, 4, 20}.
//   V^T operand: two ds_read_b64_tr_b16 per (key block, d-tile) at keys base_g + q and
//   base_g + 8 + q; V plane c stores key k in slot k ^ (4 bit4(k) + 8 (c & 1)), which puts
//   a 32-lane half's reads (2 planes x 2 key runs) on 64 distinct banks.
//   O^T (16x16 tiles): lane l holds query 16 u + (l & 15), rows 4 g + reg of each d-tile;
//   the running max lives with the S^T lanes, so the (lazy) rescale shuffles alpha over.
// ---------------------------------------------------------------------------
// SKIP: 0 none; 1 = a tile whose second 32-key block lies wholly past the keys skips that
// block's MFMAs (round 2's kind 62, now dev kind 63); 2 = the same with literal-zero accumulator
// starts (production kind 62 since round 3).
// DBG (dev kinds 76 / 77, round 4): printf trace of one (batch 1, head 8, query 334) through the
// tile loop -- running max, two O^T elements (d 7, d 22) and the weight sum -- per tile.
// RING (dev kind 78, round 4): LDS slots of the K / V tile ring. 2 = production (tile t + 1's DMA
// issued after tile t's barrier; hipcc drains it with vmcnt(0) before tile t's V^T reads, which it
// cannot prove disjoint from the DMA); 3 = tile t + 2's DMA issued there from inline asm (invisible
// to hipcc), each tile waiting with a counted vmcnt that leaves the next tile's DMA in flight;
// 4 (dev kind 79) = RING 3's DMA with the late wave row's PV one tile behind (stagger, below).
// XT (dev kinds 80-83): VALU trims. 1 = exp2 arguments as packed FMAs (RING 4's qks only; the same
// per-element fma); 2 = rescale O only when some query's max grows by more than 2^8 in the exp2
// domain (P <= 256 otherwise; the weight sums use the same stale max: not bit-identical to kind 62).
// 4 (round 6, with 2; RING 2, hd 72) = the exp2 argument straight out of the QK^T MFMA: Q carries
// the factor c = scale * log2(e) (8: the caller folded it into the Q projection; else multiplied in
// here, one extra bf16 rounding of Q), and Q^T row 72 carries -M, the query's running max in that
// domain held as a bf16 value, against a ones row of K (the hh = 1 lanes of the last k-step read the
// ones plane instead of V plane 0), so the MFMA yields c s - M and the per-element FMA goes. The
// threshold test is lane-local (max of the lane's 32 scores > 8); the first tile always sets M.
template <int HD, int NW, int MINW, bool PRIO, int SKIP = 0, bool DBG = false, int RING = 2, int XT = 0>
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(MINW))) void attn_hyb_kernel(AttnArgs a) {
    static_assert(RING >= 2 && RING <= 4, "two to four ring slots");
    static_assert(HD == 72 || HD == 80, "80-deep QK^T, 80 PV rows");
    constexpr bool ONES = HD == 72;  // hd 72: V^T row 72 = ones (weight sums); hd 80: f32 sums
    constexpr int NCHL = HD / 8;     // K / V planes with data
    constexpr int NKS = 5;           // QK^T k-steps of 16 (80 deep)
    constexpr int NDT = 5;           // PV d-tiles of 16 (80 rows)
    constexpr int NVP = 2 * NDT;     // V planes read: data (+ the ones plane at hd 72)
    constexpr int TILE = (NCHL + NVP) * 1024;
    constexpr int NINS = 2 * NCHL;
    constexpr int MAXI = (NINS + NW - 1) / NW;
    constexpr int QB = NW * 32;
    static_assert(2 * NKS <= NCHL + NVP, "K reads past the head dim stay inside the tile");
    typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
    __shared__ __attribute__((aligned(16))) char lds[RING * TILE];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 31, hh = lane >> 5;
    const int g = lane >> 4, li = lane & 15;
    const int nqb = (a.T + QB - 1) / QB;
    int id;
    {
        const int bid = blockIdx.x, nwg = gridDim.x;
        const int xcd = bid & 7, loc = bid >> 3, q8 = nwg >> 3, r8 = nwg & 7;
        id = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
    }
    const int qb = id % nqb, h = (id / nqb) % a.H, b = id / (nqb * a.H);
    const int T = a.T, D = a.H * HD;
    const bf16* base = a.qkv + (long)b * T * a.ld;
    const int qw0 = qb * QB + wave * 32;
    const int Tk = a.seq_lens ? a.seq_lens[b] : T;
    const float c = a.scale_log2;

    // the ones plane (V plane 9 at hd 72) in every ring slot
    if (ONES)
        for (int i = tid; i < RING * 64; i += NW * 64)
            *reinterpret_cast<u16x8*>(lds + (i >> 6) * TILE + (2 * NCHL) * 1024 + (i & 63) * 16) =
                u16x8{0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80};

    bf16x8 qf[NKS];  // B operand of QK^T: Q^T[d = 16 ks + 8 hh + j][query r]
    {
        const bf16* qrow = base + (long)min(qw0 + r, T - 1) * a.ld + h * HD;
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
            const int col = ks * 16 + 8 * hh;
            if (col < HD)
                qf[ks] = *reinterpret_cast<const bf16x8*>(qrow + col);
            else
                qf[ks] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
            if constexpr ((XT & 4) && !(XT & 8)) {
#pragma unroll
                for (int j = 0; j < 8; ++j) qf[ks][j] = f2bf(bf2f(qf[ks][j]) * c);
            }
        }
    }
    static_assert(!(XT & 4) || (HD == 72 && RING == 2 && (XT & 2)), "the MFMA bias form: hd 72, RING 2, XT 2");
    float mb = 0.f;  // XT 4: the running max M (bf16 value) that Q^T row 72 holds as -M

    int nkt = (Tk + 63) / 64;
    if (a.causal) nkt = min(nkt, (min(T, qb * QB + QB) + 63) / 64);

    auto vslot = [](int key, int plane) { return key ^ (4 * ((key >> 4) & 1) + 8 * (plane & 1)); };
    auto issue = [&](int t, int slot) {
        char* tb = lds + slot * TILE;
#pragma unroll
        for (int i = 0; i < MAXI; ++i) {
            const int idx = wave + NW * i;
            if (i < MAXI - 1 || idx < NINS) {
                const bool isV = idx >= NCHL;
                const int plane = isV ? idx - NCHL : idx;
                const int key = isV ? vslot(lane, plane) : lane;  // slot lane holds this key (involution)
                const bf16* src = base + (long)min(t * 64 + key, T - 1) * a.ld + (isV ? 2 : 1) * D + h * HD + plane * 8;
                if constexpr (RING >= 3)
                    glds16_asm(src, tb + idx * 1024);  // counted by the ring's own waits only
                else
                    glds16(src, tb + idx * 1024);
            }
        }
    };
    // this wave's DMA count per tile (wave-uniform): MAXI, or MAXI - 1 when its last chunk is past NINS
    const bool full_issue = wave + NW * (MAXI - 1) < NINS;

    const unsigned lds0 = (unsigned)(uintptr_t)(LDS_AS char*)lds;
    const unsigned kb0 = lds0 + hh * 1024 + r * 16;  // K fragment: plane 2 ks + hh, key 32 kb + r
    // XT 4: the last k-step's hh = 1 lanes (K dims 72..79) read the ones plane (plane 2 NCHL)
    const unsigned kb4 = kb0 + (NKS - 1) * 2048 + ((XT & 4) ? hh * (2 * NCHL - 2 * NKS + 1) * 1024 : 0);
    auto kaddr = [&](int ks) { return ((XT & 4) && ks == NKS - 1) ? kb4 : kb0 + ks * 2048; };
    unsigned vbj[2];
    {
        const int q = li >> 2, p = li & 3, pc = p >> 1;
        const int bg = 16 * (g & 1) + 4 * (g >> 1);
#pragma unroll
        for (int j = 0; j < 2; ++j)
            vbj[j] = lds0 + (NCHL + pc) * 1024 + vslot(bg + 8 * j + q, pc) * 16 + (p & 1) * 8;
    }

    f32x4 o[2][NDT];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int i = 0; i < NDT; ++i) o[u][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    float m = -1e30f, lsum = 0.f;  // lsum (hd 80): this lane's share of query r's weight sum

    auto tile_step = [&](int t, const unsigned so) __attribute__((always_inline)) {
        // SKIP: a tile whose second 32-key block lies wholly past the keys (the last tile at
        // T = 729) skips that block's QK^T and PV MFMAs; its P is 0 either way (exact: see
        // attn_m32_kernel's SKIP for the rare 1-ulp code-generation differences)
        const bool half = SKIP && t * 64 + 32 >= Tk;
        f32x16 sc[2];
        if (SKIP == 2) {
            // SKIP 2: both QK^T chains start from a literal-zero accumulator (no register init);
            // only the skipped half of the last tile fills its scores with -inf
#pragma unroll
            for (int kb = 0; kb < 2; ++kb) {
                if (kb == 1 && half) {
                    // volatile: hipcc would otherwise hoist these fills into every tile (and let
                    // the MFMAs overwrite them), which is the register init SKIP 2 removes
#pragma unroll
                    for (int e = 0; e < 16; ++e) {
                        float f;
                        asm volatile("v_mov_b32 %0, 0xff800000" : "=v"(f));
                        sc[1][e] = f;
                    }
                } else {
                    f32x16 z = {};
#pragma unroll
                    for (int ks = 0; ks < NKS; ++ks) {
                        const bf16x8 kf =
                            *reinterpret_cast<const LDS_AS bf16x8*>((uintptr_t)(kaddr(ks) + so + kb * 512));
                        z = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[ks], z, 0, 0, 0);
                    }
                    sc[kb] = z;
                }
            }
        } else {
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
            f32x16 z;
#pragma unroll
            for (int e = 0; e < 16; ++e) z[e] = kb == 1 && half ? -INFINITY : 0.f;
            if (kb == 1 && half) {
                sc[kb] = z;
                continue;
            }
#pragma unroll
            for (int ks = 0; ks < NKS; ++ks) {
                const bf16x8 kf = *reinterpret_cast<const LDS_AS bf16x8*>((uintptr_t)(kaddr(ks) + so + kb * 512));
                z = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[ks], z, 0, 0, 0);
            }
            sc[kb] = z;
        }
        }
        if (DBG && b == 1 && h == 8 && qb == 1 && wave == 2 && t == 1 && (lane == 14 || lane == 46))
            for (int kb = 0; kb < 2; ++kb)
                printf("K%d S lane %d kb %d: %a %a %a %a %a %a %a %a %a %a %a %a %a %a %a %a\n", SKIP, lane, kb,
                       sc[kb][0], sc[kb][1], sc[kb][2], sc[kb][3], sc[kb][4], sc[kb][5], sc[kb][6], sc[kb][7],
                       sc[kb][8], sc[kb][9], sc[kb][10], sc[kb][11], sc[kb][12], sc[kb][13], sc[kb][14], sc[kb][15]);
        if ((t * 64 + 64 > Tk) || (a.causal && t * 64 + 63 > qw0)) {
            const int q = qw0 + r;
            const int lim = a.causal ? min(Tk, q + 1) : Tk;
#pragma unroll
            for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                for (int e = 0; e < 16; ++e)
                    if (t * 64 + kb * 32 + (e & 3) + 8 * (e >> 2) + 4 * hh >= lim) sc[kb][e] = -INFINITY;
        }
        float mloc = fmaxf(sc[0][0], sc[0][1]);
#pragma unroll
        for (int e = 2; e < 16; ++e) mloc = fmaxf(mloc, sc[0][e]);
#pragma unroll
        for (int e = 0; e < 16; ++e) mloc = fmaxf(mloc, sc[1][e]);
        if constexpr (XT & 4) {
            // scores are c s - M already; the first tile sets M (O is still zero), later tiles move
            // it only when some lane's score exceeds 8 (P <= 256 otherwise)
            if (t == 0 || __builtin_amdgcn_ballot_w64(mloc > 8.0f)) {
                const float mq = xmax32(mloc);
                const float mn = bf2f(f2bf(mb + (t == 0 ? mq : fmaxf(mq, 0.f))));  // >= mb for t > 0
                const float d = mn - mb;  // exact: both bf16 values
                if (t > 0) {
                    const float alpha = __builtin_amdgcn_exp2f(-d);
#pragma unroll
                    for (int u = 0; u < 2; ++u) {
                        const float au = __shfl(alpha, 16 * u + li, 64);
#pragma unroll
                        for (int i = 0; i < NDT; ++i) o[u][i] *= au;
                    }
                }
#pragma unroll
                for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                    for (int e = 0; e < 16; ++e) sc[kb][e] -= d;
                mb = mn;
                uint4 w = __builtin_bit_cast(uint4, qf[NKS - 1]);
                const unsigned nb = __builtin_bit_cast(unsigned short, f2bf(-mn));
                w.x = hh ? nb : w.x;  // Q^T row 72 (row 73 stays 0)
                qf[NKS - 1] = __builtin_bit_cast(bf16x8, w);
            }
#pragma unroll
            for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                for (int e = 0; e < 16; ++e) sc[kb][e] = __builtin_amdgcn_exp2f(sc[kb][e]);
        } else {
        mloc = xmax32(mloc);
        const float mnew = fmaxf(m, mloc);
        if (__builtin_amdgcn_ballot_w64((XT & 2) ? (mloc - m) * c > 8.0f : mnew != m)) {
            const float alpha = __builtin_amdgcn_exp2f((m - mnew) * c);  // of query r
            if (!ONES) lsum *= alpha;
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const float au = __shfl(alpha, 16 * u + li, 64);  // O^T lanes hold query 16 u + li
#pragma unroll
                for (int i = 0; i < NDT; ++i) o[u][i] *= au;
            }
            if (XT & 2) m = mnew;
        }
        if (!(XT & 2)) m = mnew;
        const float mc = m * c;
        if (DBG && b == 1 && h == 8 && qb == 1 && wave == 2 && t == 1 && (lane == 14 || lane == 46))
            printf("K%d mc lane %d: m %a c %a mc %a\n", SKIP, lane, mnew, c, mc);
        float psum = 0.f;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                sc[kb][e] = __builtin_amdgcn_exp2f(__builtin_fmaf(sc[kb][e], c, -mc));
                if (!ONES) psum += sc[kb][e];
            }
        if (!ONES) lsum += psum;
        }
        if (DBG && b == 1 && h == 8 && qb == 1 && wave == 2 && t == 1 && (lane == 14 || lane == 46))
            for (int kb = 0; kb < 2; ++kb)
                printf("K%d E lane %d kb %d: %a %a %a %a %a %a %a %a %a %a %a %a %a %a %a %a\n", SKIP, lane, kb,
                       sc[kb][0], sc[kb][1], sc[kb][2], sc[kb][3], sc[kb][4], sc[kb][5], sc[kb][6], sc[kb][7],
                       sc[kb][8], sc[kb][9], sc[kb][10], sc[kb][11], sc[kb][12], sc[kb][13], sc[kb][14], sc[kb][15]);
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
            if (kb == 1 && half) break;
            // packed bf16 pairs: x = registers 0..7, y = 8..15 of key block kb
            unsigned xw[4], yw[4];
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                bf16x2_t px = {f2bf(sc[kb][2 * w]), f2bf(sc[kb][2 * w + 1])};
                bf16x2_t py = {f2bf(sc[kb][8 + 2 * w]), f2bf(sc[kb][8 + 2 * w + 1])};
                xw[w] = __builtin_bit_cast(unsigned, px);
                yw[w] = __builtin_bit_cast(unsigned, py);
            }
            unsigned b0w[4], b1w[4];
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                const auto sw = __builtin_amdgcn_permlane16_swap(xw[w], yw[w], false, false);
                b0w[w] = sw[0];  // queries 0..15
                b1w[w] = sw[1];  // queries 16..31
            }
            const bf16x8 pb0 = __builtin_bit_cast(bf16x8, make_uint4(b0w[0], b0w[1], b0w[2], b0w[3]));
            const bf16x8 pb1 = __builtin_bit_cast(bf16x8, make_uint4(b1w[0], b1w[1], b1w[2], b1w[3]));
            if (DBG && b == 1 && h == 8 && qb == 1 && wave == 2 && t == 1 && (lane == 14 || lane == 30 || lane == 46))
                printf("K%d P lane %d kb %d: %08x %08x %08x %08x | %08x %08x %08x %08x\n", SKIP, lane, kb, b0w[0], b0w[1],
                       b0w[2], b0w[3], b1w[0], b1w[1], b1w[2], b1w[3]);
#pragma unroll
            for (int dt = 0; dt < NDT; ++dt) {
                const unsigned off = so + kb * 512 + dt * 2048;
                const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(uintptr_t)(vbj[0] + off));
                const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(uintptr_t)(vbj[1] + off));
                const bf16x8 vv = __builtin_bit_cast(bf16x8, __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7));
                o[0][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vv, pb0, o[0][dt], 0, 0, 0);
                o[1][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vv, pb1, o[1][dt], 0, 0, 0);
            }
        }
    };

    // RING 4 (stagger): tile_step split at the P hand-off. qks(t): QK^T, mask, running max, lazy
    // rescale of O, exp2, P packed into the PV B operands (pq); pvs(t): PV from pq. The early wave
    // row (waves 0 .. NW/2-1) runs qks(t), pvs(t) between two barriers; the late row runs pvs(t - 1),
    // qks(t), so on each SIMD one wave's MFMAs meet the other's softmax VALU. The O updates keep
    // their order (PV(t - 1) before tile t's rescale), so both rows compute kind 62's arithmetic.
    bf16x8 pq[2][2];
    auto qks = [&](int t, const unsigned so) __attribute__((always_inline)) {
        const bool half = SKIP && t * 64 + 32 >= Tk;
        f32x16 sc[2];
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
            if (kb == 1 && half) {
#pragma unroll
                for (int e = 0; e < 16; ++e) {
                    float f;
                    asm volatile("v_mov_b32 %0, 0xff800000" : "=v"(f));
                    sc[1][e] = f;
                }
            } else {
                f32x16 z = {};
#pragma unroll
                for (int ks = 0; ks < NKS; ++ks) {
                    const bf16x8 kf =
                        *reinterpret_cast<const LDS_AS bf16x8*>((uintptr_t)(kaddr(ks) + so + kb * 512));
                    z = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[ks], z, 0, 0, 0);
                }
                sc[kb] = z;
            }
        }
        if ((t * 64 + 64 > Tk) || (a.causal && t * 64 + 63 > qw0)) {
            const int q = qw0 + r;
            const int lim = a.causal ? min(Tk, q + 1) : Tk;
#pragma unroll
            for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                for (int e = 0; e < 16; ++e)
                    if (t * 64 + kb * 32 + (e & 3) + 8 * (e >> 2) + 4 * hh >= lim) sc[kb][e] = -INFINITY;
        }
        float mloc = fmaxf(sc[0][0], sc[0][1]);
#pragma unroll
        for (int e = 2; e < 16; ++e) mloc = fmaxf(mloc, sc[0][e]);
#pragma unroll
        for (int e = 0; e < 16; ++e) mloc = fmaxf(mloc, sc[1][e]);
        mloc = xmax32(mloc);
        const float mnew = fmaxf(m, mloc);
        if (__builtin_amdgcn_ballot_w64((XT & 2) ? (mloc - m) * c > 8.0f : mnew != m)) {
            const float alpha = __builtin_amdgcn_exp2f((m - mnew) * c);
            if (!ONES) lsum *= alpha;
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const float au = __shfl(alpha, 16 * u + li, 64);
#pragma unroll
                for (int i = 0; i < NDT; ++i) o[u][i] *= au;
            }
            m = mnew;
        } else if (!(XT & 2)) {
            m = mnew;
        }
        const float mc = m * c;
        float psum = 0.f;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int e = 0; e < 16; e += 2) {
                if (XT & 1) {
                    const f32x2 x = pk_fma(f32x2{sc[kb][e], sc[kb][e + 1]}, f32x2{c, c}, f32x2{-mc, -mc});
                    sc[kb][e] = __builtin_amdgcn_exp2f(x.x);
                    sc[kb][e + 1] = __builtin_amdgcn_exp2f(x.y);
                } else {
                    sc[kb][e] = __builtin_amdgcn_exp2f(__builtin_fmaf(sc[kb][e], c, -mc));
                    sc[kb][e + 1] = __builtin_amdgcn_exp2f(__builtin_fmaf(sc[kb][e + 1], c, -mc));
                }
                if (!ONES) {
                    psum += sc[kb][e];
                    psum += sc[kb][e + 1];
                }
            }
        if (!ONES) lsum += psum;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
            if (kb == 1 && half) break;
            unsigned xw[4], yw[4];
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                bf16x2_t px = {f2bf(sc[kb][2 * w]), f2bf(sc[kb][2 * w + 1])};
                bf16x2_t py = {f2bf(sc[kb][8 + 2 * w]), f2bf(sc[kb][8 + 2 * w + 1])};
                xw[w] = __builtin_bit_cast(unsigned, px);
                yw[w] = __builtin_bit_cast(unsigned, py);
            }
            unsigned b0w[4], b1w[4];
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                const auto sw = __builtin_amdgcn_permlane16_swap(xw[w], yw[w], false, false);
                b0w[w] = sw[0];
                b1w[w] = sw[1];
            }
            pq[kb][0] = __builtin_bit_cast(bf16x8, make_uint4(b0w[0], b0w[1], b0w[2], b0w[3]));
            pq[kb][1] = __builtin_bit_cast(bf16x8, make_uint4(b1w[0], b1w[1], b1w[2], b1w[3]));
        }
    };
    auto pvs = [&](int t, const unsigned so) __attribute__((always_inline)) {
        const bool half = SKIP && t * 64 + 32 >= Tk;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
            if (kb == 1 && half) break;
#pragma unroll
            for (int dt = 0; dt < NDT; ++dt) {
                const unsigned off = so + kb * 512 + dt * 2048;
                const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(uintptr_t)(vbj[0] + off));
                const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(uintptr_t)(vbj[1] + off));
                const bf16x8 vv = __builtin_bit_cast(bf16x8, __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7));
                o[0][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vv, pq[kb][0], o[0][dt], 0, 0, 0);
                o[1][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vv, pq[kb][1], o[1][dt], 0, 0, 0);
            }
        }
    };

    const bool dbg = DBG && b == 1 && h == 8 && qb == 1 && wave == 2;
    auto trace = [&](int t) {
        if (!dbg) return;
        if (lane == 14) printf("K%d t %2d m %a\n", SKIP, t, m);
        if (lane == 30) printf("K%d t %2d o7 %a o22 %a\n", SKIP, t, o[0][0][3], o[0][1][2]);
        if (lane == 46) printf("K%d t %2d sum %a\n", SKIP, t, o[0][4][0]);
    };
    if (PRIO && wave >= NW / 2) __builtin_amdgcn_s_setprio(1);
    if constexpr (RING == 2) {
        (void)qks;
        (void)pvs;
        if (nkt > 0) issue(0, 0);
        for (int t = 0; t < nkt; t += 2) {
            vm_wait<0>();
            __builtin_amdgcn_s_barrier();
            if (t + 1 < nkt) issue(t + 1, 1);
            tile_step(t, 0);
            if (DBG) trace(t);
            if (t + 1 < nkt) {
                vm_wait<0>();
                __builtin_amdgcn_s_barrier();
                if (t + 2 < nkt) issue(t + 2, 0);
                tile_step(t + 1, TILE);
                if (DBG) trace(t + 1);
            }
        }
    } else if constexpr (RING == 3) {
        // Q landed before the first asm DMA: hipcc cannot count those, so it must not wait on Q later
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) asm volatile("" ::"v"(qf[ks]));
        // tile t sits in slot t % 3; at tile t's barrier every wave is done with tile t - 1, whose
        // slot takes tile t + 2. The wait leaves tile t + 1's DMA (this wave's last issue) in flight.
        if (nkt > 0) issue(0, 0);
        if (nkt > 1) issue(1, 1);
        auto step = [&](int t, int slot) __attribute__((always_inline)) {
            if (t + 1 < nkt) {
                if (full_issue)
                    vm_wait<MAXI>();
                else
                    vm_wait<MAXI - 1>();
            } else {
                vm_wait<0>();
            }
            __builtin_amdgcn_s_barrier();
            if (t + 2 < nkt) issue(t + 2, slot == 0 ? 2 : slot - 1);
            tile_step(t, slot * TILE);
            if (DBG) trace(t);
        };
        for (int t = 0; t < nkt; t += 3) {
            step(t, 0);
            if (t + 1 < nkt) step(t + 1, 1);
            if (t + 2 < nkt) step(t + 2, 2);
        }
    } else {
        // RING 4 (stagger): tile t in slot t % 4. At tile t's barrier the late row still needs tile
        // t - 1 (its PV), so tile t + 2 goes to the slot of tile t - 2.
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) asm volatile("" ::"v"(qf[ks]));
        if (nkt > 0) issue(0, 0);
        if (nkt > 1) issue(1, 1);
        // one straight-line loop per row (a per-step branch on the row made hipcc spill O / P)
        auto loop = [&](auto late_c) __attribute__((always_inline)) {
            constexpr bool LATE = decltype(late_c)::value;
            auto step = [&](int t, int slot) __attribute__((always_inline)) {
                if (t + 1 < nkt) {
                    if (full_issue)
                        vm_wait<MAXI>();
                    else
                        vm_wait<MAXI - 1>();
                } else {
                    vm_wait<0>();
                }
                __builtin_amdgcn_s_barrier();
                if (t + 2 < nkt) issue(t + 2, (slot + 2) & 3);
                if constexpr (LATE) {
                    if (t > 0) pvs(t - 1, ((slot + 3) & 3) * TILE);
                    qks(t, slot * TILE);
                } else {
                    qks(t, slot * TILE);
                    pvs(t, slot * TILE);
                }
            };
            for (int t = 0; t < nkt; t += 4) {
                step(t, 0);
                if (t + 1 < nkt) step(t + 1, 1);
                if (t + 2 < nkt) step(t + 2, 2);
                if (t + 3 < nkt) step(t + 3, 3);
            }
            if (LATE && nkt > 0) pvs(nkt - 1, ((nkt - 1) & 3) * TILE);
        };
        if (wave >= NW / 2)
            loop(std::integral_constant<bool, true>{});
        else
            loop(std::integral_constant<bool, false>{});
    }

    const float lq = ONES ? 0.f : xsum32(lsum);  // hd 80: query r's weight sum (S^T lanes)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        // hd 72: O^T row 72 = d-tile 4, rows 4 g + reg with g = 2, reg = 0: lanes 32..47 hold the
        // sums; hd 80: from the S^T lane of query 16 u + li
        const float ltot = ONES ? __shfl(o[u][NDT - 1][0], 32 + li, 64) : __shfl(lq, 16 * u + li, 64);
        const float inv = 1.0f / ltot;
        const int q = qw0 + 16 * u + li;
        if (q < T) {
            bf16* orow = a.out + ((long)b * T + q) * a.ldo + h * HD;
#pragma unroll
            for (int dt = 0; dt < NDT; ++dt) {
                const int d0 = dt * 16 + 4 * g;
                if (d0 < HD) {
                    bf16x4 v;
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] = f2bf(o[u][dt][e] * inv);
                    *reinterpret_cast<bf16x4*>(orow + d0) = v;
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------
// attn_pp_kernel (round 4, head dim 72): attn_hyb_kernel's arithmetic (kind 62: 32x32x16 QK^T
// 80 deep from literal-zero starts, 16x16x32 PV with the ones row, lazy rescale, last-tile
// skip) in a matrix / vector ping-pong. Every 64-key tile is two phases per wave:
//   M(t): PV(t - 1) (20 MFMAs + 20 transposed V reads) and QK^T(t) (10 MFMAs + 10 K reads);
//   V(t): mask, row max, lazy rescale of O, 32 exp2, bf16 packing into P(t) (VALU only).
// The block's two wave rows (waves 0-3 and 4-7, one of each per SIMD) run one phase apart
// between raw barriers, so on every SIMD one wave's MFMAs meet the other's softmax VALU
// instead of both waves needing the same pipe at once (attn_hyb_kernel's waves all reach
// their QK^T and their softmax together; its counters put MFMA-busy + VALU-busy at the
// kernel time: the pipes take turns). Same per-accumulator MFMA order and the same VALU
// sequence as kind 62, so the outputs are bit-identical to it.
// Ring: 3 slots of K / V chunk planes (tile t in slot t % 3): V(t) is read one phase pair
// after K(t), so tile t + 1, issued when the early row opens M(t), may only overwrite the
// tile read last by the late row's M(t - 1).
// Intervals between barriers: the early row runs M(t) in interval 2t and V(t) in 2t + 1, the
// late row one interval later; each wave issues its pieces of tile t + 1 at the start of
// interval 2t and retires them (vmcnt 0) before the barrier that closes interval 2t + 1.
// PRIO: 0 none, 1 = s_setprio 1 for the late row (static), 2 = s_setprio 1 in every M phase.
// ---------------------------------------------------------------------------
template <int HD, int PRIO, int MINW>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(MINW))) void attn_pp_kernel(AttnArgs a) {
    static_assert(HD == 72, "the ones-row weight sums need V^T row 72 inside the 80-row PV");
    constexpr int NW = 8, QB = NW * 32;
    constexpr int NCHL = HD / 8, NKS = 5, NDT = 5, NVP = 2 * NDT;
    constexpr int TILE = (NCHL + NVP) * 1024, NSLOT = 3;
    constexpr int NINS = 2 * NCHL, MAXI = (NINS + NW - 1) / NW;
    typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
    __shared__ __attribute__((aligned(16))) char lds[NSLOT * TILE];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool late = wave >= NW / 2;
    const int r = lane & 31, hh = lane >> 5;
    const int g = lane >> 4, li = lane & 15;
    const int nqb = (a.T + QB - 1) / QB;
    int id;
    {
        const int bid = blockIdx.x, nwg = gridDim.x;
        const int xcd = bid & 7, loc = bid >> 3, q8 = nwg >> 3, r8 = nwg & 7;
        id = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
    }
    const int qb = id % nqb, h = (id / nqb) % a.H, b = id / (nqb * a.H);
    const int T = a.T, D = a.H * HD;
    const bf16* base = a.qkv + (long)b * T * a.ld;
    const int qw0 = qb * QB + wave * 32;
    const int Tk = a.seq_lens ? a.seq_lens[b] : T;
    const float c = a.scale_log2;

    for (int i = tid; i < NSLOT * 64; i += NW * 64)  // the ones plane in every ring slot
        *reinterpret_cast<u16x8*>(lds + (i >> 6) * TILE + (2 * NCHL) * 1024 + (i & 63) * 16) =
            u16x8{0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80};

    bf16x8 qf[NKS];
    {
        const bf16* qrow = base + (long)min(qw0 + r, T - 1) * a.ld + h * HD;
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
            const int col = ks * 16 + 8 * hh;
            qf[ks] = col < HD ? *reinterpret_cast<const bf16x8*>(qrow + col) : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
        }
    }
    int nkt = (Tk + 63) / 64;
    if (a.causal) nkt = min(nkt, (min(T, qb * QB + QB) + 63) / 64);

    auto vslot = [](int key, int plane) { return key ^ (4 * ((key >> 4) & 1) + 8 * (plane & 1)); };
    auto issue = [&](int t) __attribute__((always_inline)) {
        char* tb = lds + (t % NSLOT) * TILE;
#pragma unroll
        for (int i = 0; i < MAXI; ++i) {
            const int idx = wave + NW * i;
            if (i < MAXI - 1 || idx < NINS) {
                const bool isV = idx >= NCHL;
                const int plane = isV ? idx - NCHL : idx;
                const int key = isV ? vslot(lane, plane) : lane;
                const bf16* src = base + (long)min(t * 64 + key, T - 1) * a.ld + (isV ? 2 : 1) * D + h * HD + plane * 8;
                glds16(src, tb + idx * 1024);
            }
        }
    };

    const unsigned lds0 = (unsigned)(uintptr_t)(LDS_AS char*)lds;
    const unsigned kb0 = lds0 + hh * 1024 + r * 16;
    unsigned vbj[2];
    {
        const int q = li >> 2, p = li & 3, pc = p >> 1;
        const int bg = 16 * (g & 1) + 4 * (g >> 1);
#pragma unroll
        for (int j = 0; j < 2; ++j)
            vbj[j] = lds0 + (NCHL + pc) * 1024 + vslot(bg + 8 * j + q, pc) * 16 + (p & 1) * 8;
    }

    f32x4 o[2][NDT];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int i = 0; i < NDT; ++i) o[u][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    float m = -1e30f;
    f32x16 sc[2];       // S^T of the tile between its M and V phases
    bf16x8 pb[2][2];    // P of the tile between its V phase and the next M phase: [key block][query half]
    bool phalf = false;  // that tile's second key block skipped

    auto barrier = [&]() __attribute__((always_inline)) {
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
    };
    // M phase: PV of the previous tile (slot sp, if any), then QK^T of tile t (slot sk, if any)
    auto mphase = [&](int t, bool pv, bool qk) __attribute__((always_inline)) {
        if (PRIO == 2) __builtin_amdgcn_s_setprio(1);
        if (pv) {
            const unsigned sp = (unsigned)((t - 1) % NSLOT) * TILE;
#pragma unroll
            for (int kb = 0; kb < 2; ++kb) {
                if (kb == 1 && phalf) break;
#pragma unroll
                for (int dt = 0; dt < NDT; ++dt) {
                    const unsigned off = sp + kb * 512 + dt * 2048;
                    const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(uintptr_t)(vbj[0] + off));
                    const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(uintptr_t)(vbj[1] + off));
                    const bf16x8 vv = __builtin_bit_cast(bf16x8, __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7));
                    o[0][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vv, pb[kb][0], o[0][dt], 0, 0, 0);
                    o[1][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vv, pb[kb][1], o[1][dt], 0, 0, 0);
                }
            }
        }
        if (qk) {
            const unsigned so = (unsigned)(t % NSLOT) * TILE;
            const bool half = t * 64 + 32 >= Tk;
#pragma unroll
            for (int kb = 0; kb < 2; ++kb) {
                if (kb == 1 && half) {
#pragma unroll
                    for (int e = 0; e < 16; ++e) {
                        float f;
                        asm volatile("v_mov_b32 %0, 0xff800000" : "=v"(f));
                        sc[1][e] = f;
                    }
                } else {
                    f32x16 z = {};
#pragma unroll
                    for (int ks = 0; ks < NKS; ++ks) {
                        const bf16x8 kf =
                            *reinterpret_cast<const LDS_AS bf16x8*>((uintptr_t)(kb0 + so + kb * 512 + ks * 2048));
                        z = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[ks], z, 0, 0, 0);
                    }
                    sc[kb] = z;
                }
            }
        }
        if (PRIO == 2) __builtin_amdgcn_s_setprio(0);
    };
    // V phase of tile t: mask, max, lazy rescale, exp2, P packing
    auto vphase = [&](int t) __attribute__((always_inline)) {
        if ((t * 64 + 64 > Tk) || (a.causal && t * 64 + 63 > qw0)) {
            const int q = qw0 + r;
            const int lim = a.causal ? min(Tk, q + 1) : Tk;
#pragma unroll
            for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                for (int e = 0; e < 16; ++e)
                    if (t * 64 + kb * 32 + (e & 3) + 8 * (e >> 2) + 4 * hh >= lim) sc[kb][e] = -INFINITY;
        }
        float mloc = fmaxf(sc[0][0], sc[0][1]);
#pragma unroll
        for (int e = 2; e < 16; ++e) mloc = fmaxf(mloc, sc[0][e]);
#pragma unroll
        for (int e = 0; e < 16; ++e) mloc = fmaxf(mloc, sc[1][e]);
        mloc = xmax32(mloc);
        const float mnew = fmaxf(m, mloc);
        if (__builtin_amdgcn_ballot_w64(mnew != m)) {
            const float alpha = __builtin_amdgcn_exp2f((m - mnew) * c);
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const float au = __shfl(alpha, 16 * u + li, 64);
#pragma unroll
                for (int i = 0; i < NDT; ++i) o[u][i] *= au;
            }
        }
        m = mnew;
        const float mc = mnew * c;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int e = 0; e < 16; ++e) sc[kb][e] = __builtin_amdgcn_exp2f(__builtin_fmaf(sc[kb][e], c, -mc));
        phalf = t * 64 + 32 >= Tk;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
            unsigned xw[4], yw[4];
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                bf16x2_t px = {f2bf(sc[kb][2 * w]), f2bf(sc[kb][2 * w + 1])};
                bf16x2_t py = {f2bf(sc[kb][8 + 2 * w]), f2bf(sc[kb][8 + 2 * w + 1])};
                xw[w] = __builtin_bit_cast(unsigned, px);
                yw[w] = __builtin_bit_cast(unsigned, py);
            }
            unsigned b0w[4], b1w[4];
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                const auto sw = __builtin_amdgcn_permlane16_swap(xw[w], yw[w], false, false);
                b0w[w] = sw[0];
                b1w[w] = sw[1];
            }
            pb[kb][0] = __builtin_bit_cast(bf16x8, make_uint4(b0w[0], b0w[1], b0w[2], b0w[3]));
            pb[kb][1] = __builtin_bit_cast(bf16x8, make_uint4(b1w[0], b1w[1], b1w[2], b1w[3]));
        }
    };

    if (PRIO == 1 && late) __builtin_amdgcn_s_setprio(1);
    if (nkt > 0) {
        issue(0);
        vm_wait<0>();
        barrier();
        if (!late) {
            for (int t = 0; t < nkt; ++t) {
                if (t + 1 < nkt) issue(t + 1);  // interval 2t
                mphase(t, t > 0, true);
                barrier();
                vphase(t);  // interval 2t + 1
                vm_wait<0>();
                barrier();
            }
            mphase(nkt, true, false);  // interval 2 nkt
            barrier();
        } else {
            if (nkt > 1) issue(1);  // interval 0
            barrier();
            for (int t = 0; t < nkt; ++t) {
                mphase(t, t > 0, true);  // interval 2t + 1
                vm_wait<0>();
                barrier();
                if (t + 2 < nkt) issue(t + 2);  // interval 2t + 2
                vphase(t);
                barrier();
            }
            mphase(nkt, true, false);  // interval 2 nkt + 1
        }
    }

#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const float ltot = __shfl(o[u][NDT - 1][0], 32 + li, 64);
        const float inv = 1.0f / ltot;
        const int q = qw0 + 16 * u + li;
        if (q < T) {
            bf16* orow = a.out + ((long)b * T + q) * a.ldo + h * HD;
#pragma unroll
            for (int dt = 0; dt < NDT; ++dt) {
                const int d0 = dt * 16 + 4 * g;
                if (d0 < HD) {
                    bf16x4 v;
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] = f2bf(o[u][dt][e] * inv);
                    *reinterpret_cast<bf16x4*>(orow + d0) = v;
                }
            }
        }
    }
}

// SigLIP MAP head: one probe query per head, keys = the T tokens of image b.
constexpr int PROBE_MAXT = 1024;
__global__ __launch_bounds__(256) void probe_attn_kernel(const bf16* __restrict__ qv, const bf16* __restrict__ kv,
                                                         int ld, bf16* __restrict__ out, int ldo, int T, int H,
                                                         int hd, float scale) {
    __shared__ float sc[PROBE_MAXT];
    __shared__ float qs[128];
    __shared__ float red[4][128];
    __shared__ float stat[8];
    // XCD-aware: the H heads of one sequence (which share the 128-B lines of its K / V rows) run
    // on one XCD; with blockIdx = head they were spread over all eight L2s and every line was
    // fetched by two of them (2.7 GB fetched per 239-image launch for 0.8 GB of K / V)
    int id;
    {
        const int bid = blockIdx.x, nwg = gridDim.x;
        const int xcd = bid & 7, loc = bid >> 3, q8 = nwg >> 3, r8 = nwg & 7;
        id = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
    }
    const int h = id % H, b = id / H, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int D = H * hd;
    if (tid < hd) qs[tid] = bf2f(qv[h * hd + tid]);
    __syncthreads();
    const bf16* kb = kv + (long)b * T * ld + h * hd;
    float mx = -INFINITY;
    for (int t = tid; t < T; t += 256) {
        const bf16* kr = kb + (long)t * ld;
        float dot = 0.f;
        for (int d = 0; d < hd; d += 8) {
            const u16x8 u = *reinterpret_cast<const u16x8*>(kr + d);
#pragma unroll
            for (int e = 0; e < 8; ++e) dot += qs[d + e] * bits2f(u[e]);
        }
        const float s = dot * scale;
        sc[t] = s;
        mx = fmaxf(mx, s);
    }
    mx = wave_max(mx);
    if (lane == 0) stat[wave] = mx;
    __syncthreads();
    mx = fmaxf(fmaxf(stat[0], stat[1]), fmaxf(stat[2], stat[3]));
    float sum = 0.f;
    for (int t = tid; t < T; t += 256) {
        const float p = __expf(sc[t] - mx);
        sc[t] = p;
        sum += p;
    }
    sum = wave_sum(sum);
    __syncthreads();
    if (lane == 0) stat[4 + wave] = sum;
    __syncthreads();
    const float inv = 1.f / (stat[4] + stat[5] + stat[6] + stat[7]);
    // weighted V sum: wave w takes keys t = w, w+4, ...; lane holds d = 2*lane, 2*lane+1
    float acc0 = 0.f, acc1 = 0.f;
    const bf16* vb = kb + D;
    const int d = 2 * lane;
    if (d < hd) {
        for (int t = wave; t < T; t += 4) {
            const unsigned u = *reinterpret_cast<const unsigned*>(vb + (long)t * ld + d);
            acc0 += sc[t] * bits2f((unsigned short)(u & 0xffff));
            acc1 += sc[t] * bits2f((unsigned short)(u >> 16));
        }
        red[wave][d] = acc0;
        red[wave][d + 1] = acc1;
    }
    __syncthreads();
    if (tid < hd) {
        const float v = (red[0][tid] + red[1][tid] + red[2][tid] + red[3][tid]) * inv;
        out[(long)b * ldo + h * hd + tid] = f2bf(v);
    }
}

// SigLIP MAP head, one workgroup per image (all H heads; production where H * hd <= 1152,
// H <= 16, T <= PROBE_MAXT). probe_attn_kernel's (image, head) blocks each read their head's
// 144-B slice of every K / V row: the 128-B lines at head boundaries were fetched by two
// blocks, often on two XCDs (2.6x the K / V bytes fetched). Here the image's K rows stream
// through LDS in 16-row tiles by LDS-DMA (a tile = 16 whole 2304-B rows, read once,
// double-buffered), thread (row, head) takes its dot product from LDS (144-B head stride:
// the 16 lanes of a ds_read_b128 group hit 64 distinct banks), and the V rows are read once,
// coalesced (thread = 16-B column chunk). Same math as probe_attn_kernel (fp32 dots, the
// same exp and normalisation); the summation order of the V pass differs (fp32).
constexpr int PROBE2_D = 1152, PROBE2_H = 16;
__global__ __launch_bounds__(256) void probe_attn_img_kernel(const bf16* __restrict__ qv, const bf16* __restrict__ kv,
                                                             int ld, bf16* __restrict__ out, int ldo, int T, int H,
                                                             int hd, float scale) {
    __shared__ __attribute__((aligned(16))) char kt[2][16 * PROBE2_D * 2];
    __shared__ float sc[PROBE2_H * PROBE_MAXT];
    __shared__ float qs[PROBE2_D];
    __shared__ float hinv[PROBE2_H];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int b = blockIdx.x, D = H * hd, TR = 256 / H, CPR = D / 8;  // rows per tile, 16-B chunks per row
    for (int i = tid; i < D; i += 256) qs[i] = bf2f(qv[i]);
    const bf16* kb = kv + (long)b * T * ld;
    const int npiece = TR * CPR / 64, ntile = (T + TR - 1) / TR;
    auto issue = [&](int tile) {
        char* dst = kt[tile & 1];
        for (int pc = wave; pc < npiece; pc += 4) {
            const int g = pc * 64 + lane, row = g / CPR, ch = g % CPR;
            glds16(kb + (long)min(tile * TR + row, T - 1) * ld + ch * 8, dst + pc * 1024);
        }
    };
    issue(0);
    const int r = tid / H, h = tid % H;
    for (int tile = 0; tile < ntile; ++tile) {
        wait_vmcnt0();
        __syncthreads();  // tile landed for every wave; every wave is done with the other slot
        if (tile + 1 < ntile) issue(tile + 1);
        const int t = tile * TR + r;
        if (r < TR && t < T) {
            const char* kr = kt[tile & 1] + (r * D + h * hd) * 2;
            float dot = 0.f;
            for (int d = 0; d < hd; d += 8) {
                const u16x8 u = *reinterpret_cast<const u16x8*>(kr + d * 2);
#pragma unroll
                for (int e = 0; e < 8; ++e) dot += qs[h * hd + d + e] * bits2f(u[e]);
            }
            sc[h * T + t] = dot * scale;
        }
    }
    __syncthreads();
    for (int hh = wave; hh < H; hh += 4) {  // softmax of head hh
        float mx = -INFINITY;
        for (int t = lane; t < T; t += 64) mx = fmaxf(mx, sc[hh * T + t]);
        mx = wave_max(mx);
        float sum = 0.f;
        for (int t = lane; t < T; t += 64) {
            const float p = __expf(sc[hh * T + t] - mx);
            sc[hh * T + t] = p;
            sum += p;
        }
        sum = wave_sum(sum);
        if (lane == 0) hinv[hh] = 1.f / sum;
    }
    __syncthreads();
    if (tid < CPR) {  // V: thread = one 16-B column chunk, every row read once (coalesced rows)
        const bf16* vb = kb + D + tid * 8;
        const int hv = tid * 8 / hd;
        const float* ph = sc + hv * T;
        float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        int t = 0;
        for (; t + 4 <= T; t += 4) {
            u16x8 u[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) u[j] = *reinterpret_cast<const u16x8*>(vb + (long)(t + j) * ld);
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int e = 0; e < 8; ++e) acc[e] += ph[t + j] * bits2f(u[j][e]);
        }
        for (; t < T; ++t) {
            const u16x8 u = *reinterpret_cast<const u16x8*>(vb + (long)t * ld);
#pragma unroll
            for (int e = 0; e < 8; ++e) acc[e] += ph[t] * bits2f(u[e]);
        }
        const float inv = hinv[hv];
        u16x8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = __builtin_bit_cast(unsigned short, f2bf(acc[e] * inv));
        *reinterpret_cast<u16x8*>(out + (long)b * ldo + tid * 8) = o;
    }
}

// ---------------------------------------------------------------------------
// attn_m32p_kernel (round 5, kind 94): attn_m32_kernel's 9-wave, one-block-per-(image, head) form
// (kind 86: SKIP + 2^8 rescale threshold; ViT-H / LAION-CLIP-H, T = 257) as a PERSISTENT loop. Kind 86
// runs only 5 key tiles per block and, at 130 VGPRs (3 waves per SIMD), one 9-wave block fills a CU,
// so every block's Q load and first K / V DMA (~2-4 us of a ~17 us block) are exposed.
// Here one block per CU walks (image, head) units with ONE continuous K / V ring across unit
// boundaries: while the last tile of unit u runs, the next unit's tile 0 is DMA'd into the other ring
// slot and its Q fragments are loaded into a second register set, so the next unit starts on landed
// data. Units are dealt to the XCDs in contiguous ranges (the XCD's 32 blocks work on 2 images' 32
// heads at a time: their rows share L2 lines). Per-tile arithmetic, K order and MFMA chains are kind 86's
// (the ring slot is a runtime offset instead of an unrolled immediate), so the outputs are bit-identical
// to kind 86 (tests/test_gpu_kernels.py::test_attention_persistent_vith_bit_identical).
// Non-causal attention with T <= 32 NW (one query block per unit).
// Measured (round 5): ViT-H in isolation 7 % faster than kind 86 at 455 / 512 images, but 3 % slower
// inside the LAION-CLIP-H job (kernel stats 480 vs 466 us per launch, the jobs level): not dispatched.
// The 9-wave block's bound is its waves' 3 + 2 + 2 + 2 split over the SIMDs (at T = 256 the 8-wave
// kernel at 4 waves per SIMD runs 0.34-0.375 ms against 0.42-0.44 for 9-wave blocks), and the 8-wave
// form of this loop (dev kind 95: 179 VGPRs, 2 waves per SIMD) is slower still (0.47 ms at T = 256).
// ---------------------------------------------------------------------------
template <int HD, int NW, int MINW = 1>
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(MINW))) void attn_m32p_kernel(AttnArgs a,
                                                                                                      int nunits) {
    constexpr int NSTG = 2;
    constexpr bool ONES = HD % 32 != 0;
    constexpr int NCHL = HD / 8;
    constexpr int NKS = (HD + 15) / 16;
    constexpr int NDB = (HD + (ONES ? 1 : 0) + 31) / 32;
    constexpr int NVP = 4 * NDB;
    constexpr int TILE = (NCHL + NVP) * 1024;
    constexpr int NINS = 2 * NCHL;
    constexpr int MAXI = (NINS + NW - 1) / NW;
    static_assert(2 * NKS <= NCHL + NVP, "K reads past the head dim stay inside the tile");
    __shared__ __attribute__((aligned(16))) char lds[NSTG * TILE];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 31, hh = lane >> 5;
    const int T = a.T, D = a.H * HD;
    const float c = a.scale_log2;
    const int qw0 = wave * 32;

    // this block's units: XCD x = blockIdx % 8 owns a contiguous range, its blocks interleave in it
    int u, uend, ustep;
    {
        const int x = blockIdx.x & 7, l = blockIdx.x >> 3, gx = gridDim.x >> 3;
        const int q8 = nunits >> 3, r8 = nunits & 7;
        const int start = x < r8 ? x * (q8 + 1) : r8 * (q8 + 1) + (x - r8) * q8;
        u = start + l;
        uend = start + q8 + (x < r8 ? 1 : 0);
        ustep = gx;
    }
    if (u >= uend) return;  // whole block

    // V planes past the data: the ones plane (ONES) and zero padding, in both ring slots (once)
    constexpr int NPAD = NVP > NCHL ? NVP - NCHL : 1;
    for (int i = tid; i < NSTG * (NVP - NCHL) * 64; i += NW * 64) {
        const int slot = i / (NPAD * 64), rem = i % (NPAD * 64);
        const int pl = NCHL + rem / 64;
        const unsigned short v = (ONES && pl == NCHL) ? 0x3F80 : 0;
        *reinterpret_cast<u16x8*>(lds + slot * TILE + (NCHL + pl) * 1024 + (rem & 63) * 16) =
            u16x8{v, v, v, v, v, v, v, v};
    }

    auto unit_base = [&](int uu) -> const bf16* { return a.qkv + (long)(uu / a.H) * T * a.ld; };
    auto load_q = [&](int uu, bf16x8 (&qd)[NKS]) __attribute__((always_inline)) {
        const bf16* qrow = unit_base(uu) + (long)min(qw0 + r, T - 1) * a.ld + (uu % a.H) * HD;
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
            const int col = ks * 16 + 8 * hh;
            qd[ks] = col < HD ? *reinterpret_cast<const bf16x8*>(qrow + col) : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
        }
    };
    // tile t of unit uu into ring slot `slot`
    auto issue = [&](int uu, int t, int slot) __attribute__((always_inline)) {
        char* tb = lds + slot * TILE;
        const bf16* base = unit_base(uu);
        const int h = uu % a.H;
#pragma unroll
        for (int i = 0; i < MAXI; ++i) {
            const int idx = wave + NW * i;
            if (i < MAXI - 1 || idx < NINS) {
                const bool isV = idx >= NCHL;
                const int plane = isV ? idx - NCHL : idx;
                const int key = isV ? lane ^ (4 * (plane & 3)) : lane;
                const bf16* src = base + (long)min(t * 64 + key, T - 1) * a.ld + (isV ? 2 : 1) * D + h * HD + plane * 8;
                glds16(src, tb + idx * 1024);
            }
        }
    };

    const unsigned lds0 = (unsigned)(uintptr_t)(LDS_AS char*)lds;
    const unsigned kb0 = lds0 + hh * 1024 + r * 16;
    unsigned vbj[2];
    {
        const int i16 = lane & 15, q = i16 >> 2, p = i16 & 3, half = (lane >> 4) & 1;
        const int cc = 2 * half + (p >> 1);
#pragma unroll
        for (int j = 0; j < 2; ++j)
            vbj[j] = lds0 + (NCHL + cc) * 1024 + (((8 * j + 4 * hh + q) ^ (4 * cc)) * 16) + (p & 1) * 8;
    }

    bf16x8 qf[NKS], qn[NKS];
    f32x16 o[NDB];
    float m = -1e30f;
    int Tk = 0;

    // kind 86's tile arithmetic (attn_m32_kernel with SKIP and THR), ring slot at a runtime offset
    auto tile = [&](int t, const unsigned so) __attribute__((always_inline)) {
        const bool half = t * 64 + 32 >= Tk;
        f32x16 sc[2];
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
            f32x16 z;
#pragma unroll
            for (int e = 0; e < 16; ++e) z[e] = kb == 1 && half ? -INFINITY : 0.f;
            if (kb == 1 && half) {
                sc[kb] = z;
                continue;
            }
#pragma unroll
            for (int ks = 0; ks < NKS; ++ks) {
                const bf16x8 kf = *reinterpret_cast<const LDS_AS bf16x8*>((uintptr_t)(kb0 + so + kb * 512 + ks * 2048));
                z = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[ks], z, 0, 0, 0);
            }
            sc[kb] = z;
        }
        if (t * 64 + 64 > Tk) {
#pragma unroll
            for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                for (int e = 0; e < 16; ++e)
                    if (t * 64 + kb * 32 + (e & 3) + 8 * (e >> 2) + 4 * hh >= Tk) sc[kb][e] = -INFINITY;
        }
        float mloc = fmaxf(sc[0][0], sc[0][1]);
#pragma unroll
        for (int e = 2; e < 16; ++e) mloc = fmaxf(mloc, sc[0][e]);
#pragma unroll
        for (int e = 0; e < 16; ++e) mloc = fmaxf(mloc, sc[1][e]);
        mloc = xmax32(mloc);
        const float mnew = fmaxf(m, mloc);
        if (__builtin_amdgcn_ballot_w64((mloc - m) * c > 8.0f)) {
            const float alpha = __builtin_amdgcn_exp2f((m - mnew) * c);
#pragma unroll
            for (int i = 0; i < NDB; ++i) o[i] *= alpha;
            m = mnew;
        }
        const float mc = m * c;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int e = 0; e < 16; ++e) sc[kb][e] = __builtin_amdgcn_exp2f(__builtin_fmaf(sc[kb][e], c, -mc));
        bf16x8 pk[4];
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int sp = 0; sp < 2; ++sp)
#pragma unroll
                for (int j = 0; j < 8; ++j) pk[2 * kb + sp][j] = f2bf(sc[kb][8 * sp + j]);
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
            if (kb == 1 && half) break;
#pragma unroll
            for (int sp = 0; sp < 2; ++sp)
#pragma unroll
                for (int db = 0; db < NDB; ++db) {
                    const unsigned off = so + db * 4096 + kb * 512 + sp * 256;
                    const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(uintptr_t)(vbj[0] + off));
                    const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(uintptr_t)(vbj[1] + off));
                    const bf16x8 vv = __builtin_bit_cast(bf16x8, __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7));
                    o[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vv, pk[2 * kb + sp], o[db], 0, 0, 0);
                }
        }
    };

    if (wave >= NW / 2) __builtin_amdgcn_s_setprio(1);
    load_q(u, qf);
    issue(u, 0, 0);
    int slot = 0;  // ring slot of the unit's current tile (continuous across units)
    while (true) {
        const int b = u / a.H, h = u % a.H;
        Tk = a.seq_lens ? a.seq_lens[b] : T;
        const int nkt = (Tk + 63) / 64;
        const int un = u + ustep;
        const bool more = un < uend;
#pragma unroll
        for (int i = 0; i < NDB; ++i)
#pragma unroll
            for (int e = 0; e < 16; ++e) o[i][e] = 0.f;
        m = -1e30f;
        for (int t = 0; t < nkt; ++t) {
            vm_wait<0>();
            __builtin_amdgcn_s_barrier();
            if (t + 1 < nkt) {
                issue(u, t + 1, slot ^ 1);
            } else if (more) {  // the next unit's tile 0 and Q under this unit's last tile
                issue(un, 0, slot ^ 1);
                load_q(un, qn);
            }
            tile(t, slot ? TILE : 0);
            slot ^= 1;
        }
        // normalise and store (attn_m32_kernel's epilogue)
        {
            constexpr int DB1 = HD / 32, REG1 = 4 * ((HD % 32) / 8);
            static_assert(ONES, "the weight sums come from the ones plane");
            const float inv = 1.0f / o[DB1][REG1];
            const int q = qw0 + r;
            bf16* orow = a.out + ((long)b * T + min(q, T - 1)) * a.ldo + h * HD;
#pragma unroll
            for (int db = 0; db < NDB; ++db)
#pragma unroll
                for (int mm = 0; mm < 4; mm += 2) {
                    if (32 * db + 8 * mm >= HD) continue;
                    bf16x4 v0, v1;
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        v0[e] = f2bf(o[db][4 * mm + e] * inv);
                        v1[e] = f2bf(o[db][4 * mm + 4 + e] * inv);
                    }
                    const uint2 x = __builtin_bit_cast(uint2, v0), y = __builtin_bit_cast(uint2, v1);
                    const auto sx = __builtin_amdgcn_permlane32_swap(x.x, y.x, false, false);
                    const auto sy = __builtin_amdgcn_permlane32_swap(x.y, y.y, false, false);
                    const int d0 = 32 * db + 8 * (mm + hh);
                    if (q < T && d0 + 8 <= HD) *reinterpret_cast<uint4*>(orow + d0) = make_uint4(sx[0], sy[0], sx[1], sy[1]);
                }
        }
        if (!more) break;
        u = un;
        for (int ks = 0; ks < NKS; ++ks) qf[ks] = qn[ks];
    }
}

// attn_m32p_kernel launch: `per_cu` persistent blocks per CU (grid a multiple of 8 for the XCD ranges)
template <int HD, int NW, int MINW>
bool launch_m32p(const AttnArgs& a, int B, int T, int H, int per_cu, hipStream_t st) {
    if constexpr (HD % 32 != 0) {
        if (a.causal || T > 32 * NW) return false;  // one non-causal query block per unit
        const int nunits = B * H;
        int dev = 0, ncu = 256;
        if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
        const int grid = max(8, min(per_cu * (ncu / 8 * 8), (nunits + 7) / 8 * 8));
        hipLaunchKernelGGL((attn_m32p_kernel<HD, NW, MINW>), dim3(grid), dim3(NW * 64), 0, st, a, nunits);
        return true;
    } else {
        return false;
    }
}

template <int HD>
bool launch_attn_dev(int kind, const AttnArgs& a, int B, int T, int H, hipStream_t st);

// Production kinds (chosen by mme_attention's dispatch below); every other kind is a
// development form, built only into the MME_DEV library (make dev -> libmme_dev.so).
template <int HD>
bool launch_attn(int kind, const AttnArgs& a, int B, int T, int H, hipStream_t st) {
    if (kind == 0)
        hipLaunchKernelGGL((attn_fwd_kernel<HD>), dim3(cdiv(T, 128) * H * B), dim3(256), 0, st, a);
    else if (kind == 16)  // T <= 64: one key tile, two (batch, head) units per block
        hipLaunchKernelGGL((attn_short_kernel<HD>), dim3(cdiv(B * H, 2)), dim3(256), 0, st, a, B * H);
    else if (kind == 11)  // lean per-tile VALU, lazy rescale, ones column (HD 72), 8 waves
        hipLaunchKernelGGL((attn_pipe_kernel<HD, 8, 2, false, HD == 72, true>), dim3(cdiv(T, 256) * H * B), dim3(512), 0, st, a);
    else if (kind == 14)  // the same, 4 waves = 128 queries per block
        hipLaunchKernelGGL((attn_pipe_kernel<HD, 4, 2, false, HD == 72, true>), dim3(cdiv(T, 128) * H * B), dim3(256), 0, st, a);
    else if (kind == 23)  // 12 waves = 384 queries per block (hd 80, T = 730: two blocks per batch-head)
        hipLaunchKernelGGL((attn_pipe_kernel<HD, 12, 2, false, HD == 72, true>), dim3(cdiv(T, 384) * H * B), dim3(768), 0, st, a);
    else if (kind == 35)  // 9 waves (288 queries) with static priority for waves 4..8 (T = 257 in one block per
                          // batch-head; +1-4 %, bit-identical; profiles/r02_attn_prio_hd80_ab.log)
        hipLaunchKernelGGL((attn_pipe_kernel<HD, 9, 2, false, HD == 72, true, false, 1, false, 4>),
                           dim3(cdiv(T, 288) * H * B), dim3(576), 0, st, a);
    else if (kind == 38)  // attn_m32_kernel: 8 waves (<= 128 VGPRs uncapped: 4 waves / SIMD), static priority;
                          // production for hd 80 (DFN5B T 730)
        hipLaunchKernelGGL((attn_m32_kernel<HD, 8, 1, true>), dim3(cdiv(T, 256) * H * B), dim3(512), 0, st, a);
    else if (kind == 41)  // attn_m32_kernel, 9 waves (288 queries): production for hd 80 where 9-wave blocks pad least
        hipLaunchKernelGGL((attn_m32_kernel<HD, 9, 1, true>), dim3(cdiv(T, 288) * H * B), dim3(576), 0, st, a);
    else if (kind == 65)  // kind 41 skipping a tile's second key block when it lies past the keys: production
                          // for hd 80 in 9-wave blocks (ViT-H T 257: +2-4 %, profiles/r03_v11_attn_vith_ab.log)
        hipLaunchKernelGGL((attn_m32_kernel<HD, 9, 1, true, false, false, true>), dim3(cdiv(T, 288) * H * B),
                           dim3(576), 0, st, a);
    else if (kind == 58) {  // attn_hyb_kernel without the skip (round 2's production form): the bit-identity
                            // reference of kind 62 (tests/test_gpu_kernels.py::test_attention_skip_bit_identical)
        if constexpr (HD != 64)
            hipLaunchKernelGGL((attn_hyb_kernel<HD, 8, 4, true>), dim3(cdiv(T, 256) * H * B), dim3(512), 0, st, a);
        else
            hipLaunchKernelGGL((attn_m32_kernel<HD, 8, 1, true>), dim3(cdiv(T, 256) * H * B), dim3(512), 0, st, a);
    } else if (kind == 62) {  // attn_hyb_kernel skipping a tile's second key block when it lies past the keys,
                            // literal-zero QK^T starts (since round 3: +0.5-0.7 %, bit-identical,
                            // profiles/r03_v18_attn_bufdma_literal_zero_ab.log): production for hd 72
        if constexpr (HD != 64)
            hipLaunchKernelGGL((attn_hyb_kernel<HD, 8, 4, true, 2>), dim3(cdiv(T, 256) * H * B), dim3(512), 0, st, a);
        else
            hipLaunchKernelGGL((attn_m32_kernel<HD, 8, 1, true>), dim3(cdiv(T, 256) * H * B), dim3(512), 0, st, a);
    } else if (kind == 86)  // kind 65 with the 2^8 rescale threshold: production for hd 80 in 9-wave blocks
        hipLaunchKernelGGL((attn_m32_kernel<HD, 9, 1, true, false, false, true, true>), dim3(cdiv(T, 288) * H * B),
                           dim3(576), 0, st, a);
    else if (kind == 94) {  // kind 86 as a persistent loop over (image, head) units (T <= 288, non-causal; measured,
                            // not dispatched: faster alone, slower in the job -- see the dispatch comment)
        if (!launch_m32p<HD, 9, 1>(a, B, T, H, 1, st)) return false;
    } else if (kind == 87)  // kind 38 with the threshold: production for hd 80 in 8-wave blocks (DFN5B T 730)
        hipLaunchKernelGGL((attn_m32_kernel<HD, 8, 1, true, false, false, false, true>), dim3(cdiv(T, 256) * H * B),
                           dim3(512), 0, st, a);
    else if (kind == 88)  // kind 41 with the threshold: kind 86's no-skip identity reference
        hipLaunchKernelGGL((attn_m32_kernel<HD, 9, 1, true, false, false, false, true>), dim3(cdiv(T, 288) * H * B),
                           dim3(576), 0, st, a);
    else if (kind == 89)  // kind 0 (attn_fwd_kernel) with the 2^8 rescale threshold
        hipLaunchKernelGGL((attn_fwd_kernel<HD, 0, true>), dim3(cdiv(T, 128) * H * B), dim3(256), 0, st, a);
    else if (kind == 83 || kind == 84) {  // kinds 62 / 58 rescaling O only when a query's running max grows
                                            // by more than 2^8 in the exp2 domain (XT 2): production for hd 72
                                            // since round 4 (kind 83; 84 = its no-skip identity reference)
        if constexpr (HD != 64) {
            if (kind == 83)
                hipLaunchKernelGGL((attn_hyb_kernel<HD, 8, 4, true, 2, false, 2, 2>), dim3(cdiv(T, 256) * H * B),
                                   dim3(512), 0, st, a);
            else
                hipLaunchKernelGGL((attn_hyb_kernel<HD, 8, 4, true, 0, false, 2, 2>), dim3(cdiv(T, 256) * H * B),
                                   dim3(512), 0, st, a);
        } else {
            hipLaunchKernelGGL((attn_m32_kernel<HD, 8, 1, true>), dim3(cdiv(T, 256) * H * B), dim3(512), 0, st, a);
        }
    } else if (kind == 99 || kind == 100 || kind == 101) {  // attn_m32_kernel with the exp2 argument from the
                                                         // MFMA (BIAS; Q pre-scaled, mme_attention_qs only):
                                                         // 99 / 100 = kind 87 (8 waves), 101 = kind 86 (9 waves, skip)
        if constexpr (HD == 64)
            return false;
        else if (kind == 101)
            hipLaunchKernelGGL((attn_m32_kernel<HD, 9, 1, true, false, false, true, true, true>),
                               dim3(cdiv(T, 288) * H * B), dim3(576), 0, st, a);
        else
            hipLaunchKernelGGL((attn_m32_kernel<HD, 8, 1, true, false, false, false, true, true>),
                               dim3(cdiv(T, 256) * H * B), dim3(512), 0, st, a);
    } else if (kind == 97 || kind == 98) {  // kind 83 with the exp2 argument from the MFMA (XT 4): 97 scales Q
                                            // here (one more bf16 rounding of Q), 98 takes Q pre-scaled
                                            // (mme_attention_qs: production for hd 72 since round 6)
        if constexpr (HD != 72)
            return false;
        else if (kind == 97)
            hipLaunchKernelGGL((attn_hyb_kernel<HD, 8, 4, true, 2, false, 2, 6>), dim3(cdiv(T, 256) * H * B),
                               dim3(512), 0, st, a);
        else
            hipLaunchKernelGGL((attn_hyb_kernel<HD, 8, 4, true, 2, false, 2, 14>), dim3(cdiv(T, 256) * H * B),
                               dim3(512), 0, st, a);
    } else if (kind == 102) {  // T <= 128 at head dim 64 (CLIP causal text): one burst of loads per unit
        if constexpr (HD != 64)
            return false;
        else
            hipLaunchKernelGGL((attn_short2_kernel<HD>), dim3(B * H), dim3(256), 0, st, a, B * H);
    } else
        return launch_attn_dev<HD>(kind, a, B, T, H, st);
    return true;
}

#ifdef MME_DEV
// Development and diagnostic forms (tools/attn_bench.py, tests marked `dev`).
template <int HD>
bool launch_attn_dev(int kind, const AttnArgs& a, int B, int T, int H, hipStream_t st) {
    if (kind == 19)  // dev: short kernel, compact K pitch (4 blocks per CU): no gain, HBM-bound (0.138 / 0.136 ms)
        hipLaunchKernelGGL((attn_short_kernel<HD, true>), dim3(cdiv(B * H, 2)), dim3(256), 0, st, a, B * H);
    else if (kind == 95) {  // dev: kind 94 in 8-wave blocks (T <= 256), one per CU
        if (!launch_m32p<HD, 8, 1>(a, B, T, H, 1, st)) return false;
    } else if (kind == 96) {  // dev: kind 94 in 8-wave blocks held to 128 VGPRs, two per CU
        if (!launch_m32p<HD, 8, 4>(a, B, T, H, 2, st)) return false;
    } else if (kind == 66) {  // dev: short kernel as a persistent loop with the next pair's loads in flight
        const int npairs = cdiv(B * H, 2);
        hipLaunchKernelGGL((attn_short_pf_kernel<HD>), dim3(min(npairs, 256 * 2)), dim3(256), 0, st, a, B * H, npairs);
    }
    else if (kind == 1)
        hipLaunchKernelGGL((attn_dma_kernel<HD, 4, 2>), dim3(cdiv(T, 128) * H * B), dim3(256), 0, st, a);
    else if (kind == 3)
        hipLaunchKernelGGL((attn_dma_kernel<HD, 2, 2>), dim3(cdiv(T, 64) * H * B), dim3(128), 0, st, a);
    else if (kind == 4)
        hipLaunchKernelGGL((attn_dma_kernel<HD, 8, 3>), dim3(cdiv(T, 256) * H * B), dim3(512), 0, st, a);
    else if (kind == 5)
        hipLaunchKernelGGL((attn_dma_kernel<HD, 4, 3>), dim3(cdiv(T, 128) * H * B), dim3(256), 0, st, a);
    else if (kind == 6)  // dev: 8 waves, register budget for 4 waves / SIMD (2 blocks per CU)
        hipLaunchKernelGGL((attn_dma_kernel<HD, 8, 2, 0, 4>), dim3(cdiv(T, 256) * H * B), dim3(512), 0, st, a);
    else if (kind == 7)  // dev: 4 waves, 4 waves / SIMD
        hipLaunchKernelGGL((attn_dma_kernel<HD, 4, 2, 0, 4>), dim3(cdiv(T, 128) * H * B), dim3(256), 0, st, a);
    else if (kind == 8)  // dev: pipelined QK(t+1) under softmax(t)
        hipLaunchKernelGGL((attn_pipe_kernel<HD, 8, 3, true, false, false>), dim3(cdiv(T, 256) * H * B), dim3(512), 0, st, a);
    else if (kind == 9)  // dev: lean per-tile VALU (lane-base addresses, permlane reductions)
        hipLaunchKernelGGL((attn_pipe_kernel<HD, 8, 2, false, false, false>), dim3(cdiv(T, 256) * H * B), dim3(512), 0, st, a);
    else if (kind == 10)  // dev: + lazy rescale
        hipLaunchKernelGGL((attn_pipe_kernel<HD, 8, 2, false, false, true>), dim3(cdiv(T, 256) * H * B), dim3(512), 0, st, a);
    else if (kind == 13)  // dev: lean + lazy (+ ones), 2 waves = 64 queries per block (text towers)
        hipLaunchKernelGGL((attn_pipe_kernel<HD, 2, 2, false, HD == 72, true>), dim3(cdiv(T, 64) * H * B), dim3(128), 0, st, a);
    else if (kind == 15)  // dev: ping-pong halves (8 waves), lean + lazy (+ ones)
        hipLaunchKernelGGL((attn_pipe_kernel<HD, 8, 4, false, HD == 72, true, true>), dim3(cdiv(T, 256) * H * B), dim3(512), 0, st, a);
    else if (kind == 17)  // dev: kind 11 held to 128 VGPRs -> two 8-wave blocks per CU (4 waves / SIMD)
        hipLaunchKernelGGL((attn_pipe_kernel<HD, 8, 2, false, HD == 72, true, false, 4>), dim3(cdiv(T, 256) * H * B), dim3(512), 0, st, a);
    else if (kind == 18)  // dev: kind 14 held to 128 VGPRs (4-wave blocks, 4 per CU)
        hipLaunchKernelGGL((attn_pipe_kernel<HD, 4, 2, false, HD == 72, true, false, 4>), dim3(cdiv(T, 128) * H * B), dim3(256), 0, st, a);
    else if (kind == 20)  // dev: 3 waves = 96 queries per block (T = 257: 288 padded rows): 0.337 ms, no gain
        hipLaunchKernelGGL((attn_pipe_kernel<HD, 3, 2, false, HD == 72, true>), dim3(cdiv(T, 96) * H * B), dim3(192), 0, st, a);
    else if (kind == 21)  // 9 waves = 288 queries per block (T = 257 in one block per batch-head)
        hipLaunchKernelGGL((attn_pipe_kernel<HD, 9, 2, false, HD == 72, true>), dim3(cdiv(T, 288) * H * B), dim3(576), 0, st, a);
    else if (kind == 24)  // dev: 12 waves, 3 waves / SIMD register budget (hd 72 T 729: 1.033 ms vs 1.03-1.07, noise)
        hipLaunchKernelGGL((attn_pipe_kernel<HD, 12, 2, false, HD == 72, true, false, 3>), dim3(cdiv(T, 384) * H * B), dim3(768), 0, st, a);
    else if (kind == 25)  // dev: 12 waves, 3-stage ring (slower: LDS occupancy)
        hipLaunchKernelGGL((attn_pipe_kernel<HD, 12, 3, false, HD == 72, true>), dim3(cdiv(T, 384) * H * B), dim3(768), 0, st, a);
    else if (kind == 26)  // dev: 9 waves, 3-stage ring
        hipLaunchKernelGGL((attn_pipe_kernel<HD, 9, 3, false, HD == 72, true>), dim3(cdiv(T, 288) * H * B), dim3(576), 0, st, a);
    else if (kind == 22)  // dev: 5 waves = 160 queries per block
        hipLaunchKernelGGL((attn_pipe_kernel<HD, 5, 2, false, HD == 72, true>), dim3(cdiv(T, 160) * H * B), dim3(320), 0, st, a);
    else if (kind == 27)  // kind 17 unrolled by the ring depth (compile-time ring slots)
        hipLaunchKernelGGL((attn_pipe_kernel<HD, 8, 2, false, HD == 72, true, false, 4, true>), dim3(cdiv(T, 256) * H * B),
                           dim3(512), 0, st, a);
    else if (kind == 28)  // kind 27 with the K/V DMA issued from inline asm (no compiler vmcnt(0) before LDS reads)
        hipLaunchKernelGGL((attn_pipe_kernel<HD, 8, 2, false, HD == 72, true, false, 4, true, 1>),
                           dim3(cdiv(T, 256) * H * B), dim3(512), 0, st, a);
    else if (kind == 29)  // dev: kind 27 with packed exp-argument FMAs
        hipLaunchKernelGGL((attn_pipe_kernel<HD, 8, 2, false, HD == 72, true, false, 4, true, 2>),
                           dim3(cdiv(T, 256) * H * B), dim3(512), 0, st, a);
    else if (kind == 30)  // kind 27 with static priority (s_setprio 1) for waves NW/2..: production for hd 72,
                          // +1-2 % per launch, bit-identical (profiles/r02_attn_wide_prio_ab.log)
        hipLaunchKernelGGL((attn_pipe_kernel<HD, 8, 2, false, HD == 72, true, false, 4, true, 4>),
                           dim3(cdiv(T, 256) * H * B), dim3(512), 0, st, a);
    else if (kind == 32)  // diagnostic: kind 27 with only the first K/V tile staged (wrong results)
        hipLaunchKernelGGL((attn_pipe_kernel<HD, 8, 2, false, HD == 72, true, false, 4, true, 8>),
                           dim3(cdiv(T, 256) * H * B), dim3(512), 0, st, a);
    else if (kind == 33)  // dev: kind 27 with 16-B O stores (slower: 615 vs 630-650 TF/s)
        hipLaunchKernelGGL((attn_pipe_kernel<HD, 8, 2, false, HD == 72, true, false, 4, true, 16>),
                           dim3(cdiv(T, 256) * H * B), dim3(512), 0, st, a);
    else if (kind == 34)  // dev: kind 27 with 16-B O stores + static priority
        hipLaunchKernelGGL((attn_pipe_kernel<HD, 8, 2, false, HD == 72, true, false, 4, true, 20>),
                           dim3(cdiv(T, 256) * H * B), dim3(512), 0, st, a);
    else if (kind == 36)  // dev: kind 23 (12 waves) with static priority (DFN5B T 730: within noise)
        hipLaunchKernelGGL((attn_pipe_kernel<HD, 12, 2, false, HD == 72, true, false, 1, false, 4>),
                           dim3(cdiv(T, 384) * H * B), dim3(768), 0, st, a);
    else if (kind == 37)  // dev: kind 30 with a 4-tile ring and one barrier per pair of key tiles
        hipLaunchKernelGGL((attn_pipe_kernel<HD, 8, 4, false, HD == 72, true, false, 4, true, 36>),
                           dim3(cdiv(T, 256) * H * B), dim3(512), 0, st, a);
    else if (kind == 31)  // dev: both
        hipLaunchKernelGGL((attn_pipe_kernel<HD, 8, 2, false, HD == 72, true, false, 4, true, 6>),
                           dim3(cdiv(T, 256) * H * B), dim3(512), 0, st, a);
    else if (kind == 39)  // dev: attn_m32_kernel, 12 waves (384 queries), 3 waves / SIMD
        hipLaunchKernelGGL((attn_m32_kernel<HD, 12, 3, true>), dim3(cdiv(T, 384) * H * B), dim3(768), 0, st, a);
    else if (kind == 40)  // dev: attn_m32_kernel, 8 waves, amdgpu_waves_per_eu(4) (spills 8 registers)
        hipLaunchKernelGGL((attn_m32_kernel<HD, 8, 4, true>), dim3(cdiv(T, 256) * H * B), dim3(512), 0, st, a);
    else if (kind == 42)  // dev: attn_m32_kernel, 8 waves, no static priority
        hipLaunchKernelGGL((attn_m32_kernel<HD, 8, 1, false>), dim3(cdiv(T, 256) * H * B), dim3(512), 0, st, a);
    else if (kind == 43)  // dev: attn_m32_kernel with delayed PV (3-slot ring), 8 waves
        hipLaunchKernelGGL((attn_m32_kernel<HD, 8, 1, true, true>), dim3(cdiv(T, 256) * H * B), dim3(512), 0, st, a);
    else if (kind == 44)  // dev: delayed PV, 8 waves, amdgpu_waves_per_eu(4)
        hipLaunchKernelGGL((attn_m32_kernel<HD, 8, 4, true, true>), dim3(cdiv(T, 256) * H * B), dim3(512), 0, st, a);
    else if (kind == 45)  // dev: delayed PV, 12 waves
        hipLaunchKernelGGL((attn_m32_kernel<HD, 12, 1, true, true>), dim3(cdiv(T, 384) * H * B), dim3(768), 0, st, a);
    else if (kind == 46)  // dev: delayed PV, 9 waves
        hipLaunchKernelGGL((attn_m32_kernel<HD, 9, 1, true, true>), dim3(cdiv(T, 288) * H * B), dim3(576), 0, st, a);
    else if (kind == 47)  // dev: attn_m32x2_kernel (64 queries per wave), 4 waves = 256 queries per block
        hipLaunchKernelGGL((attn_m32x2_kernel<HD, 4, true>), dim3(cdiv(T, 256) * H * B), dim3(256), 0, st, a);
    else if (kind == 48)  // dev: attn_m32x2_kernel, no static priority
        hipLaunchKernelGGL((attn_m32x2_kernel<HD, 4, false>), dim3(cdiv(T, 256) * H * B), dim3(256), 0, st, a);
    else if (kind == 49)  // dev: attn_m32x2_kernel, 6 waves = 384 queries per block
        hipLaunchKernelGGL((attn_m32x2_kernel<HD, 6, true>), dim3(cdiv(T, 384) * H * B), dim3(384), 0, st, a);
    else if (kind == 50)  // dev: attn_m32x2_kernel, 8 waves = 512 queries per block
        hipLaunchKernelGGL((attn_m32x2_kernel<HD, 8, true>), dim3(cdiv(T, 512) * H * B), dim3(512), 0, st, a);
    else if (kind == 51)  // dev: attn_m32x2_kernel, MFMA / VALU interleaved per wave (sched_group_barrier)
        hipLaunchKernelGGL((attn_m32x2_kernel<HD, 4, true, true>), dim3(cdiv(T, 256) * H * B), dim3(256), 0, st, a);
    else if (kind == 52)  // dev: kind 51 without static priority
        hipLaunchKernelGGL((attn_m32x2_kernel<HD, 4, false, true>), dim3(cdiv(T, 256) * H * B), dim3(256), 0, st, a);
    else if (kind == 54)  // dev: attn_m32_kernel with fragment prefetch (PF), 8 waves, <= 256 VGPRs
        hipLaunchKernelGGL((attn_m32_kernel<HD, 8, 2, true, false, true>), dim3(cdiv(T, 256) * H * B), dim3(512), 0, st, a);
    else if (kind == 55)  // dev: PF, 12 waves, 3 waves / SIMD
        hipLaunchKernelGGL((attn_m32_kernel<HD, 12, 3, true, false, true>), dim3(cdiv(T, 384) * H * B), dim3(768), 0, st, a);
    else if (kind == 56)  // dev: PF, 8 waves, 4 waves / SIMD cap
        hipLaunchKernelGGL((attn_m32_kernel<HD, 8, 4, true, false, true>), dim3(cdiv(T, 256) * H * B), dim3(512), 0, st, a);
    else if (kind == 57)  // dev: PF, 9 waves, 3 waves / SIMD
        hipLaunchKernelGGL((attn_m32_kernel<HD, 9, 3, true, false, true>), dim3(cdiv(T, 288) * H * B), dim3(576), 0, st, a);
    else if (kind == 59 || kind == 60 || kind == 61) {  // attn_hyb_kernel (hd 72 / 80; hd 64: kind 38);
                                                        // kind 58 (production launch_attn) is the 8-wave, 4 waves / SIMD form
        if constexpr (HD != 64) {
            if (kind == 59)  // 12 waves, 3 waves / SIMD
                hipLaunchKernelGGL((attn_hyb_kernel<HD, 12, 1, true>), dim3(cdiv(T, 384) * H * B), dim3(768), 0, st, a);
            else if (kind == 60)  // 8 waves, no register cap (129 VGPRs: 3 waves / SIMD)
                hipLaunchKernelGGL((attn_hyb_kernel<HD, 8, 1, true>), dim3(cdiv(T, 256) * H * B), dim3(512), 0, st, a);
            else  // 9 waves (288 queries: T = 257 in one block per batch-head)
                hipLaunchKernelGGL((attn_hyb_kernel<HD, 9, 1, true>), dim3(cdiv(T, 288) * H * B), dim3(576), 0, st, a);
        } else {
            hipLaunchKernelGGL((attn_m32_kernel<HD, 8, 1, true>), dim3(cdiv(T, 256) * H * B), dim3(512), 0, st, a);
        }
    } else if (kind == 64) {  // dev: kind 38 (8-wave attn_m32_kernel) with the last-tile skip (round 3: 18 % slower
                              // at DFN5B T 730; the pair whose rare 1-ulp difference round 3 recorded)
        hipLaunchKernelGGL((attn_m32_kernel<HD, 8, 1, true, false, false, true>), dim3(cdiv(T, 256) * H * B), dim3(512),
                           0, st, a);
    } else if (kind == 76 || kind == 77) {  // dev: kinds 58 / 62 with the printf trace (DBG)
        if constexpr (HD == 72) {
            if (kind == 76)
                hipLaunchKernelGGL((attn_hyb_kernel<HD, 8, 4, true, 0, true>), dim3(cdiv(T, 256) * H * B), dim3(512), 0, st, a);
            else
                hipLaunchKernelGGL((attn_hyb_kernel<HD, 8, 4, true, 2, true>), dim3(cdiv(T, 256) * H * B), dim3(512), 0, st, a);
        } else {
            return false;
        }
    } else if (kind == 78) {  // dev: kind 62 on a three-slot K / V ring (tile t + 2's DMA issued at tile t)
        if constexpr (HD != 64)
            hipLaunchKernelGGL((attn_hyb_kernel<HD, 8, 4, true, 2, false, 3>), dim3(cdiv(T, 256) * H * B), dim3(512), 0,
                               st, a);
        else  // hd 64: kind 38's kernel, as the other hyb kinds
            hipLaunchKernelGGL((attn_m32_kernel<HD, 8, 1, true>), dim3(cdiv(T, 256) * H * B), dim3(512), 0, st, a);
    } else if (kind == 79) {  // dev: kind 62 staggered (RING 4): the late wave row runs PV one tile behind
        if constexpr (HD != 64)
            hipLaunchKernelGGL((attn_hyb_kernel<HD, 8, 4, true, 2, false, 4>), dim3(cdiv(T, 256) * H * B), dim3(512), 0,
                               st, a);
        else
            hipLaunchKernelGGL((attn_m32_kernel<HD, 8, 1, true>), dim3(cdiv(T, 256) * H * B), dim3(512), 0, st, a);
    } else if (kind == 80 || kind == 81) {  // dev: kind 79 with qks VALU trims (80: packed exp arguments +
                                            // 2^8 rescale threshold; 81: packed exp arguments only)
        if constexpr (HD != 64) {
            if (kind == 80)
                hipLaunchKernelGGL((attn_hyb_kernel<HD, 8, 4, true, 2, false, 4, 3>), dim3(cdiv(T, 256) * H * B),
                                   dim3(512), 0, st, a);
            else
                hipLaunchKernelGGL((attn_hyb_kernel<HD, 8, 4, true, 2, false, 4, 1>), dim3(cdiv(T, 256) * H * B),
                                   dim3(512), 0, st, a);
        } else {
            hipLaunchKernelGGL((attn_m32_kernel<HD, 8, 1, true>), dim3(cdiv(T, 256) * H * B), dim3(512), 0, st, a);
        }
    } else if (kind >= 91 && kind <= 93) {  // dev: kind 86 in 5-wave (160-query; 93: <= 128 VGPRs) / 4-wave
                                            // blocks: more, smaller blocks per CU to overlap the prologues at
                                            // T 257 (ViT-H)
        if (kind == 91)
            hipLaunchKernelGGL((attn_m32_kernel<HD, 5, 1, true, false, false, true, true>), dim3(cdiv(T, 160) * H * B),
                               dim3(320), 0, st, a);
        else if (kind == 93)  // 5-wave blocks held to 128 VGPRs: three blocks per CU
            hipLaunchKernelGGL((attn_m32_kernel<HD, 5, 4, true, false, false, true, true>), dim3(cdiv(T, 160) * H * B),
                               dim3(320), 0, st, a);
        else
            hipLaunchKernelGGL((attn_m32_kernel<HD, 4, 1, true, false, false, true, true>), dim3(cdiv(T, 128) * H * B),
                               dim3(256), 0, st, a);
    } else if (kind == 82) {  // dev: the 2^8 rescale threshold on kind 79's stagger
        if constexpr (HD != 64) {
            hipLaunchKernelGGL((attn_hyb_kernel<HD, 8, 4, true, 2, false, 4, 2>), dim3(cdiv(T, 256) * H * B),
                               dim3(512), 0, st, a);
        } else {
            hipLaunchKernelGGL((attn_m32_kernel<HD, 8, 1, true>), dim3(cdiv(T, 256) * H * B), dim3(512), 0, st, a);
        }
    } else if (kind == 63) {  // dev: kind 62 as in round 2 (the skipped block's fill and the accumulator
                              // init as per-tile register moves)
        if constexpr (HD != 64)
            hipLaunchKernelGGL((attn_hyb_kernel<HD, 8, 4, true, 1>), dim3(cdiv(T, 256) * H * B), dim3(512), 0, st, a);
        else
            hipLaunchKernelGGL((attn_m32_kernel<HD, 8, 1, true>), dim3(cdiv(T, 256) * H * B), dim3(512), 0, st, a);
    } else if (kind >= 70 && kind <= 72) {  // dev: attn_pp_kernel (hd 72), PRIO = kind - 70, 2 waves per SIMD
                                            // (155 VGPRs; a 128-VGPR cap spills 16)
        if constexpr (HD == 72) {
            const dim3 grid(cdiv(T, 256) * H * B), blk(512);
            if (kind == 70)
                hipLaunchKernelGGL((attn_pp_kernel<HD, 0, 2>), grid, blk, 0, st, a);
            else if (kind == 71)
                hipLaunchKernelGGL((attn_pp_kernel<HD, 1, 2>), grid, blk, 0, st, a);
            else
                hipLaunchKernelGGL((attn_pp_kernel<HD, 2, 2>), grid, blk, 0, st, a);
        } else {
            return false;
        }
    } else if (kind == 12)  // dev: pipelined + lazy + ones
        hipLaunchKernelGGL((attn_pipe_kernel<HD, 8, 3, true, HD == 72, true>), dim3(cdiv(T, 256) * H * B), dim3(512), 0, st, a);
    else if (kind == 2)
        hipLaunchKernelGGL((attn_dma_kernel<HD, 8, 2>), dim3(cdiv(T, 256) * H * B), dim3(512), 0, st, a);
    else
        return false;
    return true;
}
#else
template <int HD>
bool launch_attn_dev(int, const AttnArgs&, int, int, int, hipStream_t) {
    return false;  // development kinds live in the MME_DEV build only
}
#endif

// Kernel form per call (mme_attention_form): 0 = the production dispatch, 30 + kind = force kernel
// kind `kind` (the kinds compiled into this library; the bit-identity references of the tests).
// The development build keeps a process-wide default for the plain entry points
// (mme_attention_variant: tools/attn_bench.py, plus its diagnostic forms 1-4, 21-26, 200).
#ifdef MME_DEV
int g_attn_variant = 0;
inline int attn_default_form() { return g_attn_variant; }
#else
inline int attn_default_form() { return 0; }
#endif

int attention_entry(int form, const void* qkv, int ld_qkv, void* out, int ld_out, int B, int T, int H, int hd,
                    const int32_t* seq_lens, int causal, float scale, bool qs, void* stream);
}  // namespace

#ifdef MME_DEV
extern "C" int mme_attention_variant(int v) {  // development build only
    g_attn_variant = v;
    return MME_OK;
}
#endif

extern "C" int mme_attention(const void* qkv, int ld_qkv, void* out, int ld_out, int B, int T, int H, int hd,
                             const int32_t* seq_lens, int causal, float scale, void* stream) {
    return attention_entry(attn_default_form(), qkv, ld_qkv, out, ld_out, B, T, H, hd, seq_lens, causal, scale, false,
                           stream);
}

extern "C" int mme_attention_form(int form, const void* qkv, int ld_qkv, void* out, int ld_out, int B, int T, int H,
                                  int hd, const int32_t* seq_lens, int causal, float scale, void* stream) {
    MME_REQUIRE(form == 0 || (form >= 30 && form <= 199), "mme_attention_form: form %d (0 or 30 + kind)", form);
    return attention_entry(form, qkv, ld_qkv, out, ld_out, B, T, H, hd, seq_lens, causal, scale, false, stream);
}

extern "C" int mme_attention_qs(const void* qkv, int ld_qkv, void* out, int ld_out, int B, int T, int H, int hd,
                                const int32_t* seq_lens, int causal, void* stream) {
    return attention_entry(attn_default_form(), qkv, ld_qkv, out, ld_out, B, T, H, hd, seq_lens, causal, 0.f, true,
                           stream);
}

extern "C" int mme_attention_qs_form(int form, const void* qkv, int ld_qkv, void* out, int ld_out, int B, int T,
                                     int H, int hd, const int32_t* seq_lens, int causal, void* stream) {
    MME_REQUIRE(form == 0 || (form >= 30 && form <= 199), "mme_attention_qs_form: form %d (0 or 30 + kind)", form);
    return attention_entry(form, qkv, ld_qkv, out, ld_out, B, T, H, hd, seq_lens, causal, 0.f, true, stream);
}

namespace {
int attention_entry(int form, const void* qkv, int ld_qkv, void* out, int ld_out, int B, int T, int H, int hd,
                    const int32_t* seq_lens, int causal, float scale, bool qs, void* stream) {
    MME_REQUIRE(qkv && out, "mme_attention: null pointer");
    MME_REQUIRE(B >= 0 && T > 0 && H > 0, "mme_attention: bad shape");
    MME_REQUIRE(hd == 64 || hd == 72 || hd == 80, "mme_attention: head_dim %d unsupported (64/72/80)", hd);
    MME_REQUIRE(ld_qkv % 8 == 0 && ld_qkv >= 3 * H * hd, "mme_attention: bad ld_qkv");
    MME_REQUIRE(ld_out % 4 == 0 && ld_out >= H * hd, "mme_attention: bad ld_out");
    MME_REQUIRE(((uintptr_t)qkv & 15) == 0 && ((uintptr_t)out & 7) == 0, "mme_attention: misaligned");
    if (B == 0) return MME_OK;
    // exp(x*scale) = exp2(x*scale*log2 e); qs (mme_attention_qs): Q already carries scale*log2 e
    AttnArgs a{(const bf16*)qkv, (bf16*)out, seq_lens, ld_qkv, ld_out, T, H, hd, causal ? 1 : 0,
               qs ? 1.0f : scale * 1.4426950408889634f};
    // kernel choice (tools/attn_bench.py): short sequences (T <= 128: one or two key tiles)
    // and head dim 64 (3 waves/SIMD already) -> register-staged attn_fwd_kernel; otherwise
    // LDS-DMA staging, 8 waves (256 queries) per block unless that pads the query range by
    // > 10 % more than 128-query blocks (T = 257), then 4 waves. SigLIP-400M vision
    // (T 729, hd 72): 1.80 -> 1.27 ms per 256-image layer; ViT-H (T 257, hd 80): 0.40 -> 0.355.
    // The LDS-DMA kernels run as attn_pipe_kernel's lean non-pipelined form (kinds 11 / 14:
    // lane-base fragment addresses, permlane reductions, lazy rescale, and for hd 72 the
    // weight sums from a ones column of V^T): SigLIP vision 1.27-1.33 -> 1.16-1.17 ms.
    // T <= 64 (SigLIP text): attn_short_kernel, two (batch, head) units of one key tile per block.
    // Head dim 72 (SigLIP vision): kind 17 = kind 11 held to 128 VGPRs (amdgpu_waves_per_eu(4);
    // its 3 spilled registers live outside the tile loop), so two 8-wave blocks share a CU and
    // each SIMD interleaves 4 waves: 1.18 -> 0.98 ms per 256-image layer (532 -> 638 TF/s).
    // At head dim 80 the same cap spills inside the loop and gains nothing (DFN5B 0.628 / 0.622 ms).
    // Round 2: the tile loop unrolled by the ring depth (kind 27: compile-time ring slots, 611-623 ->
    // 637-639 TF/s) and static priority for the second half of the waves (kind 30, +1-2 %).
    // 9-wave blocks (288 queries, kind 21) when they pad far less than 256 / 128-query blocks: ViT-H
    // (T 257, hd 80) runs one block per batch-head, K/V staged once instead of three times and 288
    // padded query rows instead of 384: 0.342 -> 0.277 ms per 256-image layer (253 -> 313 TF/s).
    // Head dim 80: 12-wave blocks (384 queries, kind 23) where they pad no more than 256-query
    // blocks. The 133-VGPR hd-80 build fits 3 waves per SIMD, which 8-wave blocks leave at 2
    // (one block per CU either way): DFN5B (T 730) 0.640 -> 0.558 ms per 128-image layer.
    const long pad8 = (long)cdiv(T, 256) * 256, pad4 = (long)cdiv(T, 128) * 128, pad9 = (long)cdiv(T, 288) * 288;
    const long pad12 = (long)cdiv(T, 384) * 384;
    // Round 2, head dim 80: attn_m32_kernel (32x32x16 MFMAs, QK^T 80 deep instead of 96, weight
    // sums from a ones plane): DFN5B (T 730) 632 -> 700-723 TF/s with 8-wave blocks, ViT-H (T 257)
    // 308-317 -> 349 TF/s with 9-wave blocks (profiles/r02_attn_m32_bench.log). At head dim 72 it
    // measures level with kind 30 (635-645 vs 604-638) and at 64 slower than kind 0: not dispatched.
    // Head dim 72 since round 2: attn_hyb_kernel (kind 58: QK^T on 32x32x16 80 deep, PV on 16x16x32
    // 80 rows -- 9 % less MFMA work than either single-shape form under the power cap): SigLIP
    // vision level to 2 % faster than kind 30 (profiles/r02_attn_hyb_bench.log, r02_hyb_attn.log);
    // kind 62 = kind 58 skipping the last tile's second 32-key block (wholly past T = 729): +1.2 %
    // (profiles/r02_hyb_skip_bench.log, 4 of 4 A/B pairs). Round 4: kind 83 = kind 62 rescaling O only
    // when a query's running max grows by more than 2^8 in the exp2 domain (the rescale branch ran on
    // almost every tile: ~27 of ~174 VALU per wave and tile): 628 -> 660 TF/s at the job's 417-image
    // batch (profiles/r04_v19_attn_threshold_ab.log); mean |error| vs fp64 0.00045 -> 0.00052.
    // The same threshold in attn_m32_kernel (hd 80: kinds 86 / 87 = 65 / 38, ViT-H +3 %, DFN5B +4.5 %) and
    // attn_fwd_kernel (kind 89 = kind 0: CLIP-L vision +3 %, CLIP causal text +1 %;
    // profiles/r04_v20_attn_threshold_hd80_hd64_ab.log).
    // Round 5: kind 94 = kind 86 as a persistent walk over (image, head) units, the next unit's Q and
    // first K / V tile loaded under the current unit's last tile: bit-identical, 7 % faster in isolation
    // (ViT-H at 455 / 512 images: 0.48 / 0.53 -> 0.45 / 0.49 ms, profiles/r05_v10_attn_vith_batches.log)
    // but 3 % slower inside the LAION-CLIP-H job (466 vs 480 us per launch, jobs level;
    // profiles/r05_v9_laion_kind94_vs_kind86_ab.log): not dispatched.
    // Round 6: kind 98 = kind 83 with the exp2 argument c s - M out of the QK^T MFMA (mme_attention_qs: Q
    // pre-scaled by c in the projection, Q^T row 72 = -M against a ones row of K): 1.48 -> 1.40 ms per
    // 417-image launch, SigLIP job +0.8 % (profiles/r06_v5_*); chosen below when qs.
    // Round 6: kind 102 (attn_short2_kernel) for 64 < T <= 128 at head dim 64 (the CLIP causal text towers, T 77):
    // every load of a unit in one burst instead of kind 89's two-tile flash loop.
    int kind = T <= 64 ? 16
               : (T <= 128 && hd == 64) ? 102
               : (T <= 128 || hd == 64) ? 89
               : (hd == 80 && pad9 * 10 < min(pad8, pad4) * 9) ? 86
               : hd == 80 && pad8 * 10 <= pad4 * 11 ? 87
               : pad9 * 10 < min(pad8, pad4) * 9 ? 35
               : (hd == 80 && pad12 <= pad8 && pad12 * 10 <= pad4 * 11) ? 23
               : (pad8 * 10 <= pad4 * 11 ? (hd == 72 ? 83 : 11) : 14);
#ifdef MME_DEV
    if (form >= 1 && form <= 4 && hd == 72) {  // dev-only diagnostic builds
        const dim3 grid(cdiv(T, 128) * H * B);
        switch (form) {
            case 1: hipLaunchKernelGGL((attn_fwd_kernel<72, 1>), grid, dim3(256), 0, as_stream(stream), a); break;
            case 2: hipLaunchKernelGGL((attn_fwd_kernel<72, 2>), grid, dim3(256), 0, as_stream(stream), a); break;
            case 3: hipLaunchKernelGGL((attn_fwd_kernel<72, 3>), grid, dim3(256), 0, as_stream(stream), a); break;
            default: hipLaunchKernelGGL((attn_fwd_kernel<72, 4>), grid, dim3(256), 0, as_stream(stream), a); break;
        }
        return mme_check_launch("mme_attention");
    }
#endif
    // hd 72 with Q pre-scaled: kind 83's loop with the exp2 argument from the MFMA (kind 98, round 6: the
    // per-score FMA goes); a forced kind 83 keeps its own loop (c = 1), the A/B and accuracy reference
    // (kinds 100 / 101 the same in attn_m32_kernel for hd 80: kinds 87 / 86 with an extra k-step for -M)
    if (qs && kind == 83) kind = 98;
    if (qs && kind == 87) kind = 100;
    if (qs && kind == 86) kind = 101;
    if (form >= 9 && form <= 16) kind = form - 9;  // dev: force a kernel
    if (form >= 30 && form <= 199) kind = form - 30;  // dev: force a kernel
    if ((kind == 16 || kind == 19 || kind == 66) && T > 64) kind = 0;  // the short kernels hold one 64-key tile
    if (kind == 102 && (T > 128 || hd != 64)) kind = 0;                 // attn_short2_kernel: 128 keys, hd 64
    // kinds 97 / 98 are one kernel scaling Q itself / taking it pre-scaled
    if (qs && kind == 97) kind = 98;
    if (!qs && kind == 98) kind = 97;
    MME_REQUIRE(qs || (kind != 99 && kind != 100 && kind != 101), "mme_attention: kind %d needs Q pre-scaled "
                "(mme_attention_qs)", kind);
#ifdef MME_DEV
    if (form >= 21 && form <= 26 && hd == 72) {  // dev: attn_dma_kernel<72,8,2> diagnostics
        const dim3 grid(cdiv(T, 256) * H * B), blk(512);
        hipStream_t st = as_stream(stream);
        switch (form) {
            case 21: hipLaunchKernelGGL((attn_dma_kernel<72, 8, 2, 1>), grid, blk, 0, st, a); break;
            case 22: hipLaunchKernelGGL((attn_dma_kernel<72, 8, 2, 2>), grid, blk, 0, st, a); break;
            case 23: hipLaunchKernelGGL((attn_dma_kernel<72, 8, 2, 3>), grid, blk, 0, st, a); break;
            case 24: hipLaunchKernelGGL((attn_dma_kernel<72, 8, 2, 4>), grid, blk, 0, st, a); break;
            case 25: hipLaunchKernelGGL((attn_dma_kernel<72, 8, 2, 5>), grid, blk, 0, st, a); break;
            default: hipLaunchKernelGGL((attn_dma_kernel<72, 8, 2, 6>), grid, blk, 0, st, a); break;
        }
        return mme_check_launch("mme_attention");
    }
#endif
    const bool ok = hd == 64 ? launch_attn<64>(kind, a, B, T, H, as_stream(stream))
                    : hd == 72 ? launch_attn<72>(kind, a, B, T, H, as_stream(stream))
                               : launch_attn<80>(kind, a, B, T, H, as_stream(stream));
    MME_REQUIRE(ok, "mme_attention: kernel kind %d is a development form (build libmme_dev.so: make dev)", kind);
    return mme_check_launch("mme_attention");
}
}  // namespace

namespace {
// map_pool_kernel: the MAP head's attention with the probe query absorbed into the key
// projection (round 3). SigLIP's pooling head scores each token t of image b per head h as
// q_h . (W_k,h x_t + b_k,h) / sqrt(hd) = x_t . U_h + const_h with U_h = W_k,h^T q_h / sqrt(hd),
// and the constant drops out of the softmax; its output per head is
// sum_t p_t (W_v,h x_t + b_v,h) = W_v,h (sum_t p_t x_t) + b_v,h (the weights sum to 1). So
// the K and V projections of all T tokens (a [B*T, 2d] GEMM) become the [B*T, 2H] score GEMM
// S = x . [U_hi; U_lo]^T (U split into two bf16 halves, so the scores carry ~16 mantissa bits)
// and, after this kernel, one [B*H, d] GEMM of the pooled rows with W_v.
// One block per image, thread i = columns 2i, 2i+1: s[t][h] = S[t][h] + S[t][H + h] -> LDS
// (t-major, so the 16 weights of one token are one broadcast read), softmax per head
// (exp and normalisation as probe_attn_img_kernel), then out[b*H + h][c] =
// bf16(sum_t p[t][h] * x[t][c] / sum_t p[t][h]) with fp32 accumulation.
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
constexpr int MAPP_MAXT = 1024, MAPP_H = 16, MAPP_NT = 576;  // D <= 2 * 576 = 1152
__global__ __launch_bounds__(MAPP_NT) void map_pool_kernel(const float* __restrict__ S, int lds,
                                                           const bf16* __restrict__ x, int ldx,
                                                           bf16* __restrict__ out, int ldo, int T, int H, int D) {
    __shared__ __attribute__((aligned(16))) float pt[MAPP_MAXT * MAPP_H];
    __shared__ float hinv[MAPP_H];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = MAPP_NT / 64;
    const int b = blockIdx.x;
    const float* Sb = S + (size_t)b * T * lds;
    for (int i = tid; i < T * MAPP_H; i += MAPP_NT) {
        const int t = i / MAPP_H, h = i % MAPP_H;
        pt[i] = h < H ? Sb[(size_t)t * lds + h] + Sb[(size_t)t * lds + H + h] : 0.f;
    }
    __syncthreads();
    for (int h = wave; h < H; h += nw) {
        float mx = -INFINITY;
        for (int t = lane; t < T; t += 64) mx = fmaxf(mx, pt[t * MAPP_H + h]);
        mx = wave_max(mx);
        float sum = 0.f;
        for (int t = lane; t < T; t += 64) {
            const float p = __expf(pt[t * MAPP_H + h] - mx);
            pt[t * MAPP_H + h] = p;
            sum += p;
        }
        sum = wave_sum(sum);
        if (lane == 0) hinv[h] = 1.f / sum;
    }
    __syncthreads();
    const int c = 2 * tid;
    if (c >= D) return;
    const bf16* xb = x + (size_t)b * T * ldx + c;
    float acc[MAPP_H][2];
#pragma unroll
    for (int h = 0; h < MAPP_H; ++h) acc[h][0] = acc[h][1] = 0.f;
    constexpr int U = 8;
    int t = 0;
    for (; t + U <= T; t += U) {
        u16x2 xv[U];
#pragma unroll
        for (int j = 0; j < U; ++j) xv[j] = *reinterpret_cast<const u16x2*>(xb + (size_t)(t + j) * ldx);
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const float x0 = bits2f(xv[j][0]), x1 = bits2f(xv[j][1]);
            const float4* pr = reinterpret_cast<const float4*>(pt + (t + j) * MAPP_H);
#pragma unroll
            for (int q = 0; q < MAPP_H / 4; ++q) {
                const float4 p = pr[q];
                acc[4 * q][0] += p.x * x0; acc[4 * q][1] += p.x * x1;
                acc[4 * q + 1][0] += p.y * x0; acc[4 * q + 1][1] += p.y * x1;
                acc[4 * q + 2][0] += p.z * x0; acc[4 * q + 2][1] += p.z * x1;
                acc[4 * q + 3][0] += p.w * x0; acc[4 * q + 3][1] += p.w * x1;
            }
        }
    }
    for (; t < T; ++t) {
        const u16x2 xv = *reinterpret_cast<const u16x2*>(xb + (size_t)t * ldx);
        const float x0 = bits2f(xv[0]), x1 = bits2f(xv[1]);
#pragma unroll
        for (int h = 0; h < MAPP_H; ++h) {
            acc[h][0] += pt[t * MAPP_H + h] * x0;
            acc[h][1] += pt[t * MAPP_H + h] * x1;
        }
    }
#pragma unroll
    for (int h = 0; h < MAPP_H; ++h) {
        if (h >= H) break;
        const float inv = hinv[h];
        bf16x2 o;
        o[0] = f2bf(acc[h][0] * inv);
        o[1] = f2bf(acc[h][1] * inv);
        *reinterpret_cast<bf16x2*>(out + (size_t)(b * H + h) * ldo + c) = o;
    }
}
}  // namespace

extern "C" int mme_map_pool(const float* S, int ld_s, const void* x, int ld_x, void* out, int ld_out, int B, int T,
                            int H, int D, void* stream) {
    MME_REQUIRE(S && x && out, "mme_map_pool: null pointer");
    MME_REQUIRE(B >= 0 && T > 0 && T <= MAPP_MAXT && H > 0 && H <= MAPP_H, "mme_map_pool: bad shape (T<=%d, H<=%d)",
                MAPP_MAXT, MAPP_H);
    MME_REQUIRE(D > 0 && D % 2 == 0 && D <= 2 * MAPP_NT, "mme_map_pool: D=%d must be even and <= %d", D, 2 * MAPP_NT);
    MME_REQUIRE(ld_s >= 2 * H && ld_x >= D && ld_x % 2 == 0 && ld_out >= D && ld_out % 2 == 0,
                "mme_map_pool: bad leading dims");
    MME_REQUIRE(((uintptr_t)x & 3) == 0 && ((uintptr_t)out & 3) == 0, "mme_map_pool: x / out must be 4-byte aligned");
    if (B == 0) return MME_OK;
    hipLaunchKernelGGL(map_pool_kernel, dim3(B), dim3(MAPP_NT), 0, as_stream(stream), S, ld_s, (const bf16*)x, ld_x,
                       (bf16*)out, ld_out, T, H, D);
    return mme_check_launch("mme_map_pool");
}

extern "C" int mme_probe_attention(const void* q, const void* kv, int ld_kv, void* out, int ld_out, int B, int T,
                                   int H, int hd, float scale, void* stream) {
    MME_REQUIRE(q && kv && out, "mme_probe_attention: null pointer");
    MME_REQUIRE(B >= 0 && T > 0 && T <= PROBE_MAXT && H > 0, "mme_probe_attention: bad shape (T<=%d)", PROBE_MAXT);
    MME_REQUIRE(hd % 8 == 0 && hd <= 128, "mme_probe_attention: head_dim %d unsupported", hd);
    MME_REQUIRE(ld_kv % 8 == 0 && ld_kv >= 2 * H * hd, "mme_probe_attention: bad ld_kv");
    if (B == 0) return MME_OK;
    const int D = H * hd, TR = H <= 16 && 256 % H == 0 ? 256 / H : 0;
    if (TR && D <= PROBE2_D && D % 8 == 0 && (TR * D / 8) % 64 == 0 && hd % 8 == 0 && ld_kv % 8 == 0 &&
        ld_out % 8 == 0 && ((uintptr_t)out & 15) == 0 && ((uintptr_t)kv & 15) == 0 && attn_default_form() != 200)
        hipLaunchKernelGGL(probe_attn_img_kernel, dim3(B), dim3(256), 0, as_stream(stream), (const bf16*)q,
                           (const bf16*)kv, ld_kv, (bf16*)out, ld_out, T, H, hd, scale);
    else  // other geometries (and dev variant 200: the per-(image, head) form for A/B)
        hipLaunchKernelGGL(probe_attn_kernel, dim3(H * B), dim3(256), 0, as_stream(stream), (const bf16*)q,
                           (const bf16*)kv, ld_kv, (bf16*)out, ld_out, T, H, hd, scale);
    return mme_check_launch("mme_probe_attention");
}
