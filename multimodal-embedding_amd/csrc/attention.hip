// Fused multi-head attention for the ViT / text encoders (flash-style, gfx950).
//
// softmax(Q K^T * scale + mask) V for one (batch, head, 64-query block) per
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
//   * head dims 72 and 80 run as 2 x K32 + 1 x K16 MFMA steps (padding 72 to
//     80, not 96); the O^T accumulators cover 5 d-tiles of 16.
//   * K/V tiles are double-buffered through registers: the global loads of
//     tile t+1 are issued before the MFMAs of tile t and written to the other
//     LDS buffer afterwards.
#include "common.h"

namespace {

typedef short s16x8 __attribute__((ext_vector_type(8)));

struct AttnArgs {
    const bf16* qkv;
    bf16* out;
    const int32_t* seq_lens;
    int ld, ldo, T, H, hd, causal;
    float scale_log2;
};

template <int HDP>
__global__ __launch_bounds__(256) void attn_fwd_kernel(AttnArgs a) {
    constexpr int KS = HDP + 8;      // K LDS row stride (elements)
    constexpr int VS = 80;           // V LDS row stride (elements): conflict-free tr reads
    constexpr int NCH_K = HDP / 8;   // 16-B chunks of a K row kept in LDS
    constexpr int NCH_V = VS / 8;
    constexpr int NDT = HDP / 16;    // output d-tiles of 16
    constexpr int NCHUNK = 64 * (NCH_K + NCH_V);
    constexpr int CPT = (NCHUNK + 255) / 256;
    __shared__ __attribute__((aligned(16))) bf16 Ks[2][64 * KS];
    __shared__ __attribute__((aligned(16))) bf16 Vs[2][64 * VS];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int g = lane >> 4, li = lane & 15;
    const int b = blockIdx.z, h = blockIdx.y;
    const int T = a.T, hd = a.hd, D = a.H * a.hd;
    const bf16* base = a.qkv + (long)b * T * a.ld;
    const int q = blockIdx.x * 64 + wave * 16 + li;
    const int Tk = a.seq_lens ? a.seq_lens[b] : T;

    // Q^T fragments (B operand): lane holds Q[q][32ks + 8g + j]
    bf16x8 qf[2];
    s16x4 qt = {0, 0, 0, 0};
    {
        const bf16* qrow = base + (long)min(q, T - 1) * a.ld + h * hd;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) qf[ks] = *reinterpret_cast<const bf16x8*>(qrow + ks * 32 + 8 * g);
        if constexpr (HDP == 80) {
            if (64 + 4 * g < hd) qt = *reinterpret_cast<const s16x4*>(qrow + 64 + 4 * g);
        }
    }

    int nkt = (T + 63) / 64;
    if (a.causal) nkt = min(nkt, (min(T, (int)blockIdx.x * 64 + 64) + 63) / 64);

    u16x8 pre[CPT];
    auto load_tile = [&](int t) {
#pragma unroll
        for (int i = 0; i < CPT; ++i) {
            const int c = tid + i * 256;
            u16x8 v = {0, 0, 0, 0, 0, 0, 0, 0};
            if (c < NCHUNK) {
                const bool isk = c < 64 * NCH_K;
                const int cc = isk ? c : c - 64 * NCH_K;
                const int nch = isk ? NCH_K : NCH_V;
                const int row = cc / nch, ch = cc % nch;
                const int key = t * 64 + row;
                if (key < T && ch * 8 < hd)
                    v = *reinterpret_cast<const u16x8*>(base + (long)key * a.ld + (isk ? D : 2 * D) + h * hd + ch * 8);
            }
            pre[i] = v;
        }
    };
    auto store_tile = [&](int buf) {
#pragma unroll
        for (int i = 0; i < CPT; ++i) {
            const int c = tid + i * 256;
            if (c < NCHUNK) {
                if (c < 64 * NCH_K) {
                    const int row = c / NCH_K, ch = c % NCH_K;
                    *reinterpret_cast<u16x8*>(&Ks[buf][row * KS + ch * 8]) = pre[i];
                } else {
                    const int cc = c - 64 * NCH_K;
                    const int row = cc / NCH_V, ch = cc % NCH_V;
                    *reinterpret_cast<u16x8*>(&Vs[buf][row * VS + ch * 8]) = pre[i];
                }
            }
        }
    };

    f32x4 o[NDT];
#pragma unroll
    for (int i = 0; i < NDT; ++i) o[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    float m = -1e30f, lsum = 0.f;

    load_tile(0);
    store_tile(0);
    __syncthreads();
    for (int t = 0; t < nkt; ++t) {
        const int buf = t & 1;
        if (t + 1 < nkt) load_tile(t + 1);
        const bf16* Kb = Ks[buf];
        const bf16* Vb = Vs[buf];

        // S^T[key][q] for 4 sub-tiles of 16 keys
        f32x4 s[4];
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) {
            s[kt] = f32x4{0.f, 0.f, 0.f, 0.f};
            const bf16* krow = Kb + (kt * 16 + li) * KS;
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
                const bf16x8 ka = *reinterpret_cast<const bf16x8*>(krow + ks * 32 + 8 * g);
                s[kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ka, qf[ks], s[kt], 0, 0, 0);
            }
            if constexpr (HDP == 80) {
                const s16x4 ka = *reinterpret_cast<const s16x4*>(krow + 64 + 4 * g);
                s[kt] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(ka, qt, s[kt], 0, 0, 0);
            }
        }

        // online softmax over this tile (log2 domain)
        float mloc = -1e30f;
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int key = t * 64 + kt * 16 + 4 * g + r;
                const bool ok = key < Tk && (!a.causal || key <= q);
                const float x = ok ? s[kt][r] * a.scale_log2 : -INFINITY;
                s[kt][r] = x;
                mloc = fmaxf(mloc, x);
            }
        mloc = fmaxf(mloc, __shfl_xor(mloc, 16, 64));
        mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
        const float mnew = fmaxf(m, mloc);
        const float alpha = exp2f(m - mnew);
        m = mnew;
        float psum = 0.f;
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float p = exp2f(s[kt][r] - mnew);
                s[kt][r] = p;
                psum += p;
            }
        lsum = lsum * alpha + psum;
#pragma unroll
        for (int i = 0; i < NDT; ++i) o[i] *= alpha;

        // O^T[d][q] += V^T[d][key] . P^T[key][q]
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
            bf16x8 pb;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                pb[j] = f2bf(s[2 * hh][j]);
                pb[4 + j] = f2bf(s[2 * hh + 1][j]);
            }
            const int r1 = 32 * hh + 4 * g + (li >> 2);
#pragma unroll
            for (int dt = 0; dt < NDT; ++dt) {
                const int col = dt * 16 + 4 * (li & 3);
                const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(Vb + r1 * VS + col));
                const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(Vb + (r1 + 16) * VS + col));
                const s16x8 vv = __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7);
                o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, vv), pb, o[dt], 0, 0, 0);
            }
        }

        if (t + 1 < nkt) store_tile(buf ^ 1);
        __syncthreads();
    }

    float ltot = lsum + __shfl_xor(lsum, 16, 64);
    ltot += __shfl_xor(ltot, 32, 64);
    const float inv = 1.0f / ltot;
    if (q < T) {
        bf16* orow = a.out + ((long)b * T + q) * a.ldo + h * hd;
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) {
            const int d0 = dt * 16 + 4 * g;
            if (d0 < hd) {
                bf16x4 v;
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] = f2bf(o[dt][r] * inv);
                *reinterpret_cast<bf16x4*>(orow + d0) = v;
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
    const int h = blockIdx.x, b = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
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

}  // namespace

extern "C" int mme_attention(const void* qkv, int ld_qkv, void* out, int ld_out, int B, int T, int H, int hd,
                             const int32_t* seq_lens, int causal, float scale, void* stream) {
    MME_REQUIRE(qkv && out, "mme_attention: null pointer");
    MME_REQUIRE(B >= 0 && T > 0 && H > 0, "mme_attention: bad shape");
    MME_REQUIRE(hd == 64 || hd == 72 || hd == 80, "mme_attention: head_dim %d unsupported (64/72/80)", hd);
    MME_REQUIRE(ld_qkv % 8 == 0 && ld_qkv >= 3 * H * hd, "mme_attention: bad ld_qkv");
    MME_REQUIRE(ld_out % 4 == 0 && ld_out >= H * hd, "mme_attention: bad ld_out");
    MME_REQUIRE(((uintptr_t)qkv & 15) == 0 && ((uintptr_t)out & 7) == 0, "mme_attention: misaligned");
    if (B == 0) return MME_OK;
    AttnArgs a{(const bf16*)qkv, (bf16*)out, seq_lens, ld_qkv, ld_out, T, H, hd, causal ? 1 : 0,
               scale * 1.4426950408889634f};
    dim3 grid(cdiv(T, 64), H, B);
    if (hd == 64)
        hipLaunchKernelGGL(attn_fwd_kernel<64>, grid, dim3(256), 0, as_stream(stream), a);
    else
        hipLaunchKernelGGL(attn_fwd_kernel<80>, grid, dim3(256), 0, as_stream(stream), a);
    return mme_check_launch("mme_attention");
}

extern "C" int mme_probe_attention(const void* q, const void* kv, int ld_kv, void* out, int ld_out, int B, int T,
                                   int H, int hd, float scale, void* stream) {
    MME_REQUIRE(q && kv && out, "mme_probe_attention: null pointer");
    MME_REQUIRE(B >= 0 && T > 0 && T <= PROBE_MAXT && H > 0, "mme_probe_attention: bad shape (T<=%d)", PROBE_MAXT);
    MME_REQUIRE(hd % 8 == 0 && hd <= 128, "mme_probe_attention: head_dim %d unsupported", hd);
    MME_REQUIRE(ld_kv % 8 == 0 && ld_kv >= 2 * H * hd, "mme_probe_attention: bad ld_kv");
    if (B == 0) return MME_OK;
    hipLaunchKernelGGL(probe_attn_kernel, dim3(H, B), dim3(256), 0, as_stream(stream), (const bf16*)q,
                       (const bf16*)kv, ld_kv, (bf16*)out, ld_out, T, H, hd, scale);
    return mme_check_launch("mme_probe_attention");
}
