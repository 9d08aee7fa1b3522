// MX-fp8 (OCP e4m3 values + E8M0 scales per 32-element block) path for the
// encoder GEMMs: quantisers and the block-scaled fp8 MFMA GEMM.
//
// This is the "fp8 weights on CDNA4 fp8 MFMA" configuration of BASELINE.json
// (Apple-DFN5B-H, config 5): the reference runs these layers in bf16
// (TF:models/clip/modeling_clip.py CLIPMLP / CLIPAttention q,k,v projections);
// here the QKV, fc1 and fc2 products of every encoder layer run on
// v_mfma_scale_f32_32x32x64_f8f6f4 (2x the bf16 MFMA rate) with both operands
// in MX-fp8 and the block scales applied by the MFMA itself.
//
// MX tensor format ("mx8"), shared with the host (mme/mx.py) and the oracle
// (oracle/mx.py): values u8 [R][K] (row stride ld bytes, e4m3fn), scales u8
// [K/32][rows_pad] block-major "scale planes" (rows_pad a multiple of 256,
// so one 256-row GEMM tile's scales of one block are 256 contiguous bytes).
// Element (r, k) = e4m3(q[r][k]) * 2^(S[k/32][r] - 127).
//
// Quantisation of a block with absmax a (bf16 inputs, exact in fp32):
//   a == 0          -> scale byte 127, all values 0
//   otherwise       -> scale byte e = clamp(expfield(a) - 8 + (mantissa(a) > 0x600000), 1, 254),
//                      the smallest power of two with a * 2^-(e-127) <= 448;
//                      q = RNE_e4m3(clamp(x * 2^-(e-127), -448, 448))
// (v_cvt_pk_fp8_f32 is RNE once the input is clamped: tools/probes/fp8_probe.hip).
#include "gemm_core.h"

namespace {
using namespace gemmcore;

typedef int i32x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ int mx_scale_byte(float amax) {
    if (amax == 0.f) return 127;
    const unsigned u = __float_as_uint(amax);
    const int e = (int)((u >> 23) & 255) - 8 + ((u & 0x7fffff) > 0x600000 ? 1 : 0);
    return min(254, max(1, e));
}

// 8 values -> 8 e4m3 bytes (as two dwords) after scaling by 2^(127 - sb)
__device__ __forceinline__ uint2 mx_pack8(const float (&v)[8], int sb) {
    float s[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) s[e] = fminf(448.f, fmaxf(-448.f, __builtin_amdgcn_ldexpf(v[e], 127 - sb)));
    unsigned lo = 0, hi = 0;
    lo = __builtin_amdgcn_cvt_pk_fp8_f32(s[0], s[1], lo, false);
    lo = __builtin_amdgcn_cvt_pk_fp8_f32(s[2], s[3], lo, true);
    hi = __builtin_amdgcn_cvt_pk_fp8_f32(s[4], s[5], hi, false);
    hi = __builtin_amdgcn_cvt_pk_fp8_f32(s[6], s[7], hi, true);
    return make_uint2(lo, hi);
}

// mx_pack8 for the GEMM epilogue (round 6, FQ): no clamp and packed scaling. sb = mx_scale_byte(amax) makes
// amax * 2^(127 - sb) <= 448 for every finite block: amax = (1 + m) 2^(E - 127) scales to (1 + m) 2^8 <= 448 for
// m <= 0.75 and to (1 + m) 2^7 < 256 above (sb clamped at 1 only for amax < 2^-118, which scales below 1); so the
// clamp never acts and the result is mx_pack8's, bit for bit. The epilogue's values are bf16-rounded, so sb <=
// 247 and 2^(127 - sb) is a normal float, applied by one exact multiply (v_pk_mul_f32: two values per issue).
__device__ __forceinline__ uint2 mx_pack8_fast(const float (&v)[8], int sb) {
    const float m = __uint_as_float((unsigned)(254 - sb) << 23);
    const f32x2 mm = {m, m};
    const f32x2 s0 = f32x2{v[0], v[1]} * mm, s1 = f32x2{v[2], v[3]} * mm;
    const f32x2 s2 = f32x2{v[4], v[5]} * mm, s3 = f32x2{v[6], v[7]} * mm;
    unsigned lo = 0, hi = 0;
    lo = __builtin_amdgcn_cvt_pk_fp8_f32(s0.x, s0.y, lo, false);
    lo = __builtin_amdgcn_cvt_pk_fp8_f32(s1.x, s1.y, lo, true);
    hi = __builtin_amdgcn_cvt_pk_fp8_f32(s2.x, s2.y, hi, false);
    hi = __builtin_amdgcn_cvt_pk_fp8_f32(s3.x, s3.y, hi, true);
    return make_uint2(lo, hi);
}

// Scale-plane row order (round 4): inside each 128-row group of a plane, row r is stored at
// (r % 32) * 4 + (r % 128) / 32, so the 4 scale bytes a 32x32x64 MFMA lane needs for the rows
// i * 32 + r (i = 0..3) of one block are one aligned dword (gemm_mx11: one 4-byte load per block).
__device__ __forceinline__ int mx_srow(int r) { return (r & ~127) | ((r & 31) << 2) | ((r >> 5) & 3); }

// absmax over the 4 consecutive lanes holding one 32-element block
__device__ __forceinline__ float block_amax(float a) {
    a = fmaxf(a, __shfl_xor(a, 1, 64));
    a = fmaxf(a, __shfl_xor(a, 2, 64));
    return a;
}
// the same by DPP quad permutes ([1,0,3,2], then [2,3,0,1]) instead of two ds_bpermute round trips
// (max is exact in any order: bit-identical); a >= 0, so a disabled source lane's 0 is harmless
__device__ __forceinline__ float block_amax_dpp(float a) {
    a = fmaxf(a, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(a), 0xB1, 0xF, 0xF, false)));
    a = fmaxf(a, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(a), 0x4E, 0xF, 0xF, false)));
    return a;
}

// ---------------------------------------------------------------------------
// bf16 rows -> mx8. One 256-thread block per row; thread t handles 16-B
// chunks t, t+256, ...: four consecutive threads = one 32-element block.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void mx_quant_kernel(const bf16* __restrict__ x, int ldx, int k,
                                                       uint8_t* __restrict__ q, int ldq, uint8_t* __restrict__ sc,
                                                       int rows_pad) {
    const int row = blockIdx.x;
    const int nch = k >> 3;
    const bf16* xr = x + (long)row * ldx;
    for (int c0 = 0; c0 < nch; c0 += 256) {  // uniform trip count: shuffles see whole groups
        const int ch = c0 + threadIdx.x;
        float v[8];
        float a = 0.f;
        if (ch < nch) {
            const u16x8 u = *reinterpret_cast<const u16x8*>(xr + ch * 8);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                v[e] = bits2f(u[e]);
                a = fmaxf(a, fabsf(v[e]));
            }
        } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = 0.f;
        }
        const int sb = mx_scale_byte(block_amax(a));
        if (ch < nch) {
            *reinterpret_cast<uint2*>(q + (long)row * ldq + ch * 8) = mx_pack8(v, sb);
            if ((ch & 3) == 0) sc[(long)(ch >> 2) * rows_pad + mx_srow(row)] = (uint8_t)sb;
        }
    }
}

// ---------------------------------------------------------------------------
// LayerNorm -> mx8 (the QKV / fc1 operand straight from the norm): same
// statistics as layernorm_kernel (norm.hip; the shared common.h ln_*_half helpers),
// the output rounded to bf16 (the value the bf16 path would feed the GEMM) and then
// block-quantised. One row per HALF wave (round 5: at d = 1 280 every lane holds 5
// chunks, where a whole wave per row left a third of its lanes idle on the last one);
// lane chunks ch = hl + 32 c, so 4 consecutive lanes hold one 32-element block.
// ---------------------------------------------------------------------------
template <int MAXC>
__global__ __launch_bounds__(256) void layernorm_mx_kernel(const bf16* __restrict__ x, int ldx,
                                                           const bf16* __restrict__ g, const bf16* __restrict__ b,
                                                           int rows, int d, float eps, const int32_t* __restrict__ idx,
                                                           uint8_t* __restrict__ q, int ldq, uint8_t* __restrict__ sc,
                                                           int rows_pad) {
    const int row = blockIdx.x * 8 + (threadIdx.x >> 5);
    const int hl = threadIdx.x & 31;
    if (row >= rows) return;  // the half wave's 32 lanes together
    const long src = idx ? idx[row] : row;
    const int nch = d >> 3;
    float v[MAXC][8];
    u16x8 gu[MAXC], bu[MAXC];
    ln_load_half(x + src * ldx, nch, hl, v);
    ln_load_affine_half(g, b, nch, hl, gu, bu);  // in flight with the row (round 6)
    float mean, rstd;
    ln_stats_half(v, nch, hl, d, eps, mean, rstd);
    // every chunk computed without a branch (chunks past the row: x = gamma = beta = 0 give o = +0 exactly,
    // as the explicit zeros did), so hipcc keeps the gamma / beta loads up with the row's instead of sinking
    // them into per-chunk branches; only the stores are conditional
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
        const int ch = hl + 32 * c;
        float o[8];
        float a = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            o[e] = bf2f(f2bf((v[c][e] - mean) * rstd * bits2f(gu[c][e]) + bits2f(bu[c][e])));
            a = fmaxf(a, fabsf(o[e]));
        }
        const int sb = mx_scale_byte(block_amax(a));
        if (ch < nch) {
            // the outputs are bf16-rounded: mx_pack8_fast is exact (round 6)
            *reinterpret_cast<uint2*>(q + (long)row * ldq + ch * 8) = mx_pack8_fast(o, sb);
            if ((ch & 3) == 0) sc[(long)(ch >> 2) * rows_pad + mx_srow(row)] = (uint8_t)sb;
        }
    }
}

// ---------------------------------------------------------------------------
// Block-scaled fp8 GEMM: C[m][n] = act(sum_k A[m][k] B[n][k] + bias[n]) (+ residual),
// A, B in mx8. Same schedule as gemm_pipe6_kernel (gemm.hip): 256 x 256 tile,
// 8 waves in two ping-pong rows, 4-deep LDS ring of 64-deep K stages (64-B
// rows: the same byte geometry as the bf16 kernel's 32-deep stages), one
// memory and one compute phase per stage. Per stage each wave issues 8
// v_mfma_scale_f32_32x32x64_f8f6f4 (128 x 64 outputs as 4 x 2 tiles of 32 x 32)
// fed by 12 ds_read_b128 + 6 scale-byte reads.
//   * operand k-layout (probe-verified): lane (r, h = lane >> 5) holds bytes
//     k = 16h .. 16h+15 then 32+16h .. 32+16h+15 of row r -> LDS chunks h and
//     2 + h of the 64-B row; its scale operand is row r's block h;
//   * LDS swizzle chunk ^ ((row >> 2) & 3): the 16 lanes of each ds_read_b128
//     group (rows {0-3, 12-15, 20-27} / {4-11, 16-19, 28-31} of a 32-row
//     fragment) land in 16 distinct bank quads;
//   * per stage a 1 KiB scale piece ([A blk0][A blk1][B blk0][B blk1], 256 B
//     each) rides along, DMA'd by 8 lanes of every wave (uniform vmcnt).
// Epilogue: bf16 output through LDS as in gemm.hip, or (out_mx) the bf16
// value re-quantised to mx8 per 32-column block -- fc1's output is fc2's
// A operand with no extra pass.
// ---------------------------------------------------------------------------
struct MxArgs {
    const uint8_t* A;
    const uint8_t* B;
    const uint8_t* sa;
    const uint8_t* sb;
    void* C;
    uint8_t* sc;
    const bf16* bias;
    const bf16* res;
    int lda, ldb, ldc, ldr;
    int sa_rows, sb_rows, sc_rows;
    int M, N, K;
    int res_period, act, out_mx;
};

struct MxCfg {
    static constexpr int BM = 256, BN = 256, WM = 2, WN = 4, NW = WM * WN, NT = NW * 64;
    static constexpr int TM = 128, TN = 64, FM = 4, FN = 2;  // 32 x 32 tiles per wave
    static constexpr int BK = 64;                            // fp8 elements (bytes) per stage
    static constexpr int A_ST = BM * BK, B_ST = BN * BK, SC_ST = 1024;
    static constexpr int STAGE = A_ST + B_ST + SC_ST, NSTAGE = 4;
    static constexpr int A_PIECES = A_ST / 1024, PIECES = (A_ST + B_ST) / 1024, PPW = PIECES / NW;  // data
    static constexpr int OUT_LD = BN * 2 + 16;
    static constexpr int LDS_MAIN = NSTAGE * STAGE, LDS_OUT = BM * OUT_LD;
    static constexpr int LDS = LDS_MAIN > LDS_OUT ? LDS_MAIN : LDS_OUT;
};

__device__ __forceinline__ int mxswz(int row, int chunk) { return chunk ^ ((row >> 2) & 3); }
template <int V>
struct IC2 {  // an int as a type (compile-time ds offsets through generic lambdas)
    static constexpr int value = V;
};

// Raw-buffer LDS-DMA helpers (mx9 / mx10): four 1 KiB pieces LDS m0base + q KiB <- rsrc base +
// voff[q] + soff, M0 stepped by s_add (its SCC write declared).
typedef int i32x4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ i32x4v mx_rsrc(const void* base, unsigned bytes) {
    const unsigned long long b = (unsigned long long)(uintptr_t)base;
    i32x4v r;
    r[0] = __builtin_amdgcn_readfirstlane((int)(unsigned)b);
    r[1] = __builtin_amdgcn_readfirstlane((int)(unsigned)(b >> 32));
    r[2] = __builtin_amdgcn_readfirstlane((int)bytes);
    r[3] = 0x00020000;
    return r;
}
// PAD (mx12): five wait states open the statement -- an "s" operand may come straight from a v_readlane
// (an SGPR spill reload: a VALU write of an SGPR that a VMEM instruction then reads needs 5 wait states,
// which hipcc does not insert for an inline-asm consumer)
template <bool PAD = false>
__device__ __forceinline__ void mx_dma4(unsigned m0base, const unsigned (&voff)[4], i32x4v rsrc, unsigned soff) {
#define MX_DMA4_BODY                                                                                          \
    "s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %5, %6 offen lds\n\t"                          \
    "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\tbuffer_load_dwordx4 %2, %5, %6 offen lds\n\t"                   \
    "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\tbuffer_load_dwordx4 %3, %5, %6 offen lds\n\t"                   \
    "s_add_u32 m0, m0, 0x400\n\ts_nop 0\n\tbuffer_load_dwordx4 %4, %5, %6 offen lds"
    if constexpr (PAD)
        asm volatile("s_nop 4\n\t" MX_DMA4_BODY::"s"(m0base), "v"(voff[0]), "v"(voff[1]), "v"(voff[2]), "v"(voff[3]),
                     "s"(rsrc), "s"(soff)
                     : "memory", "m0", "scc");  // s_add_u32 writes SCC
    else
        asm volatile(MX_DMA4_BODY::"s"(m0base), "v"(voff[0]), "v"(voff[1]), "v"(voff[2]), "v"(voff[3]), "s"(rsrc),
                     "s"(soff)
                     : "memory", "m0", "scc");  // s_add_u32 writes SCC
#undef MX_DMA4_BODY
}
__device__ __forceinline__ void mx_dma1(unsigned m0base, unsigned voff, i32x4v rsrc, unsigned soff) {
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
                 ::"s"(m0base), "v"(voff), "s"(rsrc), "s"(soff) : "memory", "m0", "scc");
}

// Per-wave epilogue of the mx8 GEMMs (gemm_mx_kernel WEPI, mx9): each wave stages its own 128 x 64
// sub-tile in its own LDS region (pitch 144 B, 18 KiB; 144 KiB for the 8 waves), reads it back as
// 16-B row chunks and stores it (bf16, + residual) or re-quantises it to mx8 -- no workgroup barrier,
// so the early wave row's epilogue runs beside the late row's last MFMAs. Same arithmetic as the
// whole-tile epilogue of gemm_mx_kernel (bit-identical outputs).
// Staging layout (round 4, SWZ; the bf16 kernels' gemm_epilogue_wave has the reasoning): 128-B rows,
// 16-B chunk c of row r at chunk c ^ (r & 7), its 8-B halves swapped when bit 3 of r is set --
// conflict-free ds_write_b64 staging (16 contiguous lanes = rows r32 0..15) and ds_read_b128
// read-back; SWZ = false: the round-3 pitch-144 layout (2-way on both; dev form 4).
constexpr int MXW_PITCH = 144, MXW_LDS = 8 * 128 * MXW_PITCH;
// SB (mx11): a scheduling barrier after each staged column quad keeps the unrolled staging loop
// from interleaving (and holding live) all 32 quads' activations at once.
// PASSES (mx12, round 5): the sub-tile staged and stored in PASSES row bands through a region of
// 128 / PASSES rows per wave (2: 8 KiB per wave, two of the five ring units), as pipe10's epilogue.
// BPRE (mx form 15, round 5): the wave's 32 bias values loaded up front as eight 8-B loads (one wait)
// instead of four 2-B loads and a wait per column quad (needs N % 4 == 0 and an 8-B aligned bias:
// a quad's columns are then all in range or all past N, so clamping the quad start is exact).
// FQ (form 17, round 6): the mx8 output packed by mx_pack8_fast (bit-identical to mx_pack8).
template <int ACT, bool SWZ = true, bool SB = false, int PASSES = 1, bool BPRE = false, bool DPPA = false, bool FQ = false>
__device__ __forceinline__ void mx_epilogue_wave(const MxArgs& p, char* lds, f32x16 (&acc)[4][2], int m0, int n0,
                                                 int wave, int lane) {
    static_assert(PASSES == 1 || (PASSES == 2 && SWZ), "one or two staging passes");
    constexpr int TM = 128, TN = 64, MX9_PITCH = SWZ ? 128 : MXW_PITCH, BAND = TM / PASSES;
    const int wm = wave / 4, wn = wave % 4;
    const int h = lane >> 5, r32 = lane & 31;
    // lane (r32, h) holds row i*32 + r32, columns j*32 + 8q + 4h + (0..3)
    char* reg = lds + wave * (BAND * MX9_PITCH);
    const int rm0 = m0 + wm * TM, cn0 = n0 + wn * TN;
    const int rr = lane >> 3, cc = lane & 7;
    uint2 bq[BPRE ? 8 : 1];
    if constexpr (BPRE) {
#pragma unroll
        for (int jq = 0; jq < 8; ++jq) {
            const int nl = (jq >> 2) * 32 + 8 * (jq & 3) + 4 * h;
            bq[jq] = p.bias ? *reinterpret_cast<const uint2*>(p.bias + min(cn0 + nl, p.N - 4)) : uint2{0u, 0u};
        }
    }
#pragma unroll
    for (int ps = 0; ps < PASSES; ++ps) {
    if (ps > 0) lgkm_wait<0>();  // the previous band's read-back done before its region is rewritten
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int qd = 0; qd < 4; ++qd) {
            const int nl = j * 32 + 8 * qd + 4 * h;
            float bv[4] = {0.f, 0.f, 0.f, 0.f};
            if constexpr (BPRE) {  // bf16 -> f32: the 16 bits as the high half
                const uint2 w = bq[j * 4 + qd];
                bv[0] = __uint_as_float(w.x << 16), bv[1] = __uint_as_float(w.x & 0xffff0000u);
                bv[2] = __uint_as_float(w.y << 16), bv[3] = __uint_as_float(w.y & 0xffff0000u);
            } else if (p.bias) {
#pragma unroll
                for (int r = 0; r < 4; ++r) bv[r] = bf2f(p.bias[min(cn0 + nl + r, p.N - 1)]);
            }
#pragma unroll
            for (int i = ps * (4 / PASSES); i < (ps + 1) * (4 / PASSES); ++i) {
                bf16x4 o;
                if constexpr (DPPA && (ACT == MME_ACT_QUICK_GELU || ACT == MME_ACT_NONE)) {
                    // packed f32 (form 16): the same operations as apply_act's for these two, so the same bits
#pragma unroll
                    for (int r = 0; r < 4; r += 2) {
                        const f32x2 y = apply_act2(f32x2{acc[i][j][4 * qd + r], acc[i][j][4 * qd + r + 1]} +
                                                       f32x2{bv[r], bv[r + 1]},
                                                   ACT);
                        o[r] = f2bf(y.x);
                        o[r + 1] = f2bf(y.y);
                    }
                } else {
#pragma unroll
                    for (int r = 0; r < 4; ++r) o[r] = f2bf(apply_act(acc[i][j][4 * qd + r] + bv[r], ACT));
                }
                const int lrow = i * 32 + r32 - ps * BAND;
                if constexpr (SWZ)  // chunk 4 j + qd ^ (row & 7), half h ^ (row >> 3 & 1); row & 31 = r32
                    *reinterpret_cast<bf16x4*>(reg + lrow * MX9_PITCH + (((4 * j + qd) ^ (r32 & 7)) << 4) +
                                               ((h ^ ((r32 >> 3) & 1)) << 3)) = o;
                else
                    *reinterpret_cast<bf16x4*>(reg + lrow * MX9_PITCH + nl * 2) = o;
            }
            if (SB) __builtin_amdgcn_sched_barrier(0);
        }
    // the wave's own LDS writes precede its reads
    auto rd = [&](int q, int row) __attribute__((always_inline)) -> u16x8 {
        const int lrow = row - ps * BAND;
        if constexpr (SWZ) {  // row & 7 = rr, bit 3 of the row = q & 1
            const u16x8 w = *reinterpret_cast<const u16x8*>(reg + lrow * MX9_PITCH + ((cc ^ rr) << 4));
            return (q & 1) ? u16x8{w[4], w[5], w[6], w[7], w[0], w[1], w[2], w[3]} : w;
        } else {
            return *reinterpret_cast<const u16x8*>(reg + lrow * MX9_PITCH + cc * 16);
        }
    };
    constexpr int QN = 16 / PASSES;
    if (!p.out_mx) {
        bf16* Cout = reinterpret_cast<bf16*>(p.C);
#pragma unroll 4
        for (int q = ps * QN; q < (ps + 1) * QN; ++q) {
            const int row = q * 8 + rr, gr = rm0 + row, gc = cn0 + cc * 8;
            const u16x8 v = rd(q, row);
            if (gr >= p.M || gc >= p.N) continue;
            if (p.res) {
                const int r2 = p.res_period ? gr % p.res_period : gr;
                const u16x8 rv = *reinterpret_cast<const u16x8*>(p.res + (size_t)r2 * p.ldr + gc);
                u16x8 o;
#pragma unroll
                for (int e = 0; e < 8; ++e) o[e] = __builtin_bit_cast(unsigned short, f2bf(bits2f(v[e]) + bits2f(rv[e])));
                __builtin_nontemporal_store(o, reinterpret_cast<u16x8*>(Cout + (size_t)gr * p.ldc + gc));
            } else {
                __builtin_nontemporal_store(v, reinterpret_cast<u16x8*>(Cout + (size_t)gr * p.ldc + gc));
            }
        }
    } else {
        // mx8 output: lanes cc = 0..3 / 4..7 of a row hold its two 32-column blocks
        uint8_t* Cq = reinterpret_cast<uint8_t*>(p.C);
#pragma unroll 4
        for (int q = ps * QN; q < (ps + 1) * QN; ++q) {  // same trip count for every lane (shuffles)
            const int row = q * 8 + rr, gr = rm0 + row, gc = cn0 + cc * 8;
            const u16x8 v = rd(q, row);
            float f[8];
            float a = 0.f;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                f[e] = bits2f(v[e]);
                a = fmaxf(a, fabsf(f[e]));
            }
            const int sbyte = mx_scale_byte(DPPA ? block_amax_dpp(a) : block_amax(a));
            if (gr < p.M && gc < p.N) {
                *reinterpret_cast<uint2*>(Cq + (size_t)gr * p.ldc + gc) = FQ ? mx_pack8_fast(f, sbyte) : mx_pack8(f, sbyte);
                if ((cc & 3) == 0) p.sc[(size_t)(gc >> 5) * p.sc_rows + mx_srow(gr)] = (uint8_t)sbyte;
            }
        }
    }
    }  // passes
}

// WEPI (round 3): the per-wave epilogue above instead of the whole-tile LDS epilogue below; the
// late wave row's closing barrier and the early row's extra one are both dropped (equal counts).
// SC1 (round 3): wave 0 alone DMAs a stage's 1 KiB scale piece (all 64 lanes) instead of every
// wave issuing an 8-lane slice of it: 33 instead of 40 LDS-DMA issues per stage and workgroup;
// wave 0's vmcnt then counts PPW + 1 per stage, the other waves' PPW.
template <int GROUP_M, int ACT, bool WEPI = false, bool SC1 = false>
__global__ __launch_bounds__(512, 2) void gemm_mx_kernel(MxArgs p) {
    using C = MxCfg;
    __shared__ __attribute__((aligned(16))) char lds[WEPI && MXW_LDS > C::LDS ? MXW_LDS : C::LDS];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave / C::WN, wn = wave % C::WN;
    const int h = lane >> 5, r32 = lane & 31;

    const int nbm = (p.M + C::BM - 1) / C::BM;
    const int nbn = (p.N + C::BN - 1) / C::BN;
    const int tile = xcd_remap(blockIdx.x, gridDim.x);
    int bm, bn;
    tile_coords<GROUP_M>(tile, nbm, nbn, bm, bn);
    const int m0 = bm * C::BM, n0 = bn * C::BN;

    // data pieces: 16 rows x 64 B; lane -> row piece*16 + lane/4, physical chunk lane&3
    const uint8_t* src[C::PPW];
#pragma unroll
    for (int q = 0; q < C::PPW; ++q) {
        const int piece = wave * C::PPW + q;
        const bool isA = piece < C::A_PIECES;
        const int prow = (isA ? piece : piece - C::A_PIECES) * 16 + (lane >> 2);
        const int logical = mxswz(prow, lane & 3);
        src[q] = isA ? p.A + (size_t)min(m0 + prow, p.M - 1) * p.lda + logical * 16
                     : p.B + (size_t)min(n0 + prow, p.N - 1) * p.ldb + logical * 16;
    }
    // scale piece: lane L -> part L/16 (A b0, A b1, B b0, B b1), 16 rows (L%16)*16..; this wave owns lanes 8w..8w+7
    const bool sc_mine = SC1 ? wave == 0 : (lane >> 3) == wave;
    const int part = lane >> 4, srow = (lane & 15) * 16;
    const uint8_t* sc_src = part < 2 ? p.sa + (size_t)part * p.sa_rows + m0 + srow
                                     : p.sb + (size_t)(part - 2) * p.sb_rows + n0 + srow;
    const size_t sc_step = part < 2 ? (size_t)2 * p.sa_rows : (size_t)2 * p.sb_rows;  // per stage (2 blocks)

    auto issue = [&](int st) {
        char* base = lds + (st & 3) * C::STAGE;
        const int k0 = st * C::BK;
#pragma unroll
        for (int q = 0; q < C::PPW; ++q) glds16(src[q] + k0, base + (wave * C::PPW + q) * 1024);
        if (SC1) {
            if (wave == 0) glds16(sc_src + st * sc_step, base + C::A_ST + C::B_ST);
        } else if (sc_mine) {
            glds16(sc_src + st * sc_step, base + C::A_ST + C::B_ST);
        }
    };

    const unsigned lds0 = (unsigned)(uintptr_t)(LDS_AS char*)lds;
    const int sw = (lane >> 2) & 3;
    const unsigned c0 = (unsigned)((h ^ sw) << 4), c1 = (unsigned)(((2 + h) ^ sw) << 4);
    const unsigned a_row = lds0 + (wm * C::TM + r32) * 64;
    const unsigned b_row = lds0 + C::A_ST + (wn * C::TN + r32) * 64;
    const unsigned sa_l = lds0 + C::A_ST + C::B_ST + h * 256 + wm * C::TM + r32 * 4;  // mx_srow order
    const unsigned sb_l = lds0 + C::A_ST + C::B_ST + 512 + h * 256 + (wn >> 1) * 128 + r32 * 4 + (wn & 1) * 2;

    f32x16 acc[C::FM][C::FN];
#pragma unroll
    for (int i = 0; i < C::FM; ++i)
#pragma unroll
        for (int j = 0; j < C::FN; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

    const int nk = p.K / C::BK;
    auto wait_rem = [&](int rem) {  // own DMA (PPW + 1 per stage) retired except `rem` later stages
        if (SC1 && wave != 0) {  // SC1: waves 1..7 issue PPW per stage
            if (rem >= 2) vm_wait<2 * C::PPW>();
            else if (rem == 1) vm_wait<C::PPW>();
            else vm_wait<0>();
            return;
        }
        if (rem >= 2) vm_wait<2 * (C::PPW + 1)>();
        else if (rem == 1) vm_wait<C::PPW + 1>();
        else vm_wait<0>();
    };
    // every wave issues PPW + 1 DMA instructions per stage (EXEC-masked scale piece included)
    for (int st = 0; st < 3 && st < nk; ++st) issue(st);
    wait_rem(min(2, nk - 1));
    __builtin_amdgcn_s_barrier();
    if (wm == 1) __builtin_amdgcn_s_barrier();

    for (int t = 0; t < nk; ++t) {
        const unsigned so = (t & 3) * C::STAGE;
        bf16x8 a[C::FM][2], b[C::FN][2];
        unsigned sa[C::FM], sbv[C::FN];
#pragma unroll
        for (int j = 0; j < C::FN; ++j) {
            ds_read16<0>(b[j][0], b_row + so + j * 32 * 64 + c0);
            ds_read16<0>(b[j][1], b_row + so + j * 32 * 64 + c1);
        }
#pragma unroll
        for (int i = 0; i < C::FM; ++i) {
            ds_read16<0>(a[i][0], a_row + so + i * 32 * 64 + c0);
            ds_read16<0>(a[i][1], a_row + so + i * 32 * 64 + c1);
        }
        asm volatile("ds_read_u8 %0, %1 offset:0" : "=v"(sbv[0]) : "v"(sb_l + so) : "memory");
        asm volatile("ds_read_u8 %0, %1 offset:1" : "=v"(sbv[1]) : "v"(sb_l + so) : "memory");
#pragma unroll
        for (int i = 0; i < C::FM; ++i) {
            // offsets i*32 (A) / j*32 (B) as immediates
            if (i == 0) asm volatile("ds_read_u8 %0, %1 offset:0" : "=v"(sa[0]) : "v"(sa_l + so) : "memory");
            if (i == 1) asm volatile("ds_read_u8 %0, %1 offset:1" : "=v"(sa[1]) : "v"(sa_l + so) : "memory");
            if (i == 2) asm volatile("ds_read_u8 %0, %1 offset:2" : "=v"(sa[2]) : "v"(sa_l + so) : "memory");
            if (i == 3) asm volatile("ds_read_u8 %0, %1 offset:3" : "=v"(sa[3]) : "v"(sa_l + so) : "memory");
        }
        if (t + 3 < nk) {
            issue(t + 3);
            wait_rem(2);
        } else {
            wait_rem(max(0, nk - 2 - t));
        }
        lgkm_wait<0>();
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < C::FM; ++i)
#pragma unroll
            for (int j = 0; j < C::FN; ++j) {
                const i32x8 bo = __builtin_bit_cast(i32x8, __builtin_shufflevector(b[j][0], b[j][1], 0, 1, 2, 3, 4,
                                                                                  5, 6, 7, 8, 9, 10, 11, 12, 13,
                                                                                  14, 15));
                const i32x8 ao = __builtin_bit_cast(i32x8, __builtin_shufflevector(a[i][0], a[i][1], 0, 1, 2, 3, 4,
                                                                                  5, 6, 7, 8, 9, 10, 11, 12, 13,
                                                                                  14, 15));
                acc[i][j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(bo, ao, acc[i][j], 0, 0, 0,
                                                                             (int)sbv[j], 0,
                                                                             (int)sa[i]);
            }
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
        if (!(WEPI && wm == 1 && t == nk - 1)) __builtin_amdgcn_s_barrier();
    }
    if constexpr (WEPI) {
        // no LDS hazard: every wave's last fragment reads and DMA waits precede the barrier closing
        // the late row's last memory phase, which the early row passes before it writes its region
        mx_epilogue_wave<ACT>(p, lds, acc, m0, n0, wave, lane);
        return;
    }
    if (wm == 0) __builtin_amdgcn_s_barrier();

    // ---- epilogue: bias + act -> bf16 tile in LDS; lane holds m = i*32 + r32, n = j*32 + 8q + 4h + (0..3)
    __syncthreads();
#pragma unroll
    for (int j = 0; j < C::FN; ++j)
#pragma unroll
        for (int qd = 0; qd < 4; ++qd) {
            const int nl = wn * C::TN + j * 32 + 8 * qd + 4 * h;
            float bv[4] = {0.f, 0.f, 0.f, 0.f};
            if (p.bias) {
#pragma unroll
                for (int r = 0; r < 4; ++r) bv[r] = bf2f(p.bias[min(n0 + nl + r, p.N - 1)]);
            }
#pragma unroll
            for (int i = 0; i < C::FM; ++i) {
                const int ml = wm * C::TM + i * 32 + r32;
                bf16x4 o;
#pragma unroll
                for (int r = 0; r < 4; ++r) o[r] = f2bf(apply_act(acc[i][j][4 * qd + r] + bv[r], ACT));
                *reinterpret_cast<bf16x4*>(lds + ml * C::OUT_LD + nl * 2) = o;
            }
        }
    __syncthreads();
    constexpr int CPR = C::BN / 8;
    if (!p.out_mx) {
        bf16* Cout = reinterpret_cast<bf16*>(p.C);
        for (int c = tid; c < C::BM * CPR; c += C::NT) {
            const int row = c / CPR, cc = c % CPR;
            const int gr = m0 + row, gc = n0 + cc * 8;
            if (gr >= p.M || gc >= p.N) continue;
            u16x8 v = *reinterpret_cast<const u16x8*>(lds + row * C::OUT_LD + cc * 16);
            if (p.res) {
                const int rr = p.res_period ? gr % p.res_period : gr;
                const u16x8 rv = *reinterpret_cast<const u16x8*>(p.res + (size_t)rr * p.ldr + gc);
                bf16x8 o;
#pragma unroll
                for (int e = 0; e < 8; ++e) o[e] = f2bf(bits2f(v[e]) + bits2f(rv[e]));
                *reinterpret_cast<bf16x8*>(Cout + (size_t)gr * p.ldc + gc) = o;
            } else {
                *reinterpret_cast<u16x8*>(Cout + (size_t)gr * p.ldc + gc) = v;
            }
        }
    } else {
        // mx8 output: 4 consecutive threads = one 32-column block of one row (CPR % 4 == 0, NT % 4 == 0)
        uint8_t* Cq = reinterpret_cast<uint8_t*>(p.C);
        for (int c = tid; c < C::BM * CPR; c += C::NT) {  // same trip count for every thread
            const int row = c / CPR, cc = c % CPR;
            const int gr = m0 + row, gc = n0 + cc * 8;
            const u16x8 v = *reinterpret_cast<const u16x8*>(lds + row * C::OUT_LD + cc * 16);
            float f[8];
            float a = 0.f;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                f[e] = bits2f(v[e]);
                a = fmaxf(a, fabsf(f[e]));
            }
            const int sbyte = mx_scale_byte(block_amax(a));
            if (gr < p.M && gc < p.N) {
                *reinterpret_cast<uint2*>(Cq + (size_t)gr * p.ldc + gc) = mx_pack8(f, sbyte);
                if ((cc & 3) == 0) p.sc[(size_t)(gc >> 5) * p.sc_rows + mx_srow(gr)] = (uint8_t)sbyte;
            }
        }
    }
}


// ---------------------------------------------------------------------------
// mx10 (round 3): gemm_mx_kernel's LDS layout, 4-slot ring, K order, MFMA sequence and per-wave
// epilogue (so bit-identical outputs), with pipe9's treatment of the per-stage bookkeeping:
//   * the wave rows (LATE) and the scale-DMA wave (SCW, wave 0) run separate instantiations, so
//     every wait count and barrier is static;
//   * steady-state stages are unrolled by the ring depth (4): ring slots are immediates, and the
//     fragment / scale reads take them as ds offset fields (two bases: slots 0-1 and 2-3, since the
//     field holds 16 bits);
//   * the data pieces are buffer_load_dwordx4 ... lds with per-lane row offsets fixed for the tile
//     and the K offset in soffset (one SGPR add per stage) instead of a 64-bit address per piece.
// Needs K % 64 == 0, K >= 256 (4 stages) and operands < 4 GiB (32-bit offsets).
// ---------------------------------------------------------------------------
template <int ACT, bool LATE, bool SCW, bool ESWZ = true>
__device__ __forceinline__ void mx10_tile(const MxArgs& p, char* lds, const int m0, const int n0, const int wave) {
    using C = MxCfg;
    static_assert(C::PPW == 4 && C::NSTAGE == 4, "mx10: 4 data pieces per wave, 4-slot ring");
    const int lane = threadIdx.x & 63;
    const int wm = wave / C::WN, wn = wave % C::WN;
    const int h = lane >> 5, r32 = lane & 31;
    // data pieces: waves 0-3 carry A, waves 4-7 B; piece q = 16 rows x 64 B, lane -> row lane / 4
    const bool isA = wave < 4;
    unsigned voff[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int prow = ((wave & 3) * 4 + q) * 16 + (lane >> 2);
        const int logical = mxswz(prow, lane & 3);
        voff[q] = isA ? (unsigned)min(m0 + prow, p.M - 1) * (unsigned)p.lda + logical * 16
                      : (unsigned)min(n0 + prow, p.N - 1) * (unsigned)p.ldb + logical * 16;
    }
    const i32x4v rs = isA ? mx_rsrc(p.A, (unsigned)((size_t)p.M * p.lda)) : mx_rsrc(p.B, (unsigned)((size_t)p.N * p.ldb));
    // scale piece (wave 0, all lanes): part = lane / 16 (A b0, A b1, B b0, B b1), rows (lane % 16) * 16..
    const int part = lane >> 4, srow = (lane & 15) * 16;
    const uint8_t* sc_src = part < 2 ? p.sa + (size_t)part * p.sa_rows + m0 + srow
                                     : p.sb + (size_t)(part - 2) * p.sb_rows + n0 + srow;
    const size_t sc_step = part < 2 ? (size_t)2 * p.sa_rows : (size_t)2 * p.sb_rows;
    const unsigned lds0 = (unsigned)(uintptr_t)(LDS_AS char*)lds;
    const unsigned lw = __builtin_amdgcn_readfirstlane(lds0 + wave * 4096);
    char* lds_sc = lds + C::A_ST + C::B_ST;  // + slot * STAGE

    const int sw = (lane >> 2) & 3;
    const unsigned c0 = (unsigned)((h ^ sw) << 4), c1 = (unsigned)(((2 + h) ^ sw) << 4);
    // two bases per operand: slots 0 / 1 at base + {0, STAGE}, slots 2 / 3 at base2 + {0, STAGE}
    const unsigned a0 = lds0 + (wm * C::TM + r32) * 64 + c0, a1 = lds0 + (wm * C::TM + r32) * 64 + c1;
    const unsigned b0 = lds0 + C::A_ST + (wn * C::TN + r32) * 64 + c0, b1 = lds0 + C::A_ST + (wn * C::TN + r32) * 64 + c1;
    const unsigned sa_l = lds0 + C::A_ST + C::B_ST + h * 256 + wm * C::TM + r32 * 4;  // mx_srow order
    const unsigned sb_l = lds0 + C::A_ST + C::B_ST + 512 + h * 256 + (wn >> 1) * 128 + r32 * 4 + (wn & 1) * 2;
    constexpr unsigned HI = 2 * C::STAGE;

    f32x16 acc[C::FM][C::FN];
#pragma unroll
    for (int i = 0; i < C::FM; ++i)
#pragma unroll
        for (int j = 0; j < C::FN; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

    constexpr int PER = C::PPW + (SCW ? 1 : 0);  // this wave's DMA instructions per stage
    auto wait = [&](int rem) __attribute__((always_inline)) {
        if (rem >= 2) vm_wait<2 * PER>();
        else if (rem == 1) vm_wait<PER>();
        else vm_wait<0>();
    };
    auto issue = [&](int st, int slot) __attribute__((always_inline)) {  // slot: run-time or immediate
        mx_dma4(lw + (unsigned)slot * C::STAGE, voff, rs, (unsigned)st * C::BK);
        if (SCW) glds16(sc_src + st * sc_step, lds_sc + slot * C::STAGE);
    };
    // one stage: fragment / scale reads of slot SL (reads at base + OFF, OFF an immediate),
    // optional DMA of stage `ist` into slot `isl`, counted wait, barrier, 8 MFMAs, barrier
    auto stage = [&](auto SLc, unsigned abase0, unsigned abase1, unsigned bbase0, unsigned bbase1, unsigned sab,
                     unsigned sbb, bool dma, int ist, int isl, int rem, bool end_barrier) __attribute__((always_inline)) {
        constexpr int OFF = decltype(SLc)::value;
        bf16x8 a[C::FM][2], b[C::FN][2];
        unsigned sa[C::FM], sbv[C::FN];
        ds_read16<OFF + 0 * 2048>(b[0][0], bbase0);
        ds_read16<OFF + 0 * 2048>(b[0][1], bbase1);
        ds_read16<OFF + 1 * 2048>(b[1][0], bbase0);
        ds_read16<OFF + 1 * 2048>(b[1][1], bbase1);
#pragma unroll
        for (int i = 0; i < C::FM; ++i) {
            if (i == 0) { ds_read16<OFF + 0 * 2048>(a[0][0], abase0); ds_read16<OFF + 0 * 2048>(a[0][1], abase1); }
            if (i == 1) { ds_read16<OFF + 1 * 2048>(a[1][0], abase0); ds_read16<OFF + 1 * 2048>(a[1][1], abase1); }
            if (i == 2) { ds_read16<OFF + 2 * 2048>(a[2][0], abase0); ds_read16<OFF + 2 * 2048>(a[2][1], abase1); }
            if (i == 3) { ds_read16<OFF + 3 * 2048>(a[3][0], abase0); ds_read16<OFF + 3 * 2048>(a[3][1], abase1); }
        }
        asm volatile("ds_read_u8 %0, %1 offset:%2" : "=v"(sbv[0]) : "v"(sbb), "n"(OFF + 0) : "memory");
        asm volatile("ds_read_u8 %0, %1 offset:%2" : "=v"(sbv[1]) : "v"(sbb), "n"(OFF + 1) : "memory");
        asm volatile("ds_read_u8 %0, %1 offset:%2" : "=v"(sa[0]) : "v"(sab), "n"(OFF + 0) : "memory");
        asm volatile("ds_read_u8 %0, %1 offset:%2" : "=v"(sa[1]) : "v"(sab), "n"(OFF + 1) : "memory");
        asm volatile("ds_read_u8 %0, %1 offset:%2" : "=v"(sa[2]) : "v"(sab), "n"(OFF + 2) : "memory");
        asm volatile("ds_read_u8 %0, %1 offset:%2" : "=v"(sa[3]) : "v"(sab), "n"(OFF + 3) : "memory");
        if (dma) issue(ist, isl);
        wait(rem);
        lgkm_wait<0>();
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < C::FM; ++i)
#pragma unroll
            for (int j = 0; j < C::FN; ++j) {
                const i32x8 bo = __builtin_bit_cast(i32x8, __builtin_shufflevector(b[j][0], b[j][1], 0, 1, 2, 3, 4, 5, 6,
                                                                                  7, 8, 9, 10, 11, 12, 13, 14, 15));
                const i32x8 ao = __builtin_bit_cast(i32x8, __builtin_shufflevector(a[i][0], a[i][1], 0, 1, 2, 3, 4, 5, 6,
                                                                                  7, 8, 9, 10, 11, 12, 13, 14, 15));
                acc[i][j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(bo, ao, acc[i][j], 0, 0, 0, (int)sbv[j], 0,
                                                                             (int)sa[i]);
            }
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
        if (end_barrier) __builtin_amdgcn_s_barrier();
    };
    using S0 = IC2<0>;
    using S1 = IC2<C::STAGE>;
    const int nk = p.K / C::BK;

    // prologue: stages 0..2 into slots 0..2
    issue(0, 0);
    issue(1, 1);
    issue(2, 2);
    wait(2);  // stage 0 landed
    __builtin_amdgcn_s_barrier();
    if (LATE) __builtin_amdgcn_s_barrier();

    // steady state: stage t (slot t & 3) issues stage t + 3 into slot (t + 3) & 3 while t + 3 < nk
    int t = 0;
    for (; t + 4 <= nk - 3; t += 4) {
        stage(S0{}, a0, a1, b0, b1, sa_l, sb_l, true, t + 3, 3, 2, true);
        stage(S1{}, a0, a1, b0, b1, sa_l, sb_l, true, t + 4, 0, 2, true);
        stage(S0{}, a0 + HI, a1 + HI, b0 + HI, b1 + HI, sa_l + HI, sb_l + HI, true, t + 5, 1, 2, true);
        stage(S1{}, a0 + HI, a1 + HI, b0 + HI, b1 + HI, sa_l + HI, sb_l + HI, true, t + 6, 2, 2, true);
    }
    // remaining steady stages (0..3) and the last three stages: run-time slots (base + slot * STAGE)
    for (; t < nk; ++t) {
        const unsigned so = (unsigned)(t & 3) * C::STAGE;
        const bool dma = t + 3 < nk;
        const int rem = dma ? 2 : (nk - 2 - t > 0 ? nk - 2 - t : 0);
        stage(S0{}, a0 + so, a1 + so, b0 + so, b1 + so, sa_l + so, sb_l + so, dma, t + 3, (t + 3) & 3, rem,
              !(LATE && t == nk - 1));
    }
    // no LDS hazard: every wave's last fragment reads and DMA waits precede the barrier closing the
    // late row's last memory phase, which the early row passes before it writes its region
    mx_epilogue_wave<ACT, ESWZ>(p, lds, acc, m0, n0, wave, lane);
}

template <int GROUP_M, int ACT, bool ESWZ = true>
__global__ __launch_bounds__(512, 2) void gemm_mx10_kernel(MxArgs p) {
    using C = MxCfg;
    __shared__ __attribute__((aligned(16))) char lds[MXW_LDS > C::LDS ? MXW_LDS : C::LDS];
    const int nbm = (p.M + C::BM - 1) / C::BM, nbn = (p.N + C::BN - 1) / C::BN;
    const int tile = xcd_remap(blockIdx.x, gridDim.x);
    int bm, bn;
    tile_coords<GROUP_M>(tile, nbm, nbn, bm, bn);
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (wave == 0)
        mx10_tile<ACT, false, true, ESWZ>(p, lds, bm * C::BM, bn * C::BN, wave);
    else if (wave < 4)
        mx10_tile<ACT, false, false, ESWZ>(p, lds, bm * C::BM, bn * C::BN, wave);
    else
        mx10_tile<ACT, true, false, ESWZ>(p, lds, bm * C::BM, bn * C::BN, wave);
}

template <int GROUP_M, bool ESWZ = true>
int launch_mx10(const MxArgs& a, hipStream_t s) {
    const dim3 grid(((a.M + 255) / 256) * ((a.N + 255) / 256)), block(512);
    switch (a.act) {
        case MME_ACT_GELU_TANH:
            hipLaunchKernelGGL((gemm_mx10_kernel<GROUP_M, MME_ACT_GELU_TANH, ESWZ>), grid, block, 0, s, a);
            break;
        case MME_ACT_QUICK_GELU:
            hipLaunchKernelGGL((gemm_mx10_kernel<GROUP_M, MME_ACT_QUICK_GELU, ESWZ>), grid, block, 0, s, a);
            break;
        case MME_ACT_GELU_ERF:
            hipLaunchKernelGGL((gemm_mx10_kernel<GROUP_M, MME_ACT_GELU_ERF, ESWZ>), grid, block, 0, s, a);
            break;
        default:
            hipLaunchKernelGGL((gemm_mx10_kernel<GROUP_M, MME_ACT_NONE, ESWZ>), grid, block, 0, s, a);
            break;
    }
    return mme_check_launch("mme_gemm_mx");
}

// ---------------------------------------------------------------------------
// mx11 (round 4): the block-scaled fp8 GEMM on pipe9's LDS ring and schedule (gemm.hip).
// fp8 values are one byte, so a 128-deep fp8 stage of 256 rows is one 32 KiB unit of whole
// 128-B cache-line rows -- exactly pipe9's unit. The ring is pipe9's (five units: A of stage s in
// slot 2s mod 5, B in 2s + 1 mod 5, all 160 KiB of LDS), with pipe9's DMA pieces (8 rows x 128 B,
// chunk swizzle c ^ ((row >> 1) & 7): the 32-row fragment reads below hit 16 distinct 16-B bank
// slots per ds_read_b128 lane group), ping-pong wave rows (LATE), static waits / barriers and
// soffset-stepped buffer_load ... lds. A stage runs as two 64-deep k-steps, each a memory phase
// (12 ds_read_b128: lane (r, h) reads logical chunks 4 ks + h and 4 ks + 2 + h of its rows, the
// v_mfma_scale_f32_32x32x64_f8f6f4 operand layout of mx10) and a compute phase of 8 MFMAs
// (4 x 2 tiles of 32 x 32): per k-step the same LDS bytes, ds_reads and MFMA cycles as one pipe9
// step, at twice the FLOPs. The K order and MFMA chains are mx10's, so the outputs are bit-identical
// to mx10 (tests/test_gpu_mx.py).
// Scales leave LDS (mx9 kept them there and lost a ring slot: -10 %): the planes' mx_srow row order
// puts the 4 bytes lane (r, h) needs for rows i * 32 + r of one block in one aligned dword, so a
// stage costs 4 buffer_load_dword per lane (A and B, blocks 4 s + h and 4 s + 2 + h), issued one
// stage ahead with the B unit of the next stage and retired by the same counted vmcnt; the MFMA's
// scale op_sel picks the byte (A: i; B: j after a 16-bit shift for odd wn).
// Needs K % 128 == 0, K >= 384 (three stages) and operands < 4 GiB (32-bit offsets).
// ---------------------------------------------------------------------------
template <bool PAD = false>
__device__ __forceinline__ unsigned mx_sload(unsigned voff, i32x4v rsrc, unsigned soff) {
    unsigned v;
    if (PAD)  // mx_dma4's PAD: the nops inside the statement, so nothing is scheduled between them and the load
        asm volatile("s_nop 4\n\tbuffer_load_dword %0, %1, %2, %3 offen" : "=v"(v) : "v"(voff), "s"(rsrc), "s"(soff) : "memory");
    else
        asm volatile("buffer_load_dword %0, %1, %2, %3 offen" : "=v"(v) : "v"(voff), "s"(rsrc), "s"(soff) : "memory");
    return v;
}
// counted vmcnt that also marks the scale registers loaded by inline asm as written here, so no
// use of them can be scheduled before the wait that retires their loads
template <int N>
__device__ __forceinline__ void vm_wait_sc(unsigned (&sc)[4]) {
    asm volatile("s_waitcnt vmcnt(%4)" : "+v"(sc[0]), "+v"(sc[1]), "+v"(sc[2]), "+v"(sc[3]) : "n"(N) : "memory");
}
template <int I, int J>
__device__ __forceinline__ void mx11_mfma(f32x16& acc, const bf16x8 (&a)[2], const bf16x8 (&b)[2], unsigned sa,
                                          unsigned sb) {
    const i32x8 bo = __builtin_bit_cast(i32x8, __builtin_shufflevector(b[0], b[1], 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10,
                                                                       11, 12, 13, 14, 15));
    const i32x8 ao = __builtin_bit_cast(i32x8, __builtin_shufflevector(a[0], a[1], 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10,
                                                                       11, 12, 13, 14, 15));
    acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(bo, ao, acc, 0, 0, J, (int)sb, I, (int)sa);
}

template <int ACT, bool LATE, bool BPRE = false, bool DPPA = false, bool FQ = false>
__device__ __forceinline__ void mx11_tile(const MxArgs& p, char* lds, const int m0, const int n0, const int wave) {
    constexpr int UNIT = 32768;
    const int lane = threadIdx.x & 63;
    const int wm = wave / 4, wn = wave % 4;
    const int h = lane >> 5, r32 = lane & 31;

    unsigned offA[4], offB[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int prow = (wave * 4 + q) * 8 + (lane >> 3);
        const int logical = swz(prow, lane & 7);
        offA[q] = (unsigned)min(m0 + prow, p.M - 1) * (unsigned)p.lda + logical * 16;
        offB[q] = (unsigned)min(n0 + prow, p.N - 1) * (unsigned)p.ldb + logical * 16;
    }
    const i32x4v rA = mx_rsrc(p.A, (unsigned)((size_t)p.M * p.lda));
    const i32x4v rB = mx_rsrc(p.B, (unsigned)((size_t)p.N * p.ldb));
    // scale dwords: A rows m0 + wm 128 + {0, 32, 64, 96} + r32 of block b at plane b, bytes
    // m0 + wm 128 + 4 r32 + i; B columns n0 + wn 64 + {0, 32} + r32 at n0 + (wn / 2) 128 + 4 r32 + 2 (wn & 1) + j
    const i32x4v rSA = mx_rsrc(p.sa, (unsigned)((size_t)(p.K / 32) * p.sa_rows));
    const i32x4v rSB = mx_rsrc(p.sb, (unsigned)((size_t)(p.K / 32) * p.sb_rows));
    const unsigned vsa = (unsigned)(h * p.sa_rows + m0 + wm * 128 + 4 * r32);
    const unsigned vsb = (unsigned)(h * p.sb_rows + n0 + (wn >> 1) * 128 + 4 * r32);
    const unsigned sstepA = 4u * p.sa_rows, sstepB = 4u * p.sb_rows, bshift = (wn & 1) * 16;
    const unsigned s2A = 2u * p.sa_rows, s2B = 2u * p.sb_rows;  // k-step 1's blocks: two planes further

    const unsigned lds0 = (unsigned)(uintptr_t)(LDS_AS char*)lds;
    const unsigned lw = __builtin_amdgcn_readfirstlane(lds0 + wave * 4096);
    const int sw = (r32 >> 1) & 7;  // fragment rows differ by multiples of 32: the swizzle depends on r32
    // logical chunk c of the lane's row sits at chunk c ^ sw; with x = h ^ sw the k-step ks chunks
    // 4 ks + h + {0, 2} are at (x ^ (4 ks + {0, 2})), i.e. base_x ^ ((4 ks + {0, 2}) << 4) with
    // base_x = row base + (x << 4) (128-B aligned rows: no carries), and the XOR commutes with the
    // fragment (i * 4 KiB) and slot (32 KiB) offsets: two base registers, one v_xor per read address
    const unsigned a_x = lds0 + (wm * 128 + r32) * 128 + ((h ^ sw) << 4);
    const unsigned b_x = lds0 + (wn * 64 + r32) * 128 + ((h ^ sw) << 4);

    f32x16 acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
    const int nk = p.K / 128;
    unsigned cur[4], nxt[4];  // scale dwords of this / the next stage: A ks 0, A ks 1, B ks 0, B ks 1
    unsigned kscA = 0, kscB = 0;  // soffsets of the next scales to load (A / B planes)

    auto load_sc = [&](unsigned (&d)[4]) __attribute__((always_inline)) {
        d[0] = mx_sload(vsa, rSA, kscA);
        d[1] = mx_sload(vsa, rSA, kscA + s2A);
        d[2] = mx_sload(vsb, rSB, kscB);
        d[3] = mx_sload(vsb, rSB, kscB + s2B);
        kscA += sstepA;
        kscB += sstepB;
    };
    // one 64-deep k-step: memory phase (12 fragment reads, optionally the next stage's scales and
    // a DMA unit), barrier, compute phase (8 MFMAs), barrier. wm_ / wc_: vmcnt kept after the
    // memory / compute phase (-1: no wait); the waits that retire a scale load tie nxt.
    auto step = [&](unsigned aa0, unsigned aa1, unsigned bb0, unsigned bb1, unsigned sa, unsigned sb, bool scl,
                    bool dma, unsigned m0base, const unsigned (&voff)[4], i32x4v rs, unsigned soff, int wm_, int wc_,
                    bool end_barrier) __attribute__((always_inline)) {
        bf16x8 a[4][2], b[2][2];
        ds_read16<0>(b[0][0], bb0);
        ds_read16<0>(b[0][1], bb1);
        ds_read16<4096>(b[1][0], bb0);
        ds_read16<4096>(b[1][1], bb1);
        ds_read16<0>(a[0][0], aa0);
        ds_read16<0>(a[0][1], aa1);
        ds_read16<4096>(a[1][0], aa0);
        ds_read16<4096>(a[1][1], aa1);
        ds_read16<8192>(a[2][0], aa0);
        ds_read16<8192>(a[2][1], aa1);
        ds_read16<12288>(a[3][0], aa0);
        ds_read16<12288>(a[3][1], aa1);
        if (scl) load_sc(nxt);
        if (dma) mx_dma4(m0base, voff, rs, soff);
        if (wm_ == 0) vm_wait_sc<0>(nxt);
        else if (wm_ == 4) vm_wait_sc<4>(nxt);
        lgkm_wait<0>();
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_s_setprio(1);
        const unsigned sbs = sb >> bshift;
        mx11_mfma<0, 0>(acc[0][0], a[0], b[0], sa, sbs);
        mx11_mfma<0, 1>(acc[0][1], a[0], b[1], sa, sbs);
        mx11_mfma<1, 0>(acc[1][0], a[1], b[0], sa, sbs);
        mx11_mfma<1, 1>(acc[1][1], a[1], b[1], sa, sbs);
        mx11_mfma<2, 0>(acc[2][0], a[2], b[0], sa, sbs);
        mx11_mfma<2, 1>(acc[2][1], a[2], b[1], sa, sbs);
        mx11_mfma<3, 0>(acc[3][0], a[3], b[0], sa, sbs);
        mx11_mfma<3, 1>(acc[3][1], a[3], b[1], sa, sbs);
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
        if (wc_ == 0) vm_wait_sc<0>(nxt);
        else if (wc_ == 4) vm_wait_sc<4>(nxt);
        if (end_barrier) __builtin_amdgcn_s_barrier();
    };
    // soffset (bytes along K) of the B unit (stage s + 1) / A unit (s + 2) that stage s issues: from
    // stage 1 on (stage 0's successors B1 and A2 come from the prologue)
    unsigned kB = 256, kA = 384;
    // stage with its A in slot sa (B in sa + 1): issue B(s + 1) (+ its scales) into slot sa + 3, A(s + 2)
    // into sa + 4 (mod 5); need: this wave's loads kept in flight at the barrier before stage s + 1
    auto stage = [&](int sa, bool dB, bool scl, bool dA, int need, bool last) __attribute__((always_inline)) {
        const int sb = sa == 4 ? 0 : sa + 1;
        const int iB = sa + 3 >= 5 ? sa - 2 : sa + 3, iA = sa + 4 >= 5 ? sa - 1 : sa + 4;
        const unsigned as = a_x + sa * UNIT, bs = b_x + sb * UNIT;
        step(as, as ^ (2u << 4), bs, bs ^ (2u << 4), cur[0], cur[2], scl, dB, lw + iB * UNIT, offB, rB, kB, -1, -1,
             true);
        step(as ^ (4u << 4), as ^ (6u << 4), bs ^ (4u << 4), bs ^ (6u << 4), cur[1], cur[3], false, dA,
             lw + iA * UNIT, offA, rA, kA, LATE ? need : -1, LATE ? -1 : need, !(LATE && last));
        kB += 128;
        kA += 128;
#pragma unroll
        for (int q = 0; q < 4; ++q) cur[q] = nxt[q];
    };

    // prologue: scales of stage 0, units 0 and 1 (stage 0), scales of stage 1, units 2..4 (A1 B1 A2)
    load_sc(cur);
    mx_dma4(lw + 0 * UNIT, offA, rA, 0);
    mx_dma4(lw + 1 * UNIT, offB, rB, 0);
    load_sc(nxt);
    mx_dma4(lw + 2 * UNIT, offA, rA, 128);
    mx_dma4(lw + 3 * UNIT, offB, rB, 128);
    mx_dma4(lw + 4 * UNIT, offA, rA, 256);
    vm_wait_sc<12>(cur);  // stage 0's scales and units landed (and stage 1's scales)
    vm_wait_sc<12>(nxt);
    __builtin_amdgcn_s_barrier();
    if (LATE) __builtin_amdgcn_s_barrier();

    {  // stage 0: its successors' units were issued in the prologue; cur <- stage 1's scales
        const unsigned c0 = cur[0], c1 = cur[1], c2 = cur[2], c3 = cur[3];
        const unsigned bs = b_x + UNIT;
        step(a_x, a_x ^ (2u << 4), bs, bs ^ (2u << 4), c0, c2, false, false, 0, offB, rB, 0, -1, -1, true);
        step(a_x ^ (4u << 4), a_x ^ (6u << 4), bs ^ (4u << 4), bs ^ (6u << 4), c1, c3, false, false, 0, offA, rA, 0,
             LATE ? 4 : -1, LATE ? -1 : 4, true);
#pragma unroll
        for (int q = 0; q < 4; ++q) cur[q] = nxt[q];
    }
    int s = 1;
    // from here the scales of stage s + 1 are loaded in stage s (kscA / kscB at stage 2's)
    for (; s + 5 <= nk - 2; s += 5) {  // steady state: s = 1 (mod 5) -> A slots 2, 4, 1, 3, 0
        stage(2, true, true, true, 4, false);
        stage(4, true, true, true, 4, false);
        stage(1, true, true, true, 4, false);
        stage(3, true, true, true, 4, false);
        stage(0, true, true, true, 4, false);
    }
    if (s < nk - 2) {
        stage(2, true, true, true, 4, false);
        if (++s < nk - 2) {
            stage(4, true, true, true, 4, false);
            if (++s < nk - 2) {
                stage(1, true, true, true, 4, false);
                if (++s < nk - 2) {
                    stage(3, true, true, true, 4, false);
                    ++s;
                }
            }
        }
    }
    // s = nk - 2: B and the scales of the last stage only; s = nk - 1: nothing (ring slots at run time)
    const int sa2 = (2 * s) % 5, sa1 = sa2 >= 3 ? sa2 - 3 : sa2 + 2;
    stage(sa2, true, true, false, 0, false);
    stage(sa1, false, false, false, -1, true);
    vm_wait<0>();
    // the accumulators pass through an empty asm here: without it the last stage's MFMAs are sunk
    // into the epilogue's branches, holding their fragments live beside the epilogue (VGPR spills)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) asm volatile("" : "+v"(acc[i][j]));
    // no LDS hazard: every wave's last fragment reads precede the barrier closing the late row's
    // last memory phase, which the early row passes before it writes its epilogue region
    mx_epilogue_wave<ACT, true, true, 1, BPRE, DPPA, FQ>(p, lds, acc, m0, n0, wave, lane);
}

template <int GROUP_M, int ACT, bool BPRE = false, bool DPPA = false, bool FQ = false>
__global__ __launch_bounds__(512, 2) void gemm_mx11_kernel(MxArgs p) {
    __shared__ __attribute__((aligned(16))) char lds[5 * 32768];
    const int nbm = (p.M + 255) / 256, nbn = (p.N + 255) / 256;
    const int tile = xcd_remap(blockIdx.x, gridDim.x);
    int bm, bn;
    tile_coords<GROUP_M>(tile, nbm, nbn, bm, bn);
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (wave >= 4)
        mx11_tile<ACT, true, BPRE, DPPA, FQ>(p, lds, bm * 256, bn * 256, wave);
    else
        mx11_tile<ACT, false, BPRE, DPPA, FQ>(p, lds, bm * 256, bn * 256, wave);
}

template <int GROUP_M, bool BPRE = false, bool DPPA = false, bool FQ = false>
int launch_mx11(const MxArgs& a, hipStream_t s) {
    const dim3 grid(((a.M + 255) / 256) * ((a.N + 255) / 256)), block(512);
    switch (a.act) {
        case MME_ACT_GELU_TANH:
            hipLaunchKernelGGL((gemm_mx11_kernel<GROUP_M, MME_ACT_GELU_TANH, BPRE, DPPA, FQ>), grid, block, 0, s, a);
            break;
        case MME_ACT_QUICK_GELU:
            hipLaunchKernelGGL((gemm_mx11_kernel<GROUP_M, MME_ACT_QUICK_GELU, BPRE, DPPA, FQ>), grid, block, 0, s, a);
            break;
        case MME_ACT_GELU_ERF:
            hipLaunchKernelGGL((gemm_mx11_kernel<GROUP_M, MME_ACT_GELU_ERF, BPRE, DPPA, FQ>), grid, block, 0, s, a);
            break;
        default:
            hipLaunchKernelGGL((gemm_mx11_kernel<GROUP_M, MME_ACT_NONE, BPRE, DPPA, FQ>), grid, block, 0, s, a);
            break;
    }
    return mme_check_launch("mme_gemm_mx");
}


// ---------------------------------------------------------------------------
// mx12 (round 5): persistent mx11, as pipe10 is persistent pipe9 (gemm.hip). One workgroup per CU
// walks mx11's tile order (xcd_remap of the same ids: every tile on the XCD it would run on as an
// mx11 block) with mx11's main loop, K order, MFMAs and epilogue arithmetic per tile (bit-identical
// outputs). At the seam between tiles the next tile's first three ring units (A0 B0 A1) are DMA'd
// as soon as this tile's last fragment reads are done, i.e. under its epilogue, which stages through
// slots 3-4 only (two 64-row passes); after it every wave waits for its own loads, one barrier frees
// slots 3-4, and the next tile's scales and units B1 A2 follow.
// Measured (round 5, profiles/r05_v12_mx12_gemm.log, r05_v12_fp8_mx12_job_ab.log): bit-identical to mx11 but slower on
// every DFN5B-H shape with the job's epilogues (QKV 1.45 -> 1.49, fc1 2.30 -> 2.35-2.40, fc2 1.74 ->
// 1.78-1.81 ms; the fp8 job 1 172-1 174 -> 1 160-1 162 img/s): the persistent loop holds 255 VGPRs and
// spills 25-40 SGPRs, whose reloads feed the asm loads (next paragraph), so the seam it hides costs more
// than it saves. Not dispatched (form 12; form 14 = no DMA under the epilogue).
// Hazard found building it: the SGPR-spill reloads are v_readlane writes of the SGPRs that the inline-asm
// buffer loads read as soffset; the hardware needs 5 wait states between the two, hipcc pads only
// instructions it generates, and unpadded the scale loads read stale offsets -- the early wave row's
// outputs came out wrong on some tiles of some launches (profiles/r05_v15_*, r05_v16_*). mx12's asm loads
// open with s_nop 4 (PAD); tools/asm_hazard_audit.py checks every kernel of the library for the pattern
// (tests/test_abi.py::test_no_unpadded_sgpr_vmem_hazards; 12 of 12 runs identical after the fix,
// profiles/r05_v17_mx12_hazard_fixed_debug.log).
// ---------------------------------------------------------------------------
// SEAM (dev A/B): 0 = as described; 2 = no DMA under the epilogue (every tile's A0 B0 A1 at its prologue).
template <int GROUP_M, int ACT, bool LATE, int SEAM = 0>
__device__ __forceinline__ void mx12_run(const MxArgs& p, char* lds, const int wave) {
    constexpr int UNIT = 32768;
    const int lane = threadIdx.x & 63;
    const int wm = wave / 4, wn = wave % 4;
    const int h = lane >> 5, r32 = lane & 31;
    const int nbm = (p.M + 255) / 256, nbn = (p.N + 255) / 256, ntiles = nbm * nbn;

    const i32x4v rA = mx_rsrc(p.A, (unsigned)((size_t)p.M * p.lda));
    const i32x4v rB = mx_rsrc(p.B, (unsigned)((size_t)p.N * p.ldb));
    const i32x4v rSA = mx_rsrc(p.sa, (unsigned)((size_t)(p.K / 32) * p.sa_rows));
    const i32x4v rSB = mx_rsrc(p.sb, (unsigned)((size_t)(p.K / 32) * p.sb_rows));
    const unsigned sstepA = 4u * p.sa_rows, sstepB = 4u * p.sb_rows, bshift = (wn & 1) * 16;
    const unsigned s2A = 2u * p.sa_rows, s2B = 2u * p.sb_rows;
    const unsigned lds0 = (unsigned)(uintptr_t)(LDS_AS char*)lds;
    const unsigned lw = __builtin_amdgcn_readfirstlane(lds0 + wave * 4096);
    const int sw = (r32 >> 1) & 7;
    const unsigned a_x = lds0 + (wm * 128 + r32) * 128 + ((h ^ sw) << 4);
    const unsigned b_x = lds0 + (wn * 64 + r32) * 128 + ((h ^ sw) << 4);
    const int nk = p.K / 128;

    unsigned offA[4], offB[4], vsa = 0, vsb = 0;
    auto set_off = [&](int m0, int n0) __attribute__((always_inline)) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int prow = (wave * 4 + q) * 8 + (lane >> 3);
            const int logical = swz(prow, lane & 7);
            offA[q] = (unsigned)min(m0 + prow, p.M - 1) * (unsigned)p.lda + logical * 16;
            offB[q] = (unsigned)min(n0 + prow, p.N - 1) * (unsigned)p.ldb + logical * 16;
        }
        vsa = (unsigned)(h * p.sa_rows + m0 + wm * 128 + 4 * r32);
        vsb = (unsigned)(h * p.sb_rows + n0 + (wn >> 1) * 128 + 4 * r32);
    };
    auto coords = [&](int v, int& m0, int& n0) __attribute__((always_inline)) {
        int bm, bn;
        tile_coords<GROUP_M>(xcd_remap(v, ntiles), nbm, nbn, bm, bn);
        m0 = bm * 256;
        n0 = bn * 256;
    };

    f32x16 acc[4][2];
    unsigned cur[4], nxt[4];
    unsigned kscA = 0, kscB = 0;
    auto load_sc = [&](unsigned (&d)[4]) __attribute__((always_inline)) {
        d[0] = mx_sload<true>(vsa, rSA, kscA);
        d[1] = mx_sload<true>(vsa, rSA, kscA + s2A);
        d[2] = mx_sload<true>(vsb, rSB, kscB);
        d[3] = mx_sload<true>(vsb, rSB, kscB + s2B);
        kscA += sstepA;
        kscB += sstepB;
    };
    // mx11's k-step and stage (mx11_tile), unchanged
    auto step = [&](unsigned aa0, unsigned aa1, unsigned bb0, unsigned bb1, unsigned sa, unsigned sb, bool scl,
                    bool dma, unsigned m0base, const unsigned (&voff)[4], i32x4v rs, unsigned soff, int wm_, int wc_,
                    bool end_barrier) __attribute__((always_inline)) {
        bf16x8 a[4][2], b[2][2];
        ds_read16<0>(b[0][0], bb0);
        ds_read16<0>(b[0][1], bb1);
        ds_read16<4096>(b[1][0], bb0);
        ds_read16<4096>(b[1][1], bb1);
        ds_read16<0>(a[0][0], aa0);
        ds_read16<0>(a[0][1], aa1);
        ds_read16<4096>(a[1][0], aa0);
        ds_read16<4096>(a[1][1], aa1);
        ds_read16<8192>(a[2][0], aa0);
        ds_read16<8192>(a[2][1], aa1);
        ds_read16<12288>(a[3][0], aa0);
        ds_read16<12288>(a[3][1], aa1);
        if (scl) load_sc(nxt);
        if (dma) mx_dma4<true>(m0base, voff, rs, soff);
        if (wm_ == 0) vm_wait_sc<0>(nxt);
        else if (wm_ == 4) vm_wait_sc<4>(nxt);
        lgkm_wait<0>();
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_s_setprio(1);
        const unsigned sbs = sb >> bshift;
        mx11_mfma<0, 0>(acc[0][0], a[0], b[0], sa, sbs);
        mx11_mfma<0, 1>(acc[0][1], a[0], b[1], sa, sbs);
        mx11_mfma<1, 0>(acc[1][0], a[1], b[0], sa, sbs);
        mx11_mfma<1, 1>(acc[1][1], a[1], b[1], sa, sbs);
        mx11_mfma<2, 0>(acc[2][0], a[2], b[0], sa, sbs);
        mx11_mfma<2, 1>(acc[2][1], a[2], b[1], sa, sbs);
        mx11_mfma<3, 0>(acc[3][0], a[3], b[0], sa, sbs);
        mx11_mfma<3, 1>(acc[3][1], a[3], b[1], sa, sbs);
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
        if (wc_ == 0) vm_wait_sc<0>(nxt);
        else if (wc_ == 4) vm_wait_sc<4>(nxt);
        if (end_barrier) __builtin_amdgcn_s_barrier();
    };
    unsigned kB, kA;
    auto stage = [&](int sa, bool dB, bool scl, bool dA, int need, bool last) __attribute__((always_inline)) {
        const int sb = sa == 4 ? 0 : sa + 1;
        const int iB = sa + 3 >= 5 ? sa - 2 : sa + 3, iA = sa + 4 >= 5 ? sa - 1 : sa + 4;
        const unsigned as = a_x + sa * UNIT, bs = b_x + sb * UNIT;
        step(as, as ^ (2u << 4), bs, bs ^ (2u << 4), cur[0], cur[2], scl, dB, lw + iB * UNIT, offB, rB, kB, -1, -1,
             true);
        step(as ^ (4u << 4), as ^ (6u << 4), bs ^ (4u << 4), bs ^ (6u << 4), cur[1], cur[3], false, dA,
             lw + iA * UNIT, offA, rA, kA, LATE ? need : -1, LATE ? -1 : need, !(LATE && last));
        kB += 128;
        kA += 128;
#pragma unroll
        for (int q = 0; q < 4; ++q) cur[q] = nxt[q];
    };

    int v = blockIdx.x;
    if (v >= ntiles) return;  // whole workgroup
    int m0, n0;
    coords(v, m0, n0);
    bool primed = false;  // this tile's A0 B0 A1 issued (and landed) under the previous tile's epilogue
    while (true) {
        // one prologue path for every tile (as pipe10): units A0 B0 A1 unless primed, then the scales of
        // stages 0 and 1 and units B1 A2; one counted wait covers both paths (A0..A1, scales landed)
        set_off(m0, n0);
        kscA = kscB = 0;
        if (SEAM == 2 || !primed) {
            mx_dma4<true>(lw + 0 * UNIT, offA, rA, 0);
            mx_dma4<true>(lw + 1 * UNIT, offB, rB, 0);
            mx_dma4<true>(lw + 2 * UNIT, offA, rA, 128);
        }
        load_sc(cur);
        load_sc(nxt);
        mx_dma4<true>(lw + 3 * UNIT, offB, rB, 128);
        mx_dma4<true>(lw + 4 * UNIT, offA, rA, 256);
        vm_wait_sc<8>(cur);
        vm_wait_sc<8>(nxt);
        __builtin_amdgcn_s_barrier();
        if (LATE) __builtin_amdgcn_s_barrier();
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
        {  // stage 0: its successors' units were issued before it; cur <- stage 1's scales
            const unsigned c0 = cur[0], c1 = cur[1], c2 = cur[2], c3 = cur[3];
            const unsigned bs = b_x + UNIT;
            step(a_x, a_x ^ (2u << 4), bs, bs ^ (2u << 4), c0, c2, false, false, 0, offB, rB, 0, -1, -1, true);
            step(a_x ^ (4u << 4), a_x ^ (6u << 4), bs ^ (4u << 4), bs ^ (6u << 4), c1, c3, false, false, 0, offA, rA,
                 0, LATE ? 4 : -1, LATE ? -1 : 4, true);
#pragma unroll
            for (int q = 0; q < 4; ++q) cur[q] = nxt[q];
        }
        kB = 256;
        kA = 384;
        int s = 1;
        for (; s + 5 <= nk - 2; s += 5) {
            stage(2, true, true, true, 4, false);
            stage(4, true, true, true, 4, false);
            stage(1, true, true, true, 4, false);
            stage(3, true, true, true, 4, false);
            stage(0, true, true, true, 4, false);
        }
        if (s < nk - 2) {
            stage(2, true, true, true, 4, false);
            if (++s < nk - 2) {
                stage(4, true, true, true, 4, false);
                if (++s < nk - 2) {
                    stage(1, true, true, true, 4, false);
                    if (++s < nk - 2) {
                        stage(3, true, true, true, 4, false);
                        ++s;
                    }
                }
            }
        }
        const int sa2 = (2 * s) % 5, sa1 = sa2 >= 3 ? sa2 - 3 : sa2 + 2;
        stage(sa2, true, true, false, 0, false);
        stage(sa1, false, false, false, -1, true);
        vm_wait<0>();
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) asm volatile("" : "+v"(acc[i][j]));
        // every wave's fragment reads of this tile precede the barrier closing the late row's last
        // memory phase, which this wave has passed: the whole ring is free of reads
        const int vn = v + gridDim.x;
        const bool has_next = vn < ntiles;
        int m1 = 0, n1 = 0;
        if (has_next) coords(vn, m1, n1);
        const bool prime = SEAM != 2 && has_next;
        if (prime) {  // the next tile's A0 B0 A1 under this tile's epilogue
            set_off(m1, n1);
            mx_dma4<true>(lw + 0 * UNIT, offA, rA, 0);
            mx_dma4<true>(lw + 1 * UNIT, offB, rB, 0);
            mx_dma4<true>(lw + 2 * UNIT, offA, rA, 128);
        }
        {  // lane id from a volatile asm (pipe10: lane-derived epilogue addresses not hoisted and spilled)
            int ln;
            asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(ln));
            mx_epilogue_wave<ACT, true, true, 2>(p, lds + 3 * UNIT, acc, m0, n0, wave, ln);
        }
        vm_wait<0>();  // own pieces of the next A0 B0 A1 landed (and this wave's stores retired)
        __builtin_amdgcn_s_barrier();  // staging reads of every wave done: slots 3-4 free
        if (!has_next) break;
        v = vn;
        m0 = m1;
        n0 = n1;
        primed = prime;
    }
}

template <int GROUP_M, int ACT, int SEAM = 0>
__global__ __launch_bounds__(512, 2) void gemm_mx12_kernel(MxArgs p) {
    __shared__ __attribute__((aligned(16))) char lds[5 * 32768];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (wave >= 4)
        mx12_run<GROUP_M, ACT, true, SEAM>(p, lds, wave);
    else
        mx12_run<GROUP_M, ACT, false, SEAM>(p, lds, wave);
}

// one persistent workgroup per CU, a multiple of the 8 XCDs (the device's own CU count, read once)
int mx_persistent_grid(int ntiles) {
    static int cus[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
    if (cus[dev] == 0) {
        int n = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
        cus[dev] = n >= 8 ? n / 8 * 8 : n;
    }
    return ntiles < cus[dev] ? ntiles : cus[dev];
}

template <int GROUP_M, int SEAM = 0>
int launch_mx12(const MxArgs& a, hipStream_t s) {
    const dim3 grid(mx_persistent_grid(((a.M + 255) / 256) * ((a.N + 255) / 256))), block(512);
    switch (a.act) {
        case MME_ACT_GELU_TANH:
            hipLaunchKernelGGL((gemm_mx12_kernel<GROUP_M, MME_ACT_GELU_TANH, SEAM>), grid, block, 0, s, a);
            break;
        case MME_ACT_QUICK_GELU:
            hipLaunchKernelGGL((gemm_mx12_kernel<GROUP_M, MME_ACT_QUICK_GELU, SEAM>), grid, block, 0, s, a);
            break;
        case MME_ACT_GELU_ERF:
            hipLaunchKernelGGL((gemm_mx12_kernel<GROUP_M, MME_ACT_GELU_ERF, SEAM>), grid, block, 0, s, a);
            break;
        default:
            hipLaunchKernelGGL((gemm_mx12_kernel<GROUP_M, MME_ACT_NONE, SEAM>), grid, block, 0, s, a);
            break;
    }
    return mme_check_launch("mme_gemm_mx");
}

#ifdef MME_DEV
// ---------------------------------------------------------------------------
// mx9 (dev variant 9, round 3; MME_DEV builds only): the block-scaled fp8 GEMM on
// whole-line LDS-DMA rows. gemm_mx_kernel stages 64-deep fp8 stages as 64-B half-line
// rows (16 rows x 64 B per 1 KiB piece), the piece shape the LDS-DMA path moves at about
// half the rate of whole 128-B lines (tools/probes/dma_bw.hip); at the fp8 MFMA rate that
// path was the bound (1.65 PF/s). Here a stage is 128 fp8 deep, so every A / B row of a
// stage is one 128-B line (pieces of 8 rows x 128 B, XOR-swizzled as pipe8:
// chunk ^ ((row >> 1) & 7)), and runs as two 64-deep steps of pipe6 / pipe9's ping-pong
// (memory phase | barrier | compute phase | barrier, the second wave row one phase behind).
// LDS: two stage slots of A and B (4 x 32 KiB) + two 2 KiB scale slots ([A kb0..3][B kb0..3],
// 256 rows each). During stage s every wave issues stage s + 1 (its 8 data pieces; waves 0 / 1
// also the A / B scale piece) in its first memory phase, into the slot stage s - 1 released;
// the early row retires them after its last compute phase of stage s, the late row before
// the barrier closing its last memory phase (2.5 - 3.5 phases after issue). Static slots
// (stage loop unrolled by 2), DMA by buffer_load ... lds with the K offset in soffset.
// Per-wave epilogue (no workgroup barrier), bf16 + residual or mx8 re-quantisation.
// ---------------------------------------------------------------------------
constexpr int MX9_UNIT = 32768, MX9_SC = 4 * MX9_UNIT, MX9_PITCH = 144;
constexpr int MX9_LDS = 8 * 128 * MX9_PITCH;  // per-wave epilogue tiles; the main loop uses less
static_assert(MX9_SC + 4096 + 5 * 1024 + 2048 + 1024 <= MX9_LDS, "mx9: scale slots + scratch pieces fit");

template <int ACT, bool LATE>
__device__ __forceinline__ void mx9_tile(const MxArgs& p, char* lds, const int m0, const int n0, const int wave) {
    constexpr int TM = 128, TN = 64;
    const int lane = threadIdx.x & 63;
    const int wm = wave / 4, wn = wave % 4;
    const int h = lane >> 5, r32 = lane & 31;

    unsigned offA[4], offB[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int prow = (wave * 4 + q) * 8 + (lane >> 3);
        const int logical = (lane & 7) ^ ((prow >> 1) & 7);
        offA[q] = (unsigned)min(m0 + prow, p.M - 1) * (unsigned)p.lda + logical * 16;
        offB[q] = (unsigned)min(n0 + prow, p.N - 1) * (unsigned)p.ldb + logical * 16;
    }
    const int K = p.K, nk = K / 128;
    const i32x4v rA = mx_rsrc(p.A, (unsigned)((size_t)p.M * p.lda));
    const i32x4v rB = mx_rsrc(p.B, (unsigned)((size_t)p.N * p.ldb));
    // scale piece (waves 0 / 1: A / B): lane l -> block kb = l / 16 of the stage, 16 rows (l % 16) * 16..
    // waves 2..7: a zero-length range (no memory traffic) into LDS past the scale slots
    const bool sc_wave = wave < 2;
    const int sc_rows = wave == 0 ? p.sa_rows : p.sb_rows;
    const i32x4v rS = mx_rsrc(wave == 0 ? (const void*)p.sa : (const void*)p.sb,
                              sc_wave ? (unsigned)((size_t)(K / 32) * sc_rows) : 0u);
    const unsigned voS = (unsigned)((lane >> 4) * sc_rows + (wave == 0 ? m0 : n0) + (lane & 15) * 16);
    const unsigned lds0 = (unsigned)(uintptr_t)(LDS_AS char*)lds;
    const unsigned lw = __builtin_amdgcn_readfirstlane(lds0 + wave * 4096);
    const unsigned lsc = __builtin_amdgcn_readfirstlane(lds0 + MX9_SC + (sc_wave ? wave * 1024 : 4096 + (wave - 2) * 1024));

    const int sw = (r32 >> 1) & 7;
    const unsigned a_row = lds0 + (wm * TM + r32) * 128, b_row = lds0 + MX9_UNIT + (wn * TN + r32) * 128;
    // fragment addresses of step ks = 0 / 1 (logical chunks 4 ks + h, 4 ks + 2 + h); the
    // fragment rows (i, j) * 32 ride in the ds_read offset field, the stage slot is added per stage
    const unsigned a00 = a_row + (((0 + h) ^ sw) << 4), a01 = a_row + (((2 + h) ^ sw) << 4);
    const unsigned a10 = a_row + (((4 + h) ^ sw) << 4), a11 = a_row + (((6 + h) ^ sw) << 4);
    const unsigned b00 = b_row + (((0 + h) ^ sw) << 4), b01 = b_row + (((2 + h) ^ sw) << 4);
    const unsigned b10 = b_row + (((4 + h) ^ sw) << 4), b11 = b_row + (((6 + h) ^ sw) << 4);
    const unsigned sa_l = lds0 + MX9_SC + h * 256 + wm * TM + r32 * 4;  // mx_srow order
    const unsigned sb_l = lds0 + MX9_SC + 1024 + h * 256 + (wn >> 1) * 128 + r32 * 4 + (wn & 1) * 2;

    f32x16 acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
    bf16x8 a[4][2], b[2][2];
    unsigned sa[4], sbv[2];

    // one 64-deep step: fragments at aa0 / aa1 / bb0 / bb1 (chunks c0, c1 of the slot's rows),
    // scale bytes at sca / scb (blocks 2 ks + h), optionally the DMA of the next stage into slot
    // `nslot`, waits, barrier, 8 MFMAs, barrier. wm_ / wc_ = 0: drain vmcnt after the memory /
    // compute phase (-1: no wait)
    auto step = [&](unsigned aa0, unsigned aa1, unsigned bb0, unsigned bb1, unsigned sca, unsigned scb, bool dma,
                    unsigned nslot, unsigned soff, unsigned soffS, bool wm_, bool wc_, bool end_barrier)
        __attribute__((always_inline)) {
        ds_read16<0>(b[0][0], bb0);
        ds_read16<0>(b[0][1], bb1);
        ds_read16<4096>(b[1][0], bb0);
        ds_read16<4096>(b[1][1], bb1);
        ds_read16<0>(a[0][0], aa0);
        ds_read16<0>(a[0][1], aa1);
        ds_read16<4096>(a[1][0], aa0);
        ds_read16<4096>(a[1][1], aa1);
        ds_read16<8192>(a[2][0], aa0);
        ds_read16<8192>(a[2][1], aa1);
        ds_read16<12288>(a[3][0], aa0);
        ds_read16<12288>(a[3][1], aa1);
        asm volatile("ds_read_u8 %0, %1 offset:0" : "=v"(sbv[0]) : "v"(scb) : "memory");
        asm volatile("ds_read_u8 %0, %1 offset:1" : "=v"(sbv[1]) : "v"(scb) : "memory");
        asm volatile("ds_read_u8 %0, %1 offset:0" : "=v"(sa[0]) : "v"(sca) : "memory");
        asm volatile("ds_read_u8 %0, %1 offset:1" : "=v"(sa[1]) : "v"(sca) : "memory");
        asm volatile("ds_read_u8 %0, %1 offset:2" : "=v"(sa[2]) : "v"(sca) : "memory");
        asm volatile("ds_read_u8 %0, %1 offset:3" : "=v"(sa[3]) : "v"(sca) : "memory");
        if (dma) {
            mx_dma4(lw + nslot * 2 * MX9_UNIT, offA, rA, soff);
            mx_dma4(lw + nslot * 2 * MX9_UNIT + MX9_UNIT, offB, rB, soff);
            mx_dma1(lsc + nslot * 2048, voS, rS, soffS);
        }
        if (wm_) vm_wait<0>();
        lgkm_wait<0>();
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const i32x8 bo = __builtin_bit_cast(
                    i32x8, __builtin_shufflevector(b[j][0], b[j][1], 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15));
                const i32x8 ao = __builtin_bit_cast(
                    i32x8, __builtin_shufflevector(a[i][0], a[i][1], 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15));
                acc[i][j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(bo, ao, acc[i][j], 0, 0, 0, (int)sbv[j], 0,
                                                                             (int)sa[i]);
            }
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
        if (wc_) vm_wait<0>();
        if (end_barrier) __builtin_amdgcn_s_barrier();
    };
    // prologue: stage 0 into slot 0 (waves 2..7 DMA their scale piece from an empty range into
    // an LDS scratch area, so every wave's DMA count is the same)
    mx_dma4(lw, offA, rA, 0);
    mx_dma4(lw + MX9_UNIT, offB, rB, 0);
    mx_dma1(lsc, voS, rS, 0);
    vm_wait<0>();
    __builtin_amdgcn_s_barrier();
    if (LATE) __builtin_amdgcn_s_barrier();
    // stage s in slot s & 1; it issues stage s + 1 into the other slot (data soffset 128 (s + 1),
    // scale soffset 4 sc_rows (s + 1)). The early row drains its DMA after its last compute
    // phase of the stage, the late row before the barrier closing its last memory phase.
    unsigned kN = 128, kS = 4u * (unsigned)sc_rows;
    for (int s = 0; s < nk; ++s) {
        const unsigned slot = s & 1, so = slot * 2 * MX9_UNIT, ss = slot * 2048;
        const bool issue = s + 1 < nk, last = !issue;
        step(a00 + so, a01 + so, b00 + so, b01 + so, sa_l + ss, sb_l + ss, issue, 1 - slot, kN, kS, false, false,
             true);
        step(a10 + so, a11 + so, b10 + so, b11 + so, sa_l + ss + 512, sb_l + ss + 512, false, 0, 0, 0,
             LATE && issue, !LATE && issue, !(LATE && last));
        kN += 128;
        kS += 4u * (unsigned)sc_rows;
    }

    mx_epilogue_wave<ACT>(p, lds, acc, m0, n0, wave, lane);
}

template <int GROUP_M, int ACT>
__global__ __launch_bounds__(512, 2) void gemm_mx9_kernel(MxArgs p) {
    __shared__ __attribute__((aligned(16))) char lds[MX9_LDS];
    const int nbm = (p.M + 255) / 256, nbn = p.N / 256;
    const int tile = xcd_remap(blockIdx.x, gridDim.x);
    int bm, bn;
    tile_coords<GROUP_M>(tile, nbm, nbn, bm, bn);
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (wave >= 4)
        mx9_tile<ACT, true>(p, lds, bm * 256, bn * 256, wave);
    else
        mx9_tile<ACT, false>(p, lds, bm * 256, bn * 256, wave);
}

template <int GROUP_M>
int launch_mx9(const MxArgs& a, hipStream_t s) {
    const dim3 grid(((a.M + 255) / 256) * (a.N / 256)), block(512);
    switch (a.act) {
        case MME_ACT_GELU_TANH:
            hipLaunchKernelGGL((gemm_mx9_kernel<GROUP_M, MME_ACT_GELU_TANH>), grid, block, 0, s, a);
            break;
        case MME_ACT_QUICK_GELU:
            hipLaunchKernelGGL((gemm_mx9_kernel<GROUP_M, MME_ACT_QUICK_GELU>), grid, block, 0, s, a);
            break;
        case MME_ACT_GELU_ERF:
            hipLaunchKernelGGL((gemm_mx9_kernel<GROUP_M, MME_ACT_GELU_ERF>), grid, block, 0, s, a);
            break;
        default:
            hipLaunchKernelGGL((gemm_mx9_kernel<GROUP_M, MME_ACT_NONE>), grid, block, 0, s, a);
            break;
    }
    return mme_check_launch("mme_gemm_mx");
}

#endif  // MME_DEV

// Kernel form per call (mme_gemm_mx_form): -1 = production (mx11 where its geometry holds, else mx10),
// 10 = mx10, 0 = the round-2 kernel, 2 = its per-wave epilogue alone, 3 = + the scale wave (mx10's
// fallback), 9 = mx9 (development build). The development build keeps a process-wide default (mme_gemm_mx_variant).
#ifdef MME_DEV
int g_mx_variant = -1;
inline int mx_default_form() { return g_mx_variant; }
#else
inline int mx_default_form() { return -1; }
#endif
inline bool mx_form_ok(int v) {
#ifdef MME_DEV
    return v == -1 || v == 0 || v == 2 || v == 3 || v == 4 || v == 9 || v == 10 || v == 11 || v == 12 || v == 14 || v == 15 || v == 16 || v == 17;
#else
    return v == -1 || v == 0 || v == 2 || v == 3 || v == 10 || v == 11 || v == 15 || v == 16 || v == 17;  // mx12: dev only
#endif
}

template <int GROUP_M, bool WEPI = false, bool SC1 = false>
int launch_mx(const MxArgs& a, hipStream_t s) {
    const int nbm = (a.M + 255) / 256, nbn = (a.N + 255) / 256;
    const dim3 grid(nbm * nbn), block(512);
    switch (a.act) {
        case MME_ACT_GELU_TANH:
            hipLaunchKernelGGL((gemm_mx_kernel<GROUP_M, MME_ACT_GELU_TANH, WEPI, SC1>), grid, block, 0, s, a);
            break;
        case MME_ACT_QUICK_GELU:
            hipLaunchKernelGGL((gemm_mx_kernel<GROUP_M, MME_ACT_QUICK_GELU, WEPI, SC1>), grid, block, 0, s, a);
            break;
        case MME_ACT_GELU_ERF:
            hipLaunchKernelGGL((gemm_mx_kernel<GROUP_M, MME_ACT_GELU_ERF, WEPI, SC1>), grid, block, 0, s, a);
            break;
        default:
            hipLaunchKernelGGL((gemm_mx_kernel<GROUP_M, MME_ACT_NONE, WEPI, SC1>), grid, block, 0, s, a);
            break;
    }
    return mme_check_launch("mme_gemm_mx");
}

}  // namespace

extern "C" int mme_mx_quant(const void* x, int ldx, int rows, int k, void* q, int ldq, void* scales, int rows_pad,
                            void* stream) {
    MME_REQUIRE(x && q && scales, "mme_mx_quant: null pointer");
    MME_REQUIRE(rows >= 0 && k > 0 && k % 32 == 0, "mme_mx_quant: k=%d must be a positive multiple of 32", k);
    MME_REQUIRE(ldx % 8 == 0 && ldx >= k && ldq % 16 == 0 && ldq >= k, "mme_mx_quant: bad leading dims");
    MME_REQUIRE(rows_pad >= rows && rows_pad % 256 == 0, "mme_mx_quant: rows_pad must be >= rows, multiple of 256");
    MME_REQUIRE(((uintptr_t)x & 15) == 0 && ((uintptr_t)q & 15) == 0, "mme_mx_quant: misaligned");
    if (rows == 0) return MME_OK;
    hipLaunchKernelGGL(mx_quant_kernel, dim3(rows), dim3(256), 0, as_stream(stream), (const bf16*)x, ldx, k,
                       (uint8_t*)q, ldq, (uint8_t*)scales, rows_pad);
    return mme_check_launch("mme_mx_quant");
}

extern "C" int mme_layernorm_mx(const void* x, int ldx, const void* gamma, const void* beta, int rows, int d,
                                float eps, const int32_t* rows_idx, void* q, int ldq, void* scales, int rows_pad,
                                void* stream) {
    MME_REQUIRE(x && gamma && beta && q && scales, "mme_layernorm_mx: null pointer");
    MME_REQUIRE(rows >= 0 && d > 0 && d % 32 == 0 && d <= 8 * 32 * LNH_MAXC, "mme_layernorm_mx: d=%d unsupported", d);
    MME_REQUIRE(ldx % 8 == 0 && ldx >= d && ldq % 16 == 0 && ldq >= d, "mme_layernorm_mx: bad leading dims");
    MME_REQUIRE(rows_pad >= rows && rows_pad % 256 == 0, "mme_layernorm_mx: rows_pad must be >= rows, multiple of 256");
    if (rows == 0) return MME_OK;
    const int mc = (d / 8 + 31) / 32;  // chunks per lane of a half-wave row
#define MME_LN_MX(MC)                                                                                                  \
    hipLaunchKernelGGL(layernorm_mx_kernel<MC>, dim3(cdiv(rows, 8)), dim3(256), 0, as_stream(stream), (const bf16*)x,   \
                       ldx, (const bf16*)gamma, (const bf16*)beta, rows, d, eps, rows_idx, (uint8_t*)q, ldq,            \
                       (uint8_t*)scales, rows_pad)
    if (mc <= 3) MME_LN_MX(3);
    else if (mc <= 4) MME_LN_MX(4);
    else if (mc <= 5) MME_LN_MX(5);
    else MME_LN_MX(LNH_MAXC);
#undef MME_LN_MX
    return mme_check_launch("mme_layernorm_mx");
}

#ifdef MME_DEV
extern "C" int mme_gemm_mx_variant(int v) {  // development build only: the form of mme_gemm_mx
    MME_REQUIRE(mx_form_ok(v), "mme_gemm_mx_variant: unknown variant %d", v);
    g_mx_variant = v;
    return MME_OK;
}
#endif

namespace {
int gemm_mx_entry(int form, const void* A, int lda, const void* sa, int sa_rows, const void* B, int ldb, const void* sb,
                  int sb_rows, void* Cp, int ldc, void* c_scales, int c_rows_pad, int M, int N, int K, const void* bias,
                  const void* residual, int ldr, int res_period, int act, int out_mx, void* stream);
}  // namespace

extern "C" int mme_gemm_mx_form(int form, const void* A, int lda, const void* sa, int sa_rows, const void* B, int ldb,
                                const void* sb, int sb_rows, void* Cp, int ldc, void* c_scales, int c_rows_pad, int M,
                                int N, int K, const void* bias, const void* residual, int ldr, int res_period, int act,
                                int out_mx, void* stream) {
    MME_REQUIRE(mx_form_ok(form), "mme_gemm_mx_form: form %d is unknown or a development form (make dev)", form);
    return gemm_mx_entry(form, A, lda, sa, sa_rows, B, ldb, sb, sb_rows, Cp, ldc, c_scales, c_rows_pad, M, N, K, bias,
                         residual, ldr, res_period, act, out_mx, stream);
}

extern "C" int mme_gemm_mx(const void* A, int lda, const void* sa, int sa_rows, const void* B, int ldb,
                           const void* sb, int sb_rows, void* Cp, int ldc, void* c_scales, int c_rows_pad, int M,
                           int N, int K, const void* bias, const void* residual, int ldr, int res_period, int act,
                           int out_mx, void* stream) {
    return gemm_mx_entry(mx_default_form(), A, lda, sa, sa_rows, B, ldb, sb, sb_rows, Cp, ldc, c_scales, c_rows_pad, M,
                         N, K, bias, residual, ldr, res_period, act, out_mx, stream);
}

namespace {
int gemm_mx_entry(int form, const void* A, int lda, const void* sa, int sa_rows, const void* B, int ldb, const void* sb,
                  int sb_rows, void* Cp, int ldc, void* c_scales, int c_rows_pad, int M, int N, int K, const void* bias,
                  const void* residual, int ldr, int res_period, int act, int out_mx, void* stream) {
    MME_REQUIRE(A && B && sa && sb && Cp, "mme_gemm_mx: null operand");
    MME_REQUIRE(M >= 0 && N > 0 && K > 0 && K % 64 == 0, "mme_gemm_mx: K=%d must be a positive multiple of 64", K);
    MME_REQUIRE(lda % 16 == 0 && ldb % 16 == 0 && lda >= K && ldb >= K, "mme_gemm_mx: lda/ldb must be >= K, % 16");
    MME_REQUIRE(((uintptr_t)A & 15) == 0 && ((uintptr_t)B & 15) == 0 && ((uintptr_t)sa & 15) == 0 &&
                    ((uintptr_t)sb & 15) == 0 && ((uintptr_t)Cp & 15) == 0,
                "mme_gemm_mx: operands must be 16-byte aligned");
    MME_REQUIRE(sa_rows % 256 == 0 && sa_rows >= M && sb_rows % 256 == 0 && sb_rows >= N,
                "mme_gemm_mx: scale planes must cover round_up(rows, 256)");
    MME_REQUIRE(act >= MME_ACT_NONE && act <= MME_ACT_GELU_ERF, "mme_gemm_mx: bad activation %d", act);
    if (out_mx) {
        MME_REQUIRE(c_scales && N % 32 == 0 && ldc % 16 == 0 && ldc >= N && c_rows_pad % 256 == 0 && c_rows_pad >= M,
                    "mme_gemm_mx: mx8 output needs N %% 32 == 0, ldc %% 16 == 0 and a covering scale plane");
        MME_REQUIRE(!residual, "mme_gemm_mx: residual add is not supported with mx8 output");
    } else {
        MME_REQUIRE(N % 8 == 0 && ldc % 8 == 0 && ldc >= N, "mme_gemm_mx: bf16 output needs N, ldc %% 8 == 0");
        MME_REQUIRE(!residual || (ldr % 8 == 0 && ((uintptr_t)residual & 15) == 0), "mme_gemm_mx: bad residual");
    }
    if (M == 0) return MME_OK;
    MxArgs a{(const uint8_t*)A, (const uint8_t*)B, (const uint8_t*)sa, (const uint8_t*)sb, Cp, (uint8_t*)c_scales,
             (const bf16*)bias, (const bf16*)residual, lda, ldb, ldc, ldr, sa_rows, sb_rows, c_rows_pad, M, N, K,
             res_period, act, out_mx};
#ifdef MME_DEV
    // dev variant 9: mx9 where its geometry holds (every DFN5B-H encoder shape); 32-bit DMA offsets
    if (form == 9 && K % 128 == 0 && K >= 256 && N % 256 == 0 && (size_t)M * lda < (1ull << 32) &&
        (size_t)N * ldb < (1ull << 32) && (size_t)(K / 32) * (sa_rows > sb_rows ? sa_rows : sb_rows) < (1ull << 32))
        return launch_mx9<4>(a, as_stream(stream));
#endif
    // production since round 3: mx10 (static slots / waits, buffer-load DMA, per-wave epilogue, one
    // scale-DMA wave) where its geometry holds: DFN5B-H fp8 job 1 016 -> 1 028 (per-wave epilogue +
    // scale wave, profiles/r03_v14_*) -> 1 041 img/s (mx10, profiles/r03_v15_*); elsewhere the
    // gemm_mx_kernel form with the same epilogue and scale wave. A/B forms: variant 0 = the round-2
    // kernel, 2 = its per-wave epilogue alone, 3 = + the scale wave (mx10's fallback).
    const bool mx10_ok = K >= 256 && (size_t)M * lda < (1ull << 32) && (size_t)N * ldb < (1ull << 32);
#ifdef MME_DEV
    if (form == 4 && mx10_ok) return launch_mx10<4, false>(a, as_stream(stream));  // dev: round-3 epilogue staging
#endif
    if (form == 0) return launch_mx<4>(a, as_stream(stream));
    if (form == 2) return launch_mx<4, true>(a, as_stream(stream));
    if (form == 3 || !mx10_ok) return launch_mx<4, true, true>(a, as_stream(stream));
    // round 4: mx11 (pipe9's whole-line ring, scales by buffer loads) where its geometry holds;
    // form 10 = mx10 (the bit-identity reference and A/B baseline)
    const bool mx11_ok = K % 128 == 0 && K >= 384 &&
                         (size_t)(K / 32) * (sa_rows > sb_rows ? sa_rows : sb_rows) < (1ull << 32);
    if (form == 12 && mx11_ok) return launch_mx12<4>(a, as_stream(stream));
    if (form == 14 && mx11_ok) return launch_mx12<4, 2>(a, as_stream(stream));
    // round 5, production where N % 4 == 0 and the bias is 8-B aligned: the bias loaded up front (form 15:
    // DFN5B-H fp8 job 1 185-1 187 -> 1 203 img/s, profiles/r05_v20_mx15_ab.log), the mx8 output's block absmax
    // by DPP and quick_gelu in packed f32 (form 16: 1 179-1 181 -> 1 193-1 196 img/s, profiles/r05_v22_mx16_ab.log);
    // bit-identical throughout; form 11 = mx11 without either, form 15 = the bias alone
    if (form == 15 && mx11_ok && N % 4 == 0 && ((uintptr_t)bias & 7) == 0)
        return launch_mx11<4, true>(a, as_stream(stream));
    // round 6, form 17 = form 16 with the mx8 output packed without the (inactive) clamp, scaled by packed multiplies
    if (form == 16 && mx11_ok && N % 4 == 0 && ((uintptr_t)bias & 7) == 0)
        return launch_mx11<4, true, true>(a, as_stream(stream));
    if (form != 10 && form != 11 && mx11_ok && N % 4 == 0 && ((uintptr_t)bias & 7) == 0)
        return launch_mx11<4, true, true, true>(a, as_stream(stream));
    if (form != 10 && mx11_ok) return launch_mx11<4>(a, as_stream(stream));
    return launch_mx10<4>(a, as_stream(stream));
}
}  // namespace
