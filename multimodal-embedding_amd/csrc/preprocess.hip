// Image preprocessing on the device: PIL-exact BICUBIC resize of u8 RGB
// images, center crop, rescale(1/255) and normalise — what
// processor(images=batch) does on the host in the reference (main.py:407 ->
// HF PilBackend._preprocess -> PIL Image.resize(BICUBIC)).
//
// PIL's algorithm (libImaging/Resample.c, restated; no PIL source is used):
//   * per output coordinate xx: scale = in/out, filterscale = max(scale, 1),
//     support = 2 * filterscale, center = (xx + 0.5) * scale,
//     xmin = max((int)(center - support + 0.5), 0),
//     xmax = min((int)(center + support + 0.5), in) - xmin,
//     w_x = bicubic((x + xmin - center + 0.5) / filterscale), normalised by
//     their sum, then converted to 22-bit fixed point
//     (int)(w * 2^22 +- 0.5) — all in IEEE double, no FMA contraction;
//   * horizontal pass first, then vertical; each pass accumulates
//     int32 sum = 2^21 + sum(u8 * coeff) and clips (sum >> 22) to [0, 255];
//   * HF then computes float32(float64(u8) * (1/255)) and (x - mean) / std in
//     float32 (transformers image_transforms.rescale / normalize).
// Every step is integer or correctly-rounded IEEE, so the device result is
// bit-identical to PIL + HF (pinned by tests/golden/preprocess.npz).
#include "common.h"

namespace {

constexpr int PREC = 22;

#pragma clang fp contract(off)
__device__ double bicubic(double x) {
    const double a = -0.5;
    if (x < 0.0) x = -x;
    if (x < 1.0) return ((a + 2.0) * x - (a + 3.0)) * x * x + 1;
    if (x < 2.0) return (((x - 5) * x + 8) * x - 4) * a;
    return 0.0;
}

__host__ __device__ inline int ksize_for(int in, int out) {
    double scale = (double)in / out;
    double fs = scale < 1.0 ? 1.0 : scale;
    double support = 2.0 * fs;
    return (int)ceil(support) * 2 + 1;
}

// One thread per output coordinate: bounds[2*xx] = xmin, bounds[2*xx+1] = count,
// kk[xx*ksize + i] = fixed-point coefficient.
__global__ void coeffs_kernel(int in, int out, int ksize, int* __restrict__ bounds, int* __restrict__ kk) {
#pragma clang fp contract(off)
    const int xx = blockIdx.x * blockDim.x + threadIdx.x;
    if (xx >= out) return;
    const double scale = (double)in / out;
    const double fs = scale < 1.0 ? 1.0 : scale;
    const double support = 2.0 * fs;
    const double center = (xx + 0.5) * scale;
    const double ss = 1.0 / fs;
    int xmin = (int)(center - support + 0.5);
    if (xmin < 0) xmin = 0;
    int xmax = (int)(center + support + 0.5);
    if (xmax > in) xmax = in;
    xmax -= xmin;
    double w[64];
    double ww = 0.0;
    for (int x = 0; x < xmax; ++x) {
        const double v = bicubic((x + xmin - center + 0.5) * ss);
        w[x] = v;
        ww += v;
    }
    for (int x = 0; x < ksize; ++x) {
        double k = 0.0;
        if (x < xmax) k = (ww != 0.0) ? w[x] / ww : w[x];
        kk[xx * ksize + x] = k < 0 ? (int)(-0.5 + k * (1 << PREC)) : (int)(0.5 + k * (1 << PREC));
    }
    bounds[2 * xx] = xmin;
    bounds[2 * xx + 1] = xmax;
}

__device__ __forceinline__ int clip8(int v) {
    v >>= PREC;
    return v < 0 ? 0 : (v > 255 ? 255 : v);
}

// Horizontal pass for the cropped columns only: tmp[n][y][xc][3], xc < S.
__global__ void resample_h_kernel(const uint8_t* __restrict__ img, int n, int H, int W, int S, int left, int ksize,
                                  const int* __restrict__ bounds, const int* __restrict__ kk,
                                  uint8_t* __restrict__ tmp) {
    const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const long total = (long)n * H * S;
    if (t >= total) return;
    const int xc = t % S;
    const long ny = t / S;  // n*H + y
    const int xx = xc + left;
    const int xmin = bounds[2 * xx], cnt = bounds[2 * xx + 1];
    const int* k = kk + xx * ksize;
    const uint8_t* src = img + ny * W * 3;
    int s0 = 1 << (PREC - 1), s1 = s0, s2 = s0;
    for (int x = 0; x < cnt; ++x) {
        const uint8_t* p = src + (xmin + x) * 3;
        s0 += p[0] * k[x];
        s1 += p[1] * k[x];
        s2 += p[2] * k[x];
    }
    uint8_t* d = tmp + t * 3;
    d[0] = (uint8_t)clip8(s0);
    d[1] = (uint8_t)clip8(s1);
    d[2] = (uint8_t)clip8(s2);
}

__device__ __forceinline__ float normalize(int u8, float mean, float stdv) {
    const float r = (float)((double)u8 * (1.0 / 255.0));
    return (r - mean) / stdv;
}

// Vertical pass + rescale/normalise; thread = one output element of the
// requested layout (coalesced writes).
struct NormArgs {
    float mean[3], stdv[3];
};

__device__ __forceinline__ int vpass(const uint8_t* tmp_img, int S, int yy, int xc, int c, int ksize,
                                     const int* bounds, const int* kk) {
    const int ymin = bounds[2 * yy], cnt = bounds[2 * yy + 1];
    const int* k = kk + yy * ksize;
    int s = 1 << (PREC - 1);
    for (int y = 0; y < cnt; ++y) s += tmp_img[((long)(ymin + y) * S + xc) * 3 + c] * k[y];
    return clip8(s);
}

__global__ void resample_v_nchw_kernel(const uint8_t* __restrict__ tmp, int n, int H, int S, int top, int ksize,
                                       const int* __restrict__ bounds, const int* __restrict__ kk, NormArgs na,
                                       float* __restrict__ out) {
    const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const long total = (long)n * 3 * S * S;
    if (t >= total) return;
    const int xc = t % S;
    const int yc = (t / S) % S;
    const int c = (t / ((long)S * S)) % 3;
    const long b = t / (3L * S * S);
    const int u = vpass(tmp + b * H * S * 3, S, yc + top, xc, c, ksize, bounds, kk);
    out[t] = normalize(u, na.mean[c], na.stdv[c]);
}

// patches[row = b*G*G + py*G + px][col = c*p*p + ky*p + kx] (G = S/p), bf16,
// zero for col >= 3*p*p: the im2col image of Conv2d(k=s=p) fed straight to
// the patch-embedding GEMM.
__global__ void resample_v_patch_kernel(const uint8_t* __restrict__ tmp, int n, int H, int S, int top, int ksize,
                                        const int* __restrict__ bounds, const int* __restrict__ kk, NormArgs na,
                                        int p, int kpad, bf16* __restrict__ out) {
    const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const int G = S / p;
    const long total = (long)n * G * G * kpad;
    if (t >= total) return;
    const int col = t % kpad;
    const long row = t / kpad;
    if (col >= 3 * p * p) {
        out[t] = f2bf(0.f);
        return;
    }
    const int c = col / (p * p), ky = (col / p) % p, kx = col % p;
    const int px = row % G, py = (row / G) % G;
    const long b = row / ((long)G * G);
    const int u = vpass(tmp + b * H * S * 3, S, py * p + ky + top, px * p + kx, c, ksize, bounds, kk);
    out[t] = f2bf(normalize(u, na.mean[c], na.stdv[c]));
}

// Fused patch path (production for MME_PIX_PATCHES): one workgroup per (image, patch row).
// The input rows that patch row's p output rows need (vertical support included) are
// staged in LDS once, the horizontal pass fills an LDS u8 raster of those rows x the S
// cropped columns, and the vertical pass + rescale / normalise (a 256-entry per-channel
// table of the exact float32 values) writes the patch row's G patches x kpad bf16 -- one
// contiguous range of the im2col image -- as 16-B stores. The two-kernel path above it
// stored the h-pass raster to HBM and re-read it byte by byte (7.9x its bytes fetched,
// ~1 TB/s); same integer arithmetic in the same order, so the output is bit-identical.
constexpr int FUSED_LDS = 64 * 1024;  // staged input rows + h-pass raster (bytes)
__global__ __launch_bounds__(256) void resample_patch_fused_kernel(
    const uint8_t* __restrict__ img, int n, int H, int W, int S, int top, int left, int kx, int ky,
    const int* __restrict__ xb, const int* __restrict__ xk, const int* __restrict__ yb, const int* __restrict__ yk,
    NormArgs na, int p, int kpad, bf16* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) uint8_t buf[FUSED_LDS];
    __shared__ unsigned short lut[3][256];
    const int G = S / p;
    const int b = blockIdx.x / G, py = blockIdx.x % G, tid = threadIdx.x;
    const int oy0 = py * p + top, oy1 = oy0 + p - 1;
    const int r0 = yb[2 * oy0], r1 = yb[2 * oy1] + yb[2 * oy1 + 1];  // input rows [r0, r1) (ymin is monotone)
    const int R = r1 - r0, rowb = W * 3;
    uint8_t* in_l = buf;                                             // [R][W][3]
    uint8_t* hr = buf + ((R * rowb + 15) & ~15);                     // [R][S][3]
    for (int i = tid; i < 3 * 256; i += 256) {
        const int c = i >> 8, u = i & 255;
        lut[c][u] = __builtin_bit_cast(unsigned short, f2bf(normalize(u, na.mean[c], na.stdv[c])));
    }
    const uint8_t* src = img + ((long)b * H + r0) * rowb;
    const int nbytes = R * rowb;
    if ((((uintptr_t)src | (unsigned)nbytes) & 15) == 0) {
        for (int i = tid; i < nbytes / 16; i += 256)
            reinterpret_cast<uint4*>(in_l)[i] = reinterpret_cast<const uint4*>(src)[i];
    } else {
        for (int i = tid; i < nbytes; i += 256) in_l[i] = src[i];
    }
    __syncthreads();
    for (int i = tid; i < R * S * 3; i += 256) {  // horizontal pass (resample_h_kernel's sums)
        const int c = i % 3, xc = (i / 3) % S, r = i / (3 * S);
        const int xx = xc + left;
        const int xmin = xb[2 * xx], cnt = xb[2 * xx + 1];
        const int* k = xk + xx * kx;
        const uint8_t* sp = in_l + r * rowb + xmin * 3 + c;
        int sum = 1 << (PREC - 1);
        for (int x = 0; x < cnt; ++x) sum += sp[3 * x] * k[x];
        hr[i] = (uint8_t)clip8(sum);
    }
    __syncthreads();
    const int P2 = p * p, C3 = 3 * P2;
    bf16* dst = out + ((long)b * G * G + (long)py * G) * kpad;
    const int n8 = G * kpad / 8;  // 16-B chunks of the patch row (kpad % 8 == 0)
    for (int i = tid; i < n8; i += 256) {
        const int px = (i * 8) / kpad, col0 = (i * 8) % kpad;
        u16x8 v;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const int col = col0 + e;
            unsigned short o = 0;  // bf16 +0 for the K padding
            if (col < C3) {
                const int c = col / P2, kyy = (col / p) % p, kxx = col % p;
                const int oy = oy0 + kyy, xc = px * p + kxx;
                const int ymin = yb[2 * oy] - r0, cnt = yb[2 * oy + 1];
                const int* kk = yk + oy * ky;
                const uint8_t* hp = hr + ((long)ymin * S + xc) * 3 + c;
                int sum = 1 << (PREC - 1);
                for (int y = 0; y < cnt; ++y) sum += hp[(long)y * S * 3] * kk[y];
                o = lut[c][clip8(sum)];
            }
            v[e] = o;
        }
        *reinterpret_cast<u16x8*>(dst + (long)i * 8) = v;
    }
}

// Fused patch path at a compile-time patch size (production for p = 14, every registry
// vision tower; round 3). resample_patch_fused_kernel above spends its time in index
// arithmetic, not bytes: every output element re-derives (channel, ky, kx) by runtime
// division, and every tap of both passes re-reads its bounds and weights (0.97 ms per 239
// SigLIP images = 0.27 TB/s). Here each loop runs over the axis along which nothing but the
// data changes:
//   * horizontal pass: thread = one (column, channel) of the patch row's used columns
//     (G * P of the S cropped ones -- the conv never reads the rest); its bounds and <= 8
//     weights are loaded once, then it walks the staged input rows;
//   * vertical pass: same thread mapping, walking the P output rows; a row's bounds and
//     weights are the same for every thread (scalar loads);
//   * im2col write: thread = one 16-B chunk of a patch's kpad columns; its 8 LDS source
//     offsets and LUT bases are computed once, then it walks every G / 3-rd patch.
// The u8 raster of the P output rows stays in LDS ([P][G * P * 3]) and the LUT turns it into
// the exact float32 -> bf16 values. Same integer sums, so the output is bit-identical.
// K (round 4): a compile-time tap count (5 for every registry tower: 224 px upscaled to 224-384);
// the taps then run unconditionally (the coefficients past a window's count are exactly 0, and the
// extra bytes they read lie inside the LDS allocation) as 24-bit multiplies (__mul24, v_mad_i32_i24:
// |u8 * w| < 2^30 with |w| <= 2^22, exact), where the K = 0 form branches per tap around 32-bit
// multiplies. Same integer sums, so the output is bit-identical.
template <int P, int K = 0>
__global__ __launch_bounds__(256) void resample_patch_p_kernel(
    const uint8_t* __restrict__ img, int n, int H, int W, int S, int top, int left, int kx, int ky,
    const int* __restrict__ xb, const int* __restrict__ xk, const int* __restrict__ yb, const int* __restrict__ yk,
    NormArgs na, int kpad, bf16* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) uint8_t dyn[];
    __shared__ unsigned short lut[3 * 256];
    const int G = S / P, E = G * P * 3;  // used columns x channels
    const int b = blockIdx.x / G, py = blockIdx.x % G, tid = threadIdx.x;
    const int oy0 = py * P + top, oy1 = oy0 + P - 1;
    const int r0 = yb[2 * oy0], r1 = yb[2 * oy1] + yb[2 * oy1 + 1];
    const int R = r1 - r0, rowb = W * 3;
    uint8_t* in_l = dyn;                                  // [R][W * 3]
    uint8_t* hr = dyn + ((R * rowb + 15) & ~15);          // [R][E]
    uint8_t* vr = hr + ((R * E + 15) & ~15);              // [P][E]
    for (int i = tid; i < 3 * 256; i += 256) {
        const int c = i >> 8, u = i & 255;
        lut[i] = __builtin_bit_cast(unsigned short, f2bf(normalize(u, na.mean[c], na.stdv[c])));
    }
    const uint8_t* src = img + ((long)b * H + r0) * rowb;
    const int nbytes = R * rowb;
    if ((((uintptr_t)src | (unsigned)nbytes) & 15) == 0) {
        for (int i = tid; i < nbytes / 16; i += 256)
            reinterpret_cast<uint4*>(in_l)[i] = reinterpret_cast<const uint4*>(src)[i];
    } else {
        for (int i = tid; i < nbytes; i += 256) in_l[i] = src[i];
    }
    __syncthreads();
    for (int e = tid; e < E; e += 256) {  // horizontal pass
        const int xc = e / 3, c = e - 3 * xc;
        const int xx = xc + left;
        const int xmin = xb[2 * xx], cnt = xb[2 * xx + 1];
        int w[8];
#pragma unroll
        for (int x = 0; x < 8; ++x) w[x] = x < cnt ? xk[xx * kx + x] : 0;
        const uint8_t* sp = in_l + xmin * 3 + c;
        for (int r = 0; r < R; ++r) {
            int sum = 1 << (PREC - 1);
            if constexpr (K > 0) {
#pragma unroll
                for (int x = 0; x < K; ++x) sum += __mul24(sp[r * rowb + 3 * x], w[x]);
            } else {
#pragma unroll
                for (int x = 0; x < 8; ++x)
                    if (x < cnt) sum += sp[r * rowb + 3 * x] * w[x];
            }
            hr[r * E + e] = (uint8_t)clip8(sum);
        }
    }
    __syncthreads();
    for (int e = tid; e < E; e += 256) {  // vertical pass
#pragma unroll 2
        for (int kyy = 0; kyy < P; ++kyy) {
            const int oy = oy0 + kyy;
            const int ymin = yb[2 * oy] - r0, cnt = yb[2 * oy + 1];
            const int* kk = yk + oy * ky;
            int sum = 1 << (PREC - 1);
            if constexpr (K > 0) {
#pragma unroll
                for (int y = 0; y < K; ++y) sum += __mul24(hr[(ymin + y) * E + e], kk[y]);
            } else {
                for (int y = 0; y < cnt; ++y) sum += hr[(ymin + y) * E + e] * kk[y];
            }
            vr[kyy * E + e] = (uint8_t)clip8(sum);
        }
    }
    __syncthreads();
    constexpr int P2 = P * P, C3 = 3 * P2;
    const int NC = kpad / 8, PG = 256 / NC;  // 16-B chunks per patch, patch groups
    const int q = tid % NC, g = tid / NC;
    if (g >= PG) return;
    int off[8], lb[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const int col = q * 8 + e;
        const int c = col / P2, rem = col - c * P2, kyy = rem / P, kxx = rem - kyy * P;
        off[e] = col < C3 ? kyy * E + kxx * 3 + c : -1;
        lb[e] = c * 256;
    }
    bf16* dst = out + ((long)b * G * G + (long)py * G) * kpad + q * 8;
    for (int px = g; px < G; px += PG) {
        u16x8 v;
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = off[e] >= 0 ? lut[lb[e] + vr[off[e] + px * P * 3]] : (unsigned short)0;
        *reinterpret_cast<u16x8*>(dst + (long)px * kpad) = v;
    }
}

// Plain im2col of pixel_values (the HF-API path: get_image_features(pixel_values)).
template <typename T>
__global__ void im2col_kernel(const T* __restrict__ pix, int n, int S, int p, int kpad, bf16* __restrict__ out) {
    const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const int G = S / p;
    const long total = (long)n * G * G * kpad;
    if (t >= total) return;
    const int col = t % kpad;
    const long row = t / kpad;
    if (col >= 3 * p * p) {
        out[t] = f2bf(0.f);
        return;
    }
    const int c = col / (p * p), ky = (col / p) % p, kx = col % p;
    const int px = row % G, py = (row / G) % G;
    const long b = row / ((long)G * G);
    const float v = (float)pix[((b * 3 + c) * S + py * p + ky) * (long)S + px * p + kx];
    out[t] = f2bf(v);
}

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// Host restatement of coeffs_kernel's bounds (same IEEE double operations, no contraction):
// the largest number of input rows one patch row of the fused kernel stages.
#pragma clang fp contract(off)
int fused_max_rows(int in, int out, int S, int top, int p) {
    const double scale = (double)in / out;
    const double fs = scale < 1.0 ? 1.0 : scale;
    const double support = 2.0 * fs;
    auto bounds = [&](int yy, int& lo, int& hi) {
        const double center = (yy + 0.5) * scale;
        lo = (int)(center - support + 0.5);
        if (lo < 0) lo = 0;
        hi = (int)(center + support + 0.5);
        if (hi > in) hi = in;
    };
    int best = 0;
    for (int py = 0; py < S / p; ++py) {
        int lo0, hi0, lo1, hi1;
        bounds(py * p + top, lo0, hi0);
        bounds(py * p + top + p - 1, lo1, hi1);
        best = best > hi1 - lo0 ? best : hi1 - lo0;
    }
    return best;
}

}  // namespace

extern "C" size_t mme_preprocess_workspace_bytes(int n, int H, int W, int rh, int rw) {
    const size_t kx = ksize_for(W, rw), ky = ksize_for(H, rh);
    return align256((size_t)rw * 2 * 4) + align256((size_t)rw * kx * 4) + align256((size_t)rh * 2 * 4) +
           align256((size_t)rh * ky * 4) + align256((size_t)n * H * (size_t)rw * 3);
}

extern "C" int mme_preprocess_u8(const uint8_t* imgs, int n, int H, int W, int rh, int rw, int top, int left, int S,
                                 const float* mean3, const float* std3, int out_kind, int patch, int kpad, void* out,
                                 void* workspace, size_t ws_bytes, void* stream) {
    MME_REQUIRE(imgs && out && workspace && mean3 && std3, "mme_preprocess_u8: null pointer");
    MME_REQUIRE(n >= 0 && H > 0 && W > 0 && rh > 0 && rw > 0 && S > 0, "mme_preprocess_u8: bad sizes");
    MME_REQUIRE(top >= 0 && left >= 0 && top + S <= rh && left + S <= rw, "mme_preprocess_u8: crop outside image");
    MME_REQUIRE(ksize_for(W, rw) <= 64 && ksize_for(H, rh) <= 64, "mme_preprocess_u8: downscale factor too large");
    MME_REQUIRE(ws_bytes >= mme_preprocess_workspace_bytes(n, H, W, rh, rw),
                "mme_preprocess_u8: workspace too small");
    if (out_kind == MME_PIX_PATCHES)
        MME_REQUIRE(patch > 0 && S >= patch && kpad >= 3 * patch * patch && kpad % 8 == 0,
                    "mme_preprocess_u8: bad patch/kpad");
    else
        MME_REQUIRE(out_kind == MME_PIX_F32_NCHW, "mme_preprocess_u8: bad out_kind %d", out_kind);
    if (n == 0) return MME_OK;
    hipStream_t s = as_stream(stream);
    const int kx = ksize_for(W, rw), ky = ksize_for(H, rh);
    char* ws = (char*)workspace;
    int* xb = (int*)ws;
    ws += align256((size_t)rw * 2 * 4);
    int* xk = (int*)ws;
    ws += align256((size_t)rw * kx * 4);
    int* yb = (int*)ws;
    ws += align256((size_t)rh * 2 * 4);
    int* yk = (int*)ws;
    ws += align256((size_t)rh * ky * 4);
    uint8_t* tmp = (uint8_t*)ws;

    hipLaunchKernelGGL(coeffs_kernel, dim3(cdiv(rw, 64)), dim3(64), 0, s, W, rw, kx, xb, xk);
    hipLaunchKernelGGL(coeffs_kernel, dim3(cdiv(rh, 64)), dim3(64), 0, s, H, rh, ky, yb, yk);
    NormArgs na;
    for (int c = 0; c < 3; ++c) {
        na.mean[c] = mean3[c];
        na.stdv[c] = std3[c];
    }
    if (out_kind == MME_PIX_PATCHES) {
        const int R = fused_max_rows(H, rh, S, top, patch);
        if (patch == 14 && kx <= 8 && ky <= 8 && kpad <= 8 * 256) {
            const long E = (long)(S / 14) * 14 * 3;
            const long lds = (((long)R * W * 3 + 15) & ~15L) + ((R * E + 15) & ~15L) + 14 * E;
            // K = 5 taps: the LDS allocation must also cover the reads past a window (the last input
            // row's bytes up to 4 pixels on, the h-pass rows up to 4 rows on: inside hr / vr)
            const long lds5 = lds + 16;
            if (kx == 5 && ky == 5 && lds5 <= FUSED_LDS && R >= 4) {
                hipLaunchKernelGGL((resample_patch_p_kernel<14, 5>), dim3(n * (S / 14)), dim3(256), (unsigned)lds5, s,
                                   imgs, n, H, W, S, top, left, kx, ky, xb, xk, yb, yk, na, kpad, (bf16*)out);
                return mme_check_launch("mme_preprocess_u8");
            }
            if (lds <= FUSED_LDS) {
                hipLaunchKernelGGL(resample_patch_p_kernel<14>, dim3(n * (S / 14)), dim3(256), (unsigned)lds, s, imgs,
                                   n, H, W, S, top, left, kx, ky, xb, xk, yb, yk, na, kpad, (bf16*)out);
                return mme_check_launch("mme_preprocess_u8");
            }
        }
        if ((((long)R * W * 3 + 15) & ~15L) + (long)R * S * 3 <= FUSED_LDS) {
            const int G = S / patch;
            hipLaunchKernelGGL(resample_patch_fused_kernel, dim3(n * G), dim3(256), 0, s, imgs, n, H, W, S, top, left,
                               kx, ky, xb, xk, yb, yk, na, patch, kpad, (bf16*)out);
            return mme_check_launch("mme_preprocess_u8");
        }
    }
    const long th = (long)n * H * S;
    hipLaunchKernelGGL(resample_h_kernel, dim3(cdiv(th, 256)), dim3(256), 0, s, imgs, n, H, W, S, left, kx, xb, xk,
                       tmp);
    if (out_kind == MME_PIX_F32_NCHW) {
        const long tv = (long)n * 3 * S * S;
        hipLaunchKernelGGL(resample_v_nchw_kernel, dim3(cdiv(tv, 256)), dim3(256), 0, s, tmp, n, H, S, top, ky, yb,
                           yk, na, (float*)out);
    } else {
        const int G = S / patch;
        const long tv = (long)n * G * G * kpad;
        hipLaunchKernelGGL(resample_v_patch_kernel, dim3(cdiv(tv, 256)), dim3(256), 0, s, tmp, n, H, S, top, ky, yb,
                           yk, na, patch, kpad, (bf16*)out);
    }
    return mme_check_launch("mme_preprocess_u8");
}

extern "C" int mme_im2col(const void* pixels, int in_is_f32, int n, int S, int patch, int kpad, void* out,
                          void* stream) {
    MME_REQUIRE(pixels && out, "mme_im2col: null pointer");
    MME_REQUIRE(n >= 0 && patch > 0 && S >= patch && kpad >= 3 * patch * patch && kpad % 8 == 0,
                "mme_im2col: bad shape");
    if (n == 0) return MME_OK;
    const int G = S / patch;
    const long tv = (long)n * G * G * kpad;
    if (in_is_f32)
        hipLaunchKernelGGL(im2col_kernel<float>, dim3(cdiv(tv, 256)), dim3(256), 0, as_stream(stream),
                           (const float*)pixels, n, S, patch, kpad, (bf16*)out);
    else
        hipLaunchKernelGGL(im2col_kernel<bf16>, dim3(cdiv(tv, 256)), dim3(256), 0, as_stream(stream),
                           (const bf16*)pixels, n, S, patch, kpad, (bf16*)out);
    return mme_check_launch("mme_im2col");
}
