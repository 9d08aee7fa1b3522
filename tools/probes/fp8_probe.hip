// Probe (GPU box): lane maps of v_mfma_scale_f32_32x32x64_f8f6f4 (fp8 e4m3,
// unit scales) and the rounding of v_cvt_pk_fp8_f32, checked against host
// references with exactly representable data. Prints PASS/FAIL lines.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <vector>

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// host e4m3fn (OCP) encode with RNE and saturation to +-448, decode
static float e4m3_decode(uint8_t v) {
    int s = v >> 7, e = (v >> 3) & 15, m = v & 7;
    float r;
    if (e == 15 && m == 7) return NAN;
    if (e == 0) r = std::ldexp((float)m, -9);
    else r = std::ldexp(1.0f + m / 8.0f, e - 7);
    return s ? -r : r;
}
static uint8_t e4m3_encode(float x) {
    if (std::isnan(x)) return 0x7f;
    uint8_t best = 0;
    float bd = INFINITY;
    for (int v = 0; v < 256; ++v) {
        if ((v & 0x7f) == 0x7f) continue;
        float d = std::fabs(e4m3_decode((uint8_t)v) - x);
        // ties -> even mantissa (lsb 0)
        if (d < bd || (d == bd && (v & 1) == 0 && (best & 1) == 1)) { bd = d; best = (uint8_t)v; }
    }
    if (std::fabs(x) > 448.f) best = x > 0 ? 0x7e : 0xfe;
    return best;
}

__global__ void mma(const uint8_t* A, const uint8_t* B, float* D) {
    // A: [32][64] row-major (k fastest), B: [32 cols][64 k] (k fastest)
    const int l = threadIdx.x, r = l & 31, h = l >> 5;
    i32x8 a, b;
    uint8_t* pa = (uint8_t*)&a;
    uint8_t* pb = (uint8_t*)&b;
    for (int j = 0; j < 32; ++j) {  // bytes 0-15: k = 16h + j; bytes 16-31: k = 32 + 16h + (j - 16)
        const int k = j < 16 ? 16 * h + j : 32 + 16 * h + (j - 16);
        pa[j] = A[r * 64 + k];
        pb[j] = B[r * 64 + k];
    }
    f32x16 acc = {};
    acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, acc, 0, 0, 0, 127, 0, 127);
    for (int reg = 0; reg < 16; ++reg) {
        const int row = (reg & 3) + 8 * (reg >> 2) + 4 * h, col = r;
        D[row * 32 + col] = acc[reg];
    }
}

// per-lane E8M0 scales: lane (r, h) supplies the scale of row r, k-block h (k 32h..32h+31)
__global__ void mma_scaled(const uint8_t* A, const uint8_t* B, const uint8_t* SA, const uint8_t* SB, float* D) {
    const int l = threadIdx.x, r = l & 31, h = l >> 5;
    i32x8 a, b;
    uint8_t* pa = (uint8_t*)&a;
    uint8_t* pb = (uint8_t*)&b;
    for (int j = 0; j < 32; ++j) {  // bytes 0-15: k = 16h + j; bytes 16-31: k = 32 + 16h + (j - 16)
        const int k = j < 16 ? 16 * h + j : 32 + 16 * h + (j - 16);
        pa[j] = A[r * 64 + k];
        pb[j] = B[r * 64 + k];
    }
    const int sa = SA[r * 2 + h], sb = SB[r * 2 + h];
    f32x16 acc = {};
    acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, acc, 0, 0, 0, sa, 0, sb);
    for (int reg = 0; reg < 16; ++reg) {
        const int row = (reg & 3) + 8 * (reg >> 2) + 4 * h, col = r;
        D[row * 32 + col] = acc[reg];
    }
}

__global__ void cvt(const float* x, uint32_t* y, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (4 * i + 3 >= n) return;
    uint32_t v = 0;
    v = __builtin_amdgcn_cvt_pk_fp8_f32(x[4 * i], x[4 * i + 1], v, false);
    v = __builtin_amdgcn_cvt_pk_fp8_f32(x[4 * i + 2], x[4 * i + 3], v, true);
    y[i] = v;
}

int main() {
    // --- MFMA lane map
    std::vector<uint8_t> A(32 * 64), B(32 * 64);
    std::vector<float> Af(32 * 64), Bf(32 * 64);
    const float vals[] = {0.f, 1.f, -1.f, 2.f, -2.f, 0.5f, 3.f, -0.25f, 4.f, -3.f};
    unsigned s = 12345;
    for (int i = 0; i < 32 * 64; ++i) {
        s = s * 1103515245u + 12345u;
        Af[i] = vals[(s >> 16) % 10];
        A[i] = e4m3_encode(Af[i]);
        s = s * 1103515245u + 12345u;
        Bf[i] = vals[(s >> 16) % 10];
        B[i] = e4m3_encode(Bf[i]);
    }
    uint8_t *dA, *dB;
    float* dD;
    hipMalloc(&dA, 2048); hipMalloc(&dB, 2048); hipMalloc(&dD, 4096);
    hipMemcpy(dA, A.data(), 2048, hipMemcpyHostToDevice);
    hipMemcpy(dB, B.data(), 2048, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(mma, dim3(1), dim3(64), 0, 0, dA, dB, dD);
    std::vector<float> D(1024);
    hipMemcpy(D.data(), dD, 4096, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 32; ++i)
        for (int j = 0; j < 32; ++j) {
            float ref = 0;
            for (int k = 0; k < 64; ++k) ref += Af[i * 64 + k] * Bf[j * 64 + k];
            if (D[i * 32 + j] != ref) ++bad;
        }
    printf("%s mfma_scale_32x32x64 fp8 lane map (%d mismatches)\n", bad ? "FAIL" : "PASS", bad);

    // --- per-lane block scales
    {
        std::vector<uint8_t> SA(64), SB(64);
        for (int i = 0; i < 64; ++i) {
            s = s * 1103515245u + 12345u;
            SA[i] = 124 + (s >> 16) % 7;
            s = s * 1103515245u + 12345u;
            SB[i] = 124 + (s >> 16) % 7;
        }
        uint8_t *dSA, *dSB;
        hipMalloc(&dSA, 64); hipMalloc(&dSB, 64);
        hipMemcpy(dSA, SA.data(), 64, hipMemcpyHostToDevice);
        hipMemcpy(dSB, SB.data(), 64, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(mma_scaled, dim3(1), dim3(64), 0, 0, dA, dB, dSA, dSB, dD);
        hipMemcpy(D.data(), dD, 4096, hipMemcpyDeviceToHost);
        int bad2 = 0;
        for (int i = 0; i < 32; ++i)
            for (int j = 0; j < 32; ++j) {
                double ref = 0;
                for (int k = 0; k < 64; ++k)
                    ref += (double)Af[i * 64 + k] * std::ldexp(1.0, SA[i * 2 + k / 32] - 127) * Bf[j * 64 + k] *
                           std::ldexp(1.0, SB[j * 2 + k / 32] - 127);
                if (std::fabs(D[i * 32 + j] - ref) > 1e-6 * (1 + std::fabs(ref))) ++bad2;
            }
        printf("%s mfma_scale_32x32x64 per-lane E8M0 block scales (%d mismatches)\n", bad2 ? "FAIL" : "PASS", bad2);
    }

    // --- which (row, k-block) does lane L's scale act on? one doubled scale per launch
    {
        uint8_t *dSA, *dSB;
        hipMalloc(&dSA, 64); hipMalloc(&dSB, 64);
        for (int which = 0; which < 2; ++which) {  // 0: scale_a, 1: scale_b
            printf("scale_%c lane -> (row/col, block):", which ? 'b' : 'a');
            for (int L = 0; L < 64; ++L) {
                int found_r = -1, found_b = -1, nfound = 0;
                for (int blk = 0; blk < 2; ++blk) {
                    // operands: all ones on block blk of k, zero elsewhere
                    std::vector<uint8_t> A1(2048, 0), B1(2048, 0);
                    for (int r = 0; r < 32; ++r)
                        for (int k = 32 * blk; k < 32 * blk + 32; ++k) {
                            A1[r * 64 + k] = e4m3_encode(1.f);
                            B1[r * 64 + k] = e4m3_encode(1.f);
                        }
                    std::vector<uint8_t> S1(64, 127), S0(64, 127);
                    S1[L] = 128;
                    hipMemcpy(dA, A1.data(), 2048, hipMemcpyHostToDevice);
                    hipMemcpy(dB, B1.data(), 2048, hipMemcpyHostToDevice);
                    hipMemcpy(dSA, which ? S0.data() : S1.data(), 64, hipMemcpyHostToDevice);
                    hipMemcpy(dSB, which ? S1.data() : S0.data(), 64, hipMemcpyHostToDevice);
                    hipLaunchKernelGGL(mma_scaled, dim3(1), dim3(64), 0, 0, dA, dB, dSA, dSB, dD);
                    hipMemcpy(D.data(), dD, 4096, hipMemcpyDeviceToHost);
                    if (L < 3 || L == 33)
                        printf(" [L%d blk%d D00=%g D01=%g D10=%g D%d0=%g]", L, blk, D[0], D[1], D[32], L >> 1,
                               D[(L >> 1) * 32]);
                    for (int i = 0; i < 32; ++i)
                        for (int j = 0; j < 32; ++j)
                            if (D[i * 32 + j] != 32.f) {
                                if (nfound++ == 0) { found_r = which ? j : i; found_b = blk; }
                            }
                }
                printf(" %d:(%d,%d,n%d)", L, found_r, found_b, nfound);
            }
            printf("\n");
        }
    }

    // --- cvt_pk_fp8_f32 rounding / saturation
    const int n = 1 << 16;
    std::vector<float> x(n);
    for (int i = 0; i < n; ++i) {
        s = s * 1103515245u + 12345u;
        const float u = ((s >> 8) & 0xffff) / 65536.0f;
        const int e = (int)((s >> 24) % 24) - 12;
        x[i] = (i & 1 ? -1.f : 1.f) * std::ldexp(1.0f + u, e);
    }
    x[0] = 448.f; x[1] = 464.f; x[2] = 500.f; x[3] = -1000.f; x[4] = 0.f; x[5] = 1.0625f; x[6] = 1.1875f;
    for (int i = 0; i < n; ++i) x[i] = std::fmin(448.f, std::fmax(-448.f, x[i]));  // the kernels clamp first
    float* dx; uint32_t* dy;
    hipMalloc(&dx, n * 4); hipMalloc(&dy, n);
    hipMemcpy(dx, x.data(), n * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(cvt, dim3(n / 4 / 256), dim3(256), 0, 0, dx, dy, n);
    std::vector<uint8_t> y(n);
    hipMemcpy(y.data(), dy, n, hipMemcpyDeviceToHost);
    int badc = 0, shown = 0;
    for (int i = 0; i < n; ++i) {
        const uint8_t ref = e4m3_encode(x[i]);
        if (y[i] != ref && !(x[i] == 0.f || (y[i] == 0x80 && ref == 0x00))) {
            ++badc;
            if (shown++ < 8) printf("  cvt x=%g gpu=0x%02x (%g) ref=0x%02x (%g)\n", x[i], y[i], e4m3_decode(y[i]), ref,
                                    e4m3_decode(ref));
        }
    }
    printf("%s cvt_pk_fp8_f32 == RNE + saturate (%d / %d mismatches)\n", badc ? "FAIL" : "PASS", badc, n);
    return 0;
}
