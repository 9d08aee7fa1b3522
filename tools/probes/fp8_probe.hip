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
    for (int j = 0; j < 32; ++j) {
        pa[j] = A[r * 64 + 32 * h + j];
        pb[j] = B[r * 64 + 32 * h + j];
    }
    f32x16 acc = {};
    acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, acc, 0, 0, 0, 127, 0, 127);
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
    float* dx; uint32_t* dy;
    hipMalloc(&dx, n * 4); hipMalloc(&dy, n);
    hipMemcpy(dx, x.data(), n * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(cvt, dim3(n / 4 / 256), dim3(256), 0, 0, dx, dy, n);
    std::vector<uint8_t> y(n);
    hipMemcpy(y.data(), dy, n, hipMemcpyDeviceToHost);
    int badc = 0, shown = 0;
    for (int i = 0; i < n; ++i) {
        const uint8_t ref = e4m3_encode(x[i]);
        if (y[i] != ref) {
            ++badc;
            if (shown++ < 8) printf("  cvt x=%g gpu=0x%02x (%g) ref=0x%02x (%g)\n", x[i], y[i], e4m3_decode(y[i]), ref,
                                    e4m3_decode(ref));
        }
    }
    printf("%s cvt_pk_fp8_f32 == RNE + saturate (%d / %d mismatches)\n", badc ? "FAIL" : "PASS", badc, n);
    return 0;
}
