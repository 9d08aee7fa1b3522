// Does an MFMA whose B operand is all zero leave its accumulator bit-identical?
// (round-4 diagnostic for the attention last-tile skip: kind 62 vs 58 / 65 vs 41 differ on a few
// outputs although the skipped block's P is exactly 0.)
// For v_mfma_f32_16x16x32_bf16 and v_mfma_f32_32x32x16_bf16: D = A . 0 + C with random finite A
// (bf16) and C drawn from several magnitude classes (normal values, values near 2^-126, denormals,
// values of the attention accumulators' range), reporting how many D != C bitwise.
// Build: hipcc --offload-arch=gfx950 -O2 tools/mfma_zero_probe.hip -o tools/mfma_zero_probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ void probe16(const bf16x8* a, const float* c, float* d, int zeroB) {
    const int lane = threadIdx.x, w = blockIdx.x;
    const bf16x8 av = a[w * 64 + lane];
    bf16x8 bv;
    for (int e = 0; e < 8; ++e) bv[e] = zeroB ? (__bf16)0.0f : av[(e + 3) & 7];
    f32x4 cv;
    for (int e = 0; e < 4; ++e) cv[e] = c[(w * 64 + lane) * 4 + e];
    const f32x4 r = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, cv, 0, 0, 0);
    for (int e = 0; e < 4; ++e) d[(w * 64 + lane) * 4 + e] = r[e];
}

__global__ void probe32(const bf16x8* a, const float* c, float* d, int zeroB) {
    const int lane = threadIdx.x, w = blockIdx.x;
    const bf16x8 av = a[w * 64 + lane];
    bf16x8 bv;
    for (int e = 0; e < 8; ++e) bv[e] = zeroB ? (__bf16)0.0f : av[(e + 3) & 7];
    f32x16 cv;
    for (int e = 0; e < 16; ++e) cv[e] = c[(w * 64 + lane) * 16 + e];
    const f32x16 r = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, cv, 0, 0, 0);
    for (int e = 0; e < 16; ++e) d[(w * 64 + lane) * 16 + e] = r[e];
}

static uint16_t to_bf16(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    return (uint16_t)((u + 0x7fff + ((u >> 16) & 1)) >> 16);
}

int main() {
    const int W = 4096;  // waves per launch
    std::mt19937 rng(12345);
    std::normal_distribution<float> nd(0.f, 1.5f);
    std::vector<uint16_t> a(W * 64 * 8);
    for (auto& x : a) x = to_bf16(nd(rng));
    const char* cls[] = {"normal(0, 1)", "attention O range (|x| 1e-3..50)", "near 2^-126 (1e-38..1e-37)",
                         "denormal (1e-44..1e-39)", "signed zeros / +-1"};
    bf16x8* da;
    float *dc, *dd;
    hipMalloc(&da, a.size() * 2);
    hipMalloc(&dc, (size_t)W * 64 * 16 * 4);
    hipMalloc(&dd, (size_t)W * 64 * 16 * 4);
    hipMemcpy(da, a.data(), a.size() * 2, hipMemcpyHostToDevice);
    int bad_total = 0;
    for (int k = 0; k < 5; ++k) {
        std::vector<float> c((size_t)W * 64 * 16), d(c.size());
        std::uniform_real_distribution<float> ud(0.f, 1.f);
        for (auto& x : c) {
            const float s = ud(rng) < 0.5f ? -1.f : 1.f;
            switch (k) {
                case 0: x = nd(rng); break;
                case 1: x = s * std::pow(10.f, -3.f + 4.7f * ud(rng)); break;
                case 2: x = s * std::pow(10.f, -38.f + ud(rng)); break;
                case 3: x = s * std::pow(10.f, -44.f + 5.f * ud(rng)); break;
                default: x = ud(rng) < 0.5f ? s * 0.f : s; break;
            }
        }
        hipMemcpy(dc, c.data(), c.size() * 4, hipMemcpyHostToDevice);
        for (int shape = 0; shape < 2; ++shape) {
            const int per = shape ? 16 : 4;
            if (shape)
                hipLaunchKernelGGL(probe32, dim3(W), dim3(64), 0, 0, da, dc, dd, 1);
            else
                hipLaunchKernelGGL(probe16, dim3(W), dim3(64), 0, 0, da, dc, dd, 1);
            hipMemcpy(d.data(), dd, (size_t)W * 64 * per * 4, hipMemcpyDeviceToHost);
            long n = (long)W * 64 * per, diff = 0, zsign = 0;
            for (long i = 0; i < n; ++i) {
                const long lane = i / per, e = i % per;
                const float cv = c[lane * per + e], dv = d[i];
                uint32_t cu, du;
                std::memcpy(&cu, &cv, 4);
                std::memcpy(&du, &dv, 4);
                if (cu != du) {
                    if (cv == dv) ++zsign;
                    else ++diff;
                    if (diff + zsign <= 3)
                        printf("    %s: C %.9g (0x%08x) -> D %.9g (0x%08x)\n", shape ? "32x32x16" : "16x16x32", cv, cu, dv,
                               du);
                }
            }
            printf("%-9s C %-38s: %ld of %ld accumulators changed in value, %ld only in the sign of zero\n",
                   shape ? "32x32x16" : "16x16x32", cls[k], diff, n, zsign);
            bad_total += (int)(diff > 0);
        }
    }
    printf("classes with value changes: %d\n", bad_total);
    return 0;
}
