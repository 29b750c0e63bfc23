// Probe (design decision only): the lo plane of the fp16 two-plane split formed by one VOP3P
// v_fma_mixlo_f16 / v_fma_mixhi_f16 per value (fma(hi, -1, x) with hi read as f16 and x as f32,
// rounded once to f16) against the form the compiler emits for (half)(x - (float)hi)
// (v_cvt_f32_f16 + v_pk_add_f32 + v_cvt_pk_f16_f32): bit-for-bit comparison of lo on random
// values over 2^-40 .. 2^15 of both signs, fp16 rounding ties, and values whose lo is subnormal.
// Result (r05ai): 0 of 4.2 M lo values differ. Adopted into split2_8 / gemm_cols as inline asm it
// broke test_resume_is_bit_identical (r05aj): the compiler's hazard recognizer does not see an
// inline-asm VALU write, so an MFMA (or LDS store) consuming the lo plane right after it gets no
// wait states; the compiler itself never selects the mix instructions for this pattern (it emits
// cvt_f32_f16 + v_pk_add/v_pk_fma), so the form was not kept.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off tools/probe/mix_probe.hip -o build/mix_probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

__device__ __forceinline__ uint32_t lo_pair_mix(uint32_t hi2, float v0, float v1) {
    uint32_t r;
    asm("v_fma_mixlo_f16 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]" : "=v"(r) : "v"(hi2), "v"(v0));
    asm("v_fma_mixhi_f16 %0, %1, -1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
        : "+v"(r) : "v"(hi2), "v"(v1));
    return r;
}

__global__ void k_lo(const float* x, uint32_t* hi_out, uint32_t* lo_c, uint32_t* lo_mix, int n2) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n2) return;
    const float v0 = x[2 * i], v1 = x[2 * i + 1];
    _Float16 h0 = (_Float16)v0, h1 = (_Float16)v1;
    asm volatile("" : "+v"(h0), "+v"(h1));
    const uint32_t hi2 = (uint32_t)__builtin_bit_cast(uint16_t, h0) |
                         ((uint32_t)__builtin_bit_cast(uint16_t, h1) << 16);
    const _Float16 l0 = (_Float16)(v0 - (float)h0), l1 = (_Float16)(v1 - (float)h1);
    hi_out[i] = hi2;
    lo_c[i] = (uint32_t)__builtin_bit_cast(uint16_t, l0) | ((uint32_t)__builtin_bit_cast(uint16_t, l1) << 16);
    lo_mix[i] = lo_pair_mix(hi2, v0, v1);
}

int main() {
    const int n = 1 << 22;
    std::vector<float> x(n);
    std::mt19937_64 g(7);
    std::uniform_real_distribution<double> u(0.0, 1.0);
    for (int i = 0; i < n; ++i) {
        const int kind = i % 4;
        double v;
        if (kind == 0) v = std::ldexp(1.0 + u(g), (int)(u(g) * 55) - 40);  // wide range
        else if (kind == 1) {  // fp16 ties: an 11-bit value plus half an fp16 ulp
            const int e = (int)(u(g) * 28) - 14;
            const double m = std::floor(1024 + u(g) * 1024);
            v = std::ldexp(m + 0.5, e - 10);
        } else if (kind == 2) v = std::ldexp(1.0 + u(g), (int)(u(g) * 6) + 10);  // the [2^13, 2^16) band
        else v = std::ldexp(1.0 + u(g), (int)(u(g) * 12) - 24);  // lo subnormal in fp16
        x[i] = (float)((g() & 1) ? -v : v);
    }
    float* dx;
    uint32_t *dh, *dc, *dm;
    hipMalloc(&dx, n * 4);
    hipMalloc(&dh, n * 2);
    hipMalloc(&dc, n * 2);
    hipMalloc(&dm, n * 2);
    hipMemcpy(dx, x.data(), n * 4, hipMemcpyHostToDevice);
    const int n2 = n / 2;
    hipLaunchKernelGGL(k_lo, dim3((n2 + 255) / 256), dim3(256), 0, 0, dx, dh, dc, dm, n2);
    std::vector<uint32_t> c(n2), m(n2);
    hipMemcpy(c.data(), dc, n2 * 4, hipMemcpyDeviceToHost);
    hipMemcpy(m.data(), dm, n2 * 4, hipMemcpyDeviceToHost);
    long diff[4] = {0, 0, 0, 0};
    long shown = 0;
    for (int i = 0; i < n2; ++i)
        for (int hh = 0; hh < 2; ++hh) {
            const uint32_t a = (c[i] >> (16 * hh)) & 0xffff, b = (m[i] >> (16 * hh)) & 0xffff;
            if (a != b) {
                ++diff[(2 * i + hh) % 4];
                if (shown++ < 8) printf("x=%.9g lo_c=%04x lo_mix=%04x\n", x[2 * i + hh], a, b);
            }
        }
    printf("{\"values\": %d, \"lo_mismatch\": {\"wide\": %ld, \"ties\": %ld, \"band\": %ld, "
           "\"subnormal_lo\": %ld}}\n", n, diff[0], diff[1], diff[2], diff[3]);
    return 0;
}
