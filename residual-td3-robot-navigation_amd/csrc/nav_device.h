// nav_device.h — device helpers shared by the gfx950 kernels of libnavenv.so.
// Compiled with -ffp-contract=off: every f64/f32 product and sum rounds where the reference's
// separate numpy / torch ops round; fused multiply-adds appear only where written as fma().
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "navenv.h"

#define NAV_DEV __device__ __forceinline__

namespace nav {

constexpr int kBlock = 256;
// MI355X: 256 CUs (8 XCDs x 32). A grid's first 2 x kCUs workgroups are dispatched as co-resident
// pairs (b, b + kCUs) on one CU (profiles/r04x wide phase trace).
constexpr int kCUs = 256;

// Philox4x32-10 (Salmon et al. 2011); key (k0,k1), counter (c0..c3).
NAV_DEV uint4 philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                     uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint32_t hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
        const uint32_t hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
        const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c1 = lo1;
        c3 = lo0;
        c0 = n0;
        c2 = n2;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return make_uint4(c0, c1, c2, c3);
}

// 53-bit uniform in [0,1) from two words, numpy's random_sample formula.
NAV_DEV double u01(uint32_t hi, uint32_t lo) {
    return ((double)(hi >> 5) * 67108864.0 + (double)(lo >> 6)) / 9007199254740992.0;
}

// np.clip semantics (NaN propagates).
NAV_DEV double clipd(double v, double lo, double hi) {
    if (v != v) return v;
    return v < lo ? lo : (v > hi ? hi : v);
}

// np.linalg.norm of a 2-vector: sqrt(v.dot(v)); numpy 2.2.6 + OpenBLAS ddot's tail uses fma.
NAV_DEV double norm2(double a0, double a1) { return sqrt(fma(a1, a1, a0 * a0)); }

NAV_DEV int cell_of(double v) {
    int c = (int)v;  // int() truncation; states are >= 0
    return c < 0 ? 0 : (c > 99 ? 99 : c);
}

// environment.py:98-119 Environment.dynamics. Field values come from the interleaved table
// (speed, angle) — one 8-byte gather per call.
// The reference moves by speed * |a| * (cos, sin)(atan2(a1, a0) + rot). Since |a| (cos, sin)
// (atan2(a1, a0)) = (a0, a1), that is speed * R(rot) a: the same f64 displacement up to a few ulp
// of |a| <= 5*sqrt(2) (< 1e-14 absolute, tests hold 1e-11), with one sincos of the small f32 angle
// instead of atan2 + sqrt + sincos of the sum. a = 0, NaN and the +-5 clip behave identically.
// the field value of state s (the cell table lookup of dynamics, separable so it can be issued early)
NAV_DEV float2 field_at(const float2* __restrict__ field, double2 s) {
    return field[cell_of(s.x) * 100 + cell_of(s.y)];
}
NAV_DEV double2 dynamics_f(float2 f, double2 s, double2 a);
NAV_DEV double2 dynamics(const float2* __restrict__ field, double2 s, double2 a) {
    return dynamics_f(field_at(field, s), s, a);
}
NAV_DEV double2 dynamics_f(float2 f, double2 s, double2 a) {
    const double a0 = clipd(a.x, -5.0, 5.0), a1 = clipd(a.y, -5.0, 5.0);
    // NEP 50: float32 field value * 2 * pi is a float32 product chain
    const float rot = (f.y * 2.0f) * 3.14159274101257324f;
    double sr, cr;
    sincos((double)rot, &sr, &cr);
    const double sp = (double)f.x;
    const double hi = 100.0 - 1.0001;
    double2 n;
    n.x = clipd(s.x + sp * (a0 * cr - a1 * sr), 0.0, hi);
    n.y = clipd(s.y + sp * (a0 * sr + a1 * cr), 0.0, hi);
    return n;
}

// environment.py:125 commit test.
NAV_DEV bool in_world(double2 n) { return 0.0 <= n.x && n.x < 100.0 && 0.0 <= n.y && n.y < 100.0; }

// environment.py:135-137 uniform([l, b], [r, t]).
NAV_DEV double2 region_sample(const double* reg, double u0, double u1) {
    return make_double2(reg[0] + (reg[1] - reg[0]) * u0, reg[2] + (reg[3] - reg[2]) * u1);
}

// Box-Muller pair for the exploration noise (the vectorised path's Gaussian source).
NAV_DEV double2 gauss_pair(uint4 w) {
    const double u1 = u01(w.x, w.y), u2 = u01(w.z, w.w);
    const double rad = sqrt(-2.0 * log(1.0 - u1));
    const double th = 6.283185307179586 * u2;
    return make_double2(rad * cos(th), rad * sin(th));
}

// Wave64 sum.
NAV_DEV float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

}  // namespace nav

#define NAV_CHECK_LAUNCH()                                   \
    do {                                                     \
        hipError_t _e = hipGetLastError();                   \
        if (_e != hipSuccess) return -(int)_e;               \
    } while (0)
