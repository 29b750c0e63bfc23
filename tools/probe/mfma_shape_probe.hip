// Calibration probe (design decision only): the row kernels' split GEMM (gemm_cols<8, 2>: 64 LDS
// rows x 256 x 256 per 256-thread workgroup, two workgroups per CU, the A operand split once per
// step into a shared LDS stage, B streamed from the L2-resident split image) on the two bf16 MFMA
// shapes at the SAME output tile per wave (64 rows x 64 columns):
//   s32: v_mfma_f32_32x32x16_bf16 — the product's form (2 row tiles x 2 column tiles of 32x32,
//        16-deep k steps, 24 MFMAs per step and wave)
//   s16: v_mfma_f32_16x16x32_bf16 — 4 row tiles x 4 column tiles of 16x16, 32-deep k steps
//        (96 MFMAs per step and wave), the same split image (split_entry) read with the 16x16x32
//        operand map, a 12 KB stage with the 16-B chunk of row r at chunk ^ ((r >> 1) & 3)
//        (conflict-free ds_read_b128 for the 16x16x32 A map)
//   h32: v_mfma_f32_32x32x16_f16 on a TWO-plane fp16 split (x 2^s = hi + lo, 11 + 11 significant
//        bits) with three products (hl, lh, hh): A scaled per workgroup by a power of two from
//        the block's max |a| (formed in the previous layer's epilogue), B per column (its image
//        holds W[k][n] 2^sB_n); the accumulators are unscaled exactly per lane column. Half the
//        MFMAs of s32, a 2-plane stage and image.
// Data: argv[3] = 0 rows uniform in [-1, 1); 1 = dz-like rows (each row uniform in [-1, 1) times
// a log-uniform scale in [1e-9, 6e-5], the magnitude of train_critic's dz at B = 32 768).
// Both on random data, each shape warmed >= 2 s by back-to-back launches first (MI355X_MICROARCH.md
// 'DVFS give-back' 6-7), then timed by events; a stamped build of the same kernel then records per
// workgroup s_memtime / s_memrealtime around its layer loop -> the held clock (median over
// workgroups). Prints per shape: us per launch, bf16 TF/s issued, the clock, the error of workgroup
// 0's output against fp64.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -mllvm -amdgpu-mfma-vgpr-form=1
//        -mllvm -amdgpu-sched-strategy=max-ilp tools/probe/mfma_shape_probe.hip -o build/mfma_shape_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

constexpr int HP = 256, TM = 64, SS = HP + 4, NT = HP / 32, LAYERS = 8, kBlock = 256;
constexpr int NQ = HP / 16;                  // 16-deep steps
constexpr size_t PL = (size_t)NQ * 2 * HP;   // 16-B entries per image plane

__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

struct Split3 {
    bf16x8 h, m, l;
};
__device__ __forceinline__ void split1(float x, __bf16& h, __bf16& m, __bf16& l) {
    h = (__bf16)x;
    const float r = x - (float)h;
    m = (__bf16)r;
    l = (__bf16)(r - (float)m);
}
__device__ __forceinline__ f32x16 mf32(bf16x8 a, bf16x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mf16(bf16x8 a, bf16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
template <typename C, typename F>
__device__ __forceinline__ C x6(const Split3& a, const bf16x8 (&b)[3], C c, F mf) {
    c = mf(a.m, b[1], c);
    c = mf(a.l, b[0], c);
    c = mf(a.h, b[2], c);
    c = mf(a.m, b[0], c);
    c = mf(a.h, b[1], c);
    return mf(a.h, b[0], c);
}

// ---- s32: the product's gemm_cols<8, 2> (one stage buffer, 2 barriers per step, B one step ahead)
__device__ __forceinline__ void gemm32(const float* A, const bf16x8* Bs, __bf16* stage, f32x16 (&acc)[2][2]) {
    constexpr int PP = TM * 16;
    const int tid = threadIdx.x, lane = tid & 63, wv = wave_id(), h = lane >> 5, l32 = lane & 31;
    for (int rt = 0; rt < 2; ++rt)
        for (int j = 0; j < 2; ++j)
            for (int i = 0; i < 16; ++i) acc[rt][j][i] = 0.f;
    const char* Bb = reinterpret_cast<const char*>(Bs);
    const uint32_t o0 = (uint32_t)(h * HP + wv * 32 + l32) * 16u;
    const uint32_t o1 = (uint32_t)(h * HP + (wv + 4) * 32 + l32) * 16u;
    auto ldB = [&](uint32_t o, int p, int q) {
        return *reinterpret_cast<const bf16x8*>(Bb + (o + (uint32_t)((p * PL + q * 2 * HP) * 16)));
    };
    bf16x8 bq0[2][3], bq1[2][3];
    for (int p = 0; p < 3; ++p) {
        bq0[0][p] = ldB(o0, p, 0);
        bq1[0][p] = ldB(o1, p, 0);
    }
    const int sr = tid >> 2, sk = (tid & 3) * 4;
    const float* src = A + sr * SS + sk;
    __bf16* dst = stage + sr * 16 + ((((sk >> 3) ^ (sr >> 3)) & 1) << 3) + (sk & 7);
    const __bf16* frag = stage + l32 * 16 + (((h ^ (l32 >> 3)) & 1) << 3);
    float4 x = *reinterpret_cast<const float4*>(src);
    auto produce = [&](int q) {
        const float v[4] = {x.x, x.y, x.z, x.w};
        bf16x4 ph, pm, pl;
        for (int j = 0; j < 4; ++j) {
            __bf16 a, b, c;
            split1(v[j], a, b, c);
            ph[j] = a;
            pm[j] = b;
            pl[j] = c;
        }
        *reinterpret_cast<bf16x4*>(dst) = ph;
        *reinterpret_cast<bf16x4*>(dst + PP) = pm;
        *reinterpret_cast<bf16x4*>(dst + 2 * PP) = pl;
        if (q + 1 < NQ) x = *reinterpret_cast<const float4*>(src + 16 * (q + 1));
        if (q >= 1)
            for (int p = 0; p < 3; ++p) {
                bq0[q & 1][p] = ldB(o0, p, q);
                bq1[q & 1][p] = ldB(o1, p, q);
            }
    };
    Split3 sa[2];
    auto consume = [&]() {
        __syncthreads();
        for (int rt = 0; rt < 2; ++rt) {
            const __bf16* f = frag + rt * 32 * 16;
            sa[rt].h = *reinterpret_cast<const bf16x8*>(f);
            sa[rt].m = *reinterpret_cast<const bf16x8*>(f + PP);
            sa[rt].l = *reinterpret_cast<const bf16x8*>(f + 2 * PP);
        }
        __syncthreads();
    };
    produce(0);
    consume();
    const bool favored = blockIdx.x >= (gridDim.x >> 1);
    if (favored) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        if (q + 1 < NQ) produce(q + 1);
        Split3 cur[2] = {sa[0], sa[1]};
        for (int rt = 0; rt < 2; ++rt) {
            acc[rt][0] = x6(cur[rt], bq0[q & 1], acc[rt][0], mf32);
            acc[rt][1] = x6(cur[rt], bq1[q & 1], acc[rt][1], mf32);
        }
        if (q + 1 < NQ) consume();
    }
    if (favored) __builtin_amdgcn_s_setprio(0);
}

__device__ __forceinline__ void store32(const f32x16 (&acc)[2][2], float* act) {
    const int lane = threadIdx.x & 63, wv = wave_id(), h = lane >> 5, l32 = lane & 31;
    for (int j = 0; j < 2; ++j) {
        float* col = act + (j == 0 ? wv : wv + 4) * 32 + l32 + 4 * h * SS;
        for (int rt = 0; rt < 2; ++rt)
            for (int i = 0; i < 16; ++i) col[(rt * 32 + (i & 3) + 8 * (i >> 2)) * SS] = fmaxf(acc[rt][j][i], 0.f);
    }
}

// ---- s16: 32-deep steps, stage [3][64 rows][32 k] bf16 (chunk-swizzled), B four 16-column tiles
__device__ __forceinline__ void gemm16(const float* A, const bf16x8* Bs, __bf16* stage, f32x4 (&acc)[4][4]) {
    constexpr int NS = HP / 32;
    constexpr int PP = TM * 32;
    const int tid = threadIdx.x, lane = tid & 63, wv = wave_id();
    for (int rt = 0; rt < 4; ++rt)
        for (int c = 0; c < 4; ++c)
            for (int i = 0; i < 4; ++i) acc[rt][c][i] = 0.f;
    // lane l of column tile c at step s: entry (p, q = 2s + (l >> 5), h = (l >> 4) & 1, n) = B[k =
    // 32s + 8(l >> 4) + j][n], n = wv*64 + 16c + (l & 15)
    const char* Bb = reinterpret_cast<const char*>(Bs);
    const uint32_t ob = (uint32_t)(((lane >> 5) * 2 + ((lane >> 4) & 1)) * HP + wv * 64 + (lane & 15)) * 16u;
    auto ldB = [&](int c, int p, int s) {
        return *reinterpret_cast<const bf16x8*>(Bb + (ob + (uint32_t)((p * PL + (size_t)s * 4 * HP + c * 16) * 16)));
    };
    bf16x8 bq[2][4][3];
    for (int c = 0; c < 4; ++c)
        for (int p = 0; p < 3; ++p) bq[0][c][p] = ldB(c, p, 0);
    // producer: row sr, 16-B chunk ck (k 8ck .. 8ck+7 of the step)
    const int sr = tid >> 2, ck = tid & 3;
    const float* src = A + sr * SS + 8 * ck;
    __bf16* dst = stage + sr * 32 + ((ck ^ ((sr >> 1) & 3)) << 3);
    float4 x0 = *reinterpret_cast<const float4*>(src), x1 = *reinterpret_cast<const float4*>(src + 4);
    auto produce = [&](int s) {
        const float v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
        bf16x8 ph, pm, pl;
        for (int j = 0; j < 8; ++j) {
            __bf16 a, b, c;
            split1(v[j], a, b, c);
            ph[j] = a;
            pm[j] = b;
            pl[j] = c;
        }
        *reinterpret_cast<bf16x8*>(dst) = ph;
        *reinterpret_cast<bf16x8*>(dst + PP) = pm;
        *reinterpret_cast<bf16x8*>(dst + 2 * PP) = pl;
        if (s + 1 < NS) {
            x0 = *reinterpret_cast<const float4*>(src + 32 * (s + 1));
            x1 = *reinterpret_cast<const float4*>(src + 32 * (s + 1) + 4);
        }
        if (s >= 1)
            for (int c = 0; c < 4; ++c)
                for (int p = 0; p < 3; ++p) bq[s & 1][c][p] = ldB(c, p, s);
    };
    Split3 sa[4];
    auto consume = [&]() {
        __syncthreads();
        for (int rt = 0; rt < 4; ++rt) {
            const int r = rt * 16 + (lane & 15);
            const __bf16* f = stage + r * 32 + (((lane >> 4) ^ ((r >> 1) & 3)) << 3);
            sa[rt].h = *reinterpret_cast<const bf16x8*>(f);
            sa[rt].m = *reinterpret_cast<const bf16x8*>(f + PP);
            sa[rt].l = *reinterpret_cast<const bf16x8*>(f + 2 * PP);
        }
        __syncthreads();
    };
    produce(0);
    consume();
    const bool favored = blockIdx.x >= (gridDim.x >> 1);
    if (favored) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        if (s + 1 < NS) produce(s + 1);
        Split3 cur[4] = {sa[0], sa[1], sa[2], sa[3]};
        for (int c = 0; c < 4; ++c)
            for (int rt = 0; rt < 4; ++rt) acc[rt][c] = x6(cur[rt], bq[s & 1][c], acc[rt][c], mf16);
        if (s + 1 < NS) consume();
    }
    if (favored) __builtin_amdgcn_s_setprio(0);
}

__device__ __forceinline__ void store16(const f32x4 (&acc)[4][4], float* act) {
    const int lane = threadIdx.x & 63, wv = wave_id();
    for (int rt = 0; rt < 4; ++rt)
        for (int c = 0; c < 4; ++c)
            for (int i = 0; i < 4; ++i)
                act[(rt * 16 + (lane >> 4) * 4 + i) * SS + wv * 64 + c * 16 + (lane & 15)] = fmaxf(acc[rt][c][i], 0.f);
}

// ---- h32: two fp16 planes, three products
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f32x16 mh32(f16x8 a, f16x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}
constexpr size_t PL2 = PL;  // 16-B entries per fp16 plane (same geometry as the bf16 image)
__device__ __forceinline__ void gemm32h(const float* A, const f16x8* Bs, _Float16* stage, float sa,
                                        f32x16 (&acc)[2][2]) {
    constexpr int PP = TM * 16;
    const int tid = threadIdx.x, lane = tid & 63, wv = wave_id(), h = lane >> 5, l32 = lane & 31;
    for (int rt = 0; rt < 2; ++rt)
        for (int j = 0; j < 2; ++j)
            for (int i = 0; i < 16; ++i) acc[rt][j][i] = 0.f;
    const char* Bb = reinterpret_cast<const char*>(Bs);
    const uint32_t o0 = (uint32_t)(h * HP + wv * 32 + l32) * 16u;
    const uint32_t o1 = (uint32_t)(h * HP + (wv + 4) * 32 + l32) * 16u;
    auto ldB = [&](uint32_t o, int p, int q) {
        return *reinterpret_cast<const f16x8*>(Bb + (o + (uint32_t)((p * PL2 + q * 2 * HP) * 16)));
    };
    f16x8 bq0[2][2], bq1[2][2];
    for (int p = 0; p < 2; ++p) {
        bq0[0][p] = ldB(o0, p, 0);
        bq1[0][p] = ldB(o1, p, 0);
    }
    const int sr = tid >> 2, sk = (tid & 3) * 4;
    const float* src = A + sr * SS + sk;
    _Float16* dst = stage + sr * 16 + ((((sk >> 3) ^ (sr >> 3)) & 1) << 3) + (sk & 7);
    const _Float16* frag = stage + l32 * 16 + (((h ^ (l32 >> 3)) & 1) << 3);
    float4 x = *reinterpret_cast<const float4*>(src);
    auto produce = [&](int q) {
        const float v[4] = {x.x * sa, x.y * sa, x.z * sa, x.w * sa};
        f16x4 ph, pl;
        for (int j = 0; j < 4; ++j) {
            const _Float16 a = (_Float16)v[j];
            ph[j] = a;
            pl[j] = (_Float16)(v[j] - (float)a);
        }
        *reinterpret_cast<f16x4*>(dst) = ph;
        *reinterpret_cast<f16x4*>(dst + PP) = pl;
        if (q + 1 < NQ) x = *reinterpret_cast<const float4*>(src + 16 * (q + 1));
        if (q >= 1)
            for (int p = 0; p < 2; ++p) {
                bq0[q & 1][p] = ldB(o0, p, q);
                bq1[q & 1][p] = ldB(o1, p, q);
            }
    };
    f16x8 ah[2], al[2];
    auto consume = [&]() {
        __syncthreads();
        for (int rt = 0; rt < 2; ++rt) {
            const _Float16* f = frag + rt * 32 * 16;
            ah[rt] = *reinterpret_cast<const f16x8*>(f);
            al[rt] = *reinterpret_cast<const f16x8*>(f + PP);
        }
        __syncthreads();
    };
    produce(0);
    consume();
    const bool favored = blockIdx.x >= (gridDim.x >> 1);
    if (favored) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        if (q + 1 < NQ) produce(q + 1);
        const f16x8 ch[2] = {ah[0], ah[1]}, cl[2] = {al[0], al[1]};
        for (int rt = 0; rt < 2; ++rt)
            for (int j = 0; j < 2; ++j) {
                const f16x8* b = j == 0 ? bq0[q & 1] : bq1[q & 1];
                f32x16 c = acc[rt][j];
                c = mh32(cl[rt], b[0], c);
                c = mh32(ch[rt], b[1], c);
                acc[rt][j] = mh32(ch[rt], b[0], c);
            }
        if (q + 1 < NQ) consume();
    }
    if (favored) __builtin_amdgcn_s_setprio(0);
}

// ---- h32k32: the same products, the stage holding 32 k per round (two 16-deep MFMA steps per
// barrier pair: half the barriers), chunk c of row r at c ^ ((r >> 2) & 3)
__device__ __forceinline__ void gemm32h_k32(const float* A, const f16x8* Bs, _Float16* stage, float sa,
                                            f32x16 (&acc)[2][2]) {
    constexpr int PP = TM * 32;     // fp16 per plane
    constexpr int NR = HP / 32;     // rounds
    const int tid = threadIdx.x, lane = tid & 63, wv = wave_id(), h = lane >> 5, l32 = lane & 31;
    for (int rt = 0; rt < 2; ++rt)
        for (int j = 0; j < 2; ++j)
            for (int i = 0; i < 16; ++i) acc[rt][j][i] = 0.f;
    const char* Bb = reinterpret_cast<const char*>(Bs);
    const uint32_t o0 = (uint32_t)(h * HP + wv * 32 + l32) * 16u;
    const uint32_t o1 = (uint32_t)(h * HP + (wv + 4) * 32 + l32) * 16u;
    auto ldB = [&](uint32_t o, int p, int q) {
        return *reinterpret_cast<const f16x8*>(Bb + (o + (uint32_t)((p * PL2 + q * 2 * HP) * 16)));
    };
    f16x8 bq0[2][2][2], bq1[2][2][2];  // [round parity][sub-step][plane]
    for (int u = 0; u < 2; ++u)
        for (int p = 0; p < 2; ++p) {
            bq0[0][u][p] = ldB(o0, p, u);
            bq1[0][u][p] = ldB(o1, p, u);
        }
    const int sr = tid >> 2, ck = tid & 3;
    const float* src = A + sr * SS + 8 * ck;
    _Float16* dst = stage + sr * 32 + ((ck ^ ((sr >> 2) & 3)) << 3);
    float4 x0 = *reinterpret_cast<const float4*>(src), x1 = *reinterpret_cast<const float4*>(src + 4);
    auto produce = [&](int q) {
        const float v[8] = {x0.x * sa, x0.y * sa, x0.z * sa, x0.w * sa, x1.x * sa, x1.y * sa, x1.z * sa, x1.w * sa};
        f16x8 ph, pl;
        for (int j = 0; j < 8; ++j) ph[j] = (_Float16)v[j];
        asm volatile("" : "+v"(ph));
        for (int j = 0; j < 8; ++j) pl[j] = (_Float16)(v[j] - (float)ph[j]);
        *reinterpret_cast<f16x8*>(dst) = ph;
        *reinterpret_cast<f16x8*>(dst + PP) = pl;
        if (q + 1 < NR) {
            x0 = *reinterpret_cast<const float4*>(src + 32 * (q + 1));
            x1 = *reinterpret_cast<const float4*>(src + 32 * (q + 1) + 4);
        }
        if (q >= 1)
            for (int u = 0; u < 2; ++u)
                for (int p = 0; p < 2; ++p) {
                    bq0[q & 1][u][p] = ldB(o0, p, 2 * q + u);
                    bq1[q & 1][u][p] = ldB(o1, p, 2 * q + u);
                }
    };
    f16x8 ah[2][2], al[2][2];  // [sub-step][row tile]
    auto consume = [&]() {
        __syncthreads();
        for (int u = 0; u < 2; ++u)
            for (int rt = 0; rt < 2; ++rt) {
                const int r = rt * 32 + l32, c = 2 * u + h;
                const _Float16* f = stage + r * 32 + ((c ^ ((r >> 2) & 3)) << 3);
                ah[u][rt] = *reinterpret_cast<const f16x8*>(f);
                al[u][rt] = *reinterpret_cast<const f16x8*>(f + PP);
            }
        __syncthreads();
    };
    produce(0);
    consume();
    const bool favored = blockIdx.x >= (gridDim.x >> 1);
    if (favored) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int q = 0; q < NR; ++q) {
        if (q + 1 < NR) produce(q + 1);
        f16x8 ch[2][2], cl[2][2];
        for (int u = 0; u < 2; ++u)
            for (int rt = 0; rt < 2; ++rt) {
                ch[u][rt] = ah[u][rt];
                cl[u][rt] = al[u][rt];
            }
        for (int u = 0; u < 2; ++u)
            for (int rt = 0; rt < 2; ++rt)
                for (int j = 0; j < 2; ++j) {
                    const f16x8* b = j == 0 ? bq0[q & 1][u] : bq1[q & 1][u];
                    f32x16 c = acc[rt][j];
                    c = mh32(cl[u][rt], b[0], c);
                    c = mh32(ch[u][rt], b[1], c);
                    acc[rt][j] = mh32(ch[u][rt], b[0], c);
                }
        if (q + 1 < NR) consume();
    }
    if (favored) __builtin_amdgcn_s_setprio(0);
}

// ---- h32db: the product's fp16 GEMM with a double-buffered stage and ONE barrier per step: after
// step q's barrier a wave reads step q + 1's fragments (registers, in flight under step q's
// MFMAs) and produces step q + 2 into the buffer step q was read from
__device__ __forceinline__ void gemm32h_db(const float* A, const f16x8* Bs, _Float16* stage, float sa,
                                           f32x16 (&acc)[2][2]) {
    constexpr int PP = TM * 16, SB = 2 * PP;
    const int tid = threadIdx.x, lane = tid & 63, wv = wave_id(), h = lane >> 5, l32 = lane & 31;
    for (int rt = 0; rt < 2; ++rt)
        for (int j = 0; j < 2; ++j)
            for (int i = 0; i < 16; ++i) acc[rt][j][i] = 0.f;
    const char* Bb = reinterpret_cast<const char*>(Bs);
    const uint32_t o0 = (uint32_t)(h * HP + wv * 32 + l32) * 16u;
    const uint32_t o1 = (uint32_t)(h * HP + (wv + 4) * 32 + l32) * 16u;
    auto ldB = [&](uint32_t o, int p, int q) {
        return *reinterpret_cast<const f16x8*>(Bb + (o + (uint32_t)((p * PL2 + q * 2 * HP) * 16)));
    };
    f16x8 bq0[2][2], bq1[2][2];
    for (int p = 0; p < 2; ++p) {
        bq0[0][p] = ldB(o0, p, 0);
        bq1[0][p] = ldB(o1, p, 0);
    }
    const int sr = tid >> 2, sk = (tid & 3) * 4;
    const float* src = A + sr * SS + sk;
    _Float16* dst = stage + sr * 16 + ((((sk >> 3) ^ (sr >> 3)) & 1) << 3) + (sk & 7);
    const _Float16* frag = stage + l32 * 16 + (((h ^ (l32 >> 3)) & 1) << 3);
    float4 x = *reinterpret_cast<const float4*>(src);
    auto produce = [&](int q) {  // step q into buffer q & 1; the next x; B of step q - 1 + 1
        const float v[4] = {x.x * sa, x.y * sa, x.z * sa, x.w * sa};
        f16x4 ph, pl;
        for (int j = 0; j < 4; ++j) ph[j] = (_Float16)v[j];
        asm volatile("" : "+v"(ph));
        for (int j = 0; j < 4; ++j) pl[j] = (_Float16)(v[j] - (float)ph[j]);
        _Float16* d = dst + (q & 1) * SB;
        *reinterpret_cast<f16x4*>(d) = ph;
        *reinterpret_cast<f16x4*>(d + PP) = pl;
        if (q + 1 < NQ) x = *reinterpret_cast<const float4*>(src + 16 * (q + 1));
    };
    f16x8 ah[2][2], al[2][2];  // [step parity][row tile]
    auto readf = [&](int q) {
        const _Float16* fq = frag + (q & 1) * SB;
        for (int rt = 0; rt < 2; ++rt) {
            ah[q & 1][rt] = *reinterpret_cast<const f16x8*>(fq + rt * 32 * 16);
            al[q & 1][rt] = *reinterpret_cast<const f16x8*>(fq + rt * 32 * 16 + PP);
        }
    };
    produce(0);
    produce(1);
    __syncthreads();
    readf(0);
    const bool favored = blockIdx.x >= (gridDim.x >> 1);
    if (favored) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        __syncthreads();
        if (q + 1 < NQ) {
            readf(q + 1);
            for (int p = 0; p < 2; ++p) {
                bq0[(q + 1) & 1][p] = ldB(o0, p, q + 1);
                bq1[(q + 1) & 1][p] = ldB(o1, p, q + 1);
            }
        }
        if (q + 2 < NQ) produce(q + 2);
        for (int rt = 0; rt < 2; ++rt)
            for (int j = 0; j < 2; ++j) {
                const f16x8* b = j == 0 ? bq0[q & 1] : bq1[q & 1];
                f32x16 c = acc[rt][j];
                c = mh32(al[q & 1][rt], b[0], c);
                c = mh32(ah[q & 1][rt], b[1], c);
                acc[rt][j] = mh32(ah[q & 1][rt], b[0], c);
            }
    }
    if (favored) __builtin_amdgcn_s_setprio(0);
}

__device__ __forceinline__ float wave_max(float v);
__device__ __forceinline__ float pow2_scale(float amax);

// ---- h32pre: the A operand kept in LDS as its two scaled fp16 planes [2][64][HP + 8] (written by the
// previous layer's epilogue, 4 B per element like the f32 rows): no split stage, no barrier and
// no split VALU inside the GEMM; every wave reads its fragments straight from the planes
constexpr int PS2 = HP + 8;  // plane row stride (fp16)
__device__ __forceinline__ void gemm32h_pre(const _Float16* P, const f16x8* Bs, f32x16 (&acc)[2][2]) {
    constexpr int PPL = TM * PS2;
    const int lane = threadIdx.x & 63, wv = wave_id(), h = lane >> 5, l32 = lane & 31;
    for (int rt = 0; rt < 2; ++rt)
        for (int j = 0; j < 2; ++j)
            for (int i = 0; i < 16; ++i) acc[rt][j][i] = 0.f;
    const char* Bb = reinterpret_cast<const char*>(Bs);
    const uint32_t o0 = (uint32_t)(h * HP + wv * 32 + l32) * 16u;
    const uint32_t o1 = (uint32_t)(h * HP + (wv + 4) * 32 + l32) * 16u;
    auto ldB = [&](uint32_t o, int p, int q) {
        return *reinterpret_cast<const f16x8*>(Bb + (o + (uint32_t)((p * PL2 + q * 2 * HP) * 16)));
    };
    f16x8 bq0[2][2], bq1[2][2];
    for (int p = 0; p < 2; ++p) {
        bq0[0][p] = ldB(o0, p, 0);
        bq1[0][p] = ldB(o1, p, 0);
    }
    const _Float16* arow = P + l32 * PS2 + 8 * h;
    f16x8 ah[2][2], al[2][2];
    auto rdA = [&](int q) {
        for (int rt = 0; rt < 2; ++rt) {
            ah[q & 1][rt] = *reinterpret_cast<const f16x8*>(arow + rt * 32 * PS2 + 16 * q);
            al[q & 1][rt] = *reinterpret_cast<const f16x8*>(arow + rt * 32 * PS2 + 16 * q + PPL);
        }
    };
    rdA(0);
    const bool favored = blockIdx.x >= (gridDim.x >> 1);
    if (favored) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        if (q + 1 < NQ) {
            rdA(q + 1);
            for (int p = 0; p < 2; ++p) {
                bq0[(q + 1) & 1][p] = ldB(o0, p, q + 1);
                bq1[(q + 1) & 1][p] = ldB(o1, p, q + 1);
            }
        }
        for (int rt = 0; rt < 2; ++rt)
            for (int j = 0; j < 2; ++j) {
                const f16x8* b = j == 0 ? bq0[q & 1] : bq1[q & 1];
                f32x16 c = acc[rt][j];
                c = mh32(al[q & 1][rt], b[0], c);
                c = mh32(ah[q & 1][rt], b[1], c);
                acc[rt][j] = mh32(ah[q & 1][rt], b[0], c);
            }
    }
    if (favored) __builtin_amdgcn_s_setprio(0);
}

// epilogue of h32pre: relu(acc * unscale), the block max (wave maxima through LDS, a barrier),
// then the scaled two-plane split stored into the planes (16-bit stores, C layout)
__device__ __forceinline__ void store_planes_h(f32x16 (&acc)[2][2], _Float16* P, float* wmax,
                                               const float* colinv, float& inv_next) {
    constexpr int PPL = TM * PS2;
    const int lane = threadIdx.x & 63, wv = wave_id(), h = lane >> 5, l32 = lane & 31;
    float mm = 0.f;
    for (int j = 0; j < 2; ++j) {
        const float u = inv_next * colinv[(j == 0 ? wv : wv + 4) * 32 + l32];
        for (int rt = 0; rt < 2; ++rt)
            for (int i = 0; i < 16; ++i) {
                acc[rt][j][i] = fmaxf(acc[rt][j][i] * u, 0.f);
                mm = fmaxf(mm, acc[rt][j][i]);
            }
    }
    mm = wave_max(mm);
    if (lane == 0) wmax[wv] = mm;
    __syncthreads();
    const float amax = fmaxf(fmaxf(wmax[0], wmax[1]), fmaxf(wmax[2], wmax[3]));
    const float sa = pow2_scale(amax);
    inv_next = 1.f / sa;
    for (int j = 0; j < 2; ++j) {
        _Float16* col = P + (j == 0 ? wv : wv + 4) * 32 + l32 + 4 * h * PS2;
        for (int rt = 0; rt < 2; ++rt)
            for (int i = 0; i < 16; ++i) {
                const float v = acc[rt][j][i] * sa;
                const _Float16 hh = (_Float16)v;
                const int o = (rt * 32 + (i & 3) + 8 * (i >> 2)) * PS2;
                col[o] = hh;
                col[o + PPL] = (_Float16)(v - (float)hh);
            }
    }
}

// ---- h16: two fp16 planes, three products on v_mfma_f32_16x16x32_f16 (gemm16's tiling)
__device__ __forceinline__ f32x4 mh16(f16x8 a, f16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ void gemm16h(const float* A, const f16x8* Bs, _Float16* stage, float sa,
                                        f32x4 (&acc)[4][4]) {
    constexpr int NS = HP / 32;
    constexpr int PP = TM * 32;
    const int tid = threadIdx.x, lane = tid & 63, wv = wave_id();
    for (int rt = 0; rt < 4; ++rt)
        for (int c = 0; c < 4; ++c)
            for (int i = 0; i < 4; ++i) acc[rt][c][i] = 0.f;
    const char* Bb = reinterpret_cast<const char*>(Bs);
    const uint32_t ob = (uint32_t)(((lane >> 5) * 2 + ((lane >> 4) & 1)) * HP + wv * 64 + (lane & 15)) * 16u;
    auto ldB = [&](int c, int p, int s) {
        return *reinterpret_cast<const f16x8*>(Bb + (ob + (uint32_t)((p * PL2 + (size_t)s * 4 * HP + c * 16) * 16)));
    };
    f16x8 bq[2][4][2];
    for (int c = 0; c < 4; ++c)
        for (int p = 0; p < 2; ++p) bq[0][c][p] = ldB(c, p, 0);
    const int sr = tid >> 2, ck = tid & 3;
    const float* src = A + sr * SS + 8 * ck;
    _Float16* dst = stage + sr * 32 + ((ck ^ ((sr >> 1) & 3)) << 3);
    float4 x0 = *reinterpret_cast<const float4*>(src), x1 = *reinterpret_cast<const float4*>(src + 4);
    auto produce = [&](int s) {
        const float v[8] = {x0.x * sa, x0.y * sa, x0.z * sa, x0.w * sa, x1.x * sa, x1.y * sa, x1.z * sa, x1.w * sa};
        f16x8 ph, pl;
        for (int j = 0; j < 8; ++j) ph[j] = (_Float16)v[j];
        asm volatile("" : "+v"(ph));
        for (int j = 0; j < 8; ++j) pl[j] = (_Float16)(v[j] - (float)ph[j]);
        *reinterpret_cast<f16x8*>(dst) = ph;
        *reinterpret_cast<f16x8*>(dst + PP) = pl;
        if (s + 1 < NS) {
            x0 = *reinterpret_cast<const float4*>(src + 32 * (s + 1));
            x1 = *reinterpret_cast<const float4*>(src + 32 * (s + 1) + 4);
        }
        if (s >= 1)
            for (int c = 0; c < 4; ++c)
                for (int p = 0; p < 2; ++p) bq[s & 1][c][p] = ldB(c, p, s);
    };
    f16x8 ah[4], al[4];
    auto consume = [&]() {
        __syncthreads();
        for (int rt = 0; rt < 4; ++rt) {
            const int r = rt * 16 + (lane & 15);
            const _Float16* f = stage + r * 32 + (((lane >> 4) ^ ((r >> 1) & 3)) << 3);
            ah[rt] = *reinterpret_cast<const f16x8*>(f);
            al[rt] = *reinterpret_cast<const f16x8*>(f + PP);
        }
        __syncthreads();
    };
    produce(0);
    consume();
    const bool favored = blockIdx.x >= (gridDim.x >> 1);
    if (favored) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        if (s + 1 < NS) produce(s + 1);
        f16x8 ch[4], cl[4];
        for (int rt = 0; rt < 4; ++rt) {
            ch[rt] = ah[rt];
            cl[rt] = al[rt];
        }
        for (int c = 0; c < 4; ++c)
            for (int rt = 0; rt < 4; ++rt) {
                f32x4 a4 = acc[rt][c];
                a4 = mh16(cl[rt], bq[s & 1][c][0], a4);
                a4 = mh16(ch[rt], bq[s & 1][c][1], a4);
                acc[rt][c] = mh16(ch[rt], bq[s & 1][c][0], a4);
            }
        if (s + 1 < NS) consume();
    }
    if (favored) __builtin_amdgcn_s_setprio(0);
}

__device__ __forceinline__ float wave_max(float v) {
    for (int m = 32; m >= 1; m >>= 1) v = fmaxf(v, __shfl_xor(v, m, 64));
    return v;
}
// power-of-two scale putting the block's max |a| in [2^13, 2^14)
__device__ __forceinline__ float pow2_scale(float amax) {
    if (!(amax > 0.f)) return 1.f;
    int e;
    frexpf(amax, &e);
    return ldexpf(1.f, 14 - e);
}

// ---- h32w8: 128 rows per workgroup, 8 waves (2 per SIMD, one workgroup per CU): wave w owns the
// 64 rows (w >> 2) and the column tiles (w & 3), (w & 3) + 4 — the same wave tile, half the B
// image reads per row (the B planes stream from L2 once per 128 rows instead of once per 64)
constexpr int TM8 = 128;
__device__ __forceinline__ void gemm32h_w8(const float* A, const f16x8* Bs, _Float16* stage, float sa,
                                           f32x16 (&acc)[2][2]) {
    constexpr int PP = TM8 * 16;
    const int tid = threadIdx.x, lane = tid & 63, wv = wave_id(), h = lane >> 5, l32 = lane & 31;
    const int ct = wv & 3, rh = wv >> 2;
    for (int rt = 0; rt < 2; ++rt)
        for (int j = 0; j < 2; ++j)
            for (int i = 0; i < 16; ++i) acc[rt][j][i] = 0.f;
    const char* Bb = reinterpret_cast<const char*>(Bs);
    const uint32_t o0 = (uint32_t)(h * HP + ct * 32 + l32) * 16u;
    const uint32_t o1 = (uint32_t)(h * HP + (ct + 4) * 32 + l32) * 16u;
    auto ldB = [&](uint32_t o, int p, int q) {
        return *reinterpret_cast<const f16x8*>(Bb + (o + (uint32_t)((p * PL2 + q * 2 * HP) * 16)));
    };
    f16x8 bq0[2][2], bq1[2][2];
    for (int p = 0; p < 2; ++p) {
        bq0[0][p] = ldB(o0, p, 0);
        bq1[0][p] = ldB(o1, p, 0);
    }
    const int sr = tid >> 2, sk = (tid & 3) * 4;  // 512 threads: 128 rows x 4
    const float* src = A + sr * SS + sk;
    _Float16* dst = stage + sr * 16 + ((((sk >> 3) ^ (sr >> 3)) & 1) << 3) + (sk & 7);
    const _Float16* frag = stage + (rh * 64 + l32) * 16 + (((h ^ (l32 >> 3)) & 1) << 3);
    float4 x = *reinterpret_cast<const float4*>(src);
    auto produce = [&](int q) {
        const float v[4] = {x.x * sa, x.y * sa, x.z * sa, x.w * sa};
        f16x4 ph, pl;
        for (int j = 0; j < 4; ++j) ph[j] = (_Float16)v[j];
        asm volatile("" : "+v"(ph));
        for (int j = 0; j < 4; ++j) pl[j] = (_Float16)(v[j] - (float)ph[j]);
        *reinterpret_cast<f16x4*>(dst) = ph;
        *reinterpret_cast<f16x4*>(dst + PP) = pl;
        if (q + 1 < NQ) x = *reinterpret_cast<const float4*>(src + 16 * (q + 1));
        if (q >= 1)
            for (int p = 0; p < 2; ++p) {
                bq0[q & 1][p] = ldB(o0, p, q);
                bq1[q & 1][p] = ldB(o1, p, q);
            }
    };
    f16x8 ah[2], al[2];
    auto consume = [&]() {
        __syncthreads();
        for (int rt = 0; rt < 2; ++rt) {
            const _Float16* f = frag + rt * 32 * 16;
            ah[rt] = *reinterpret_cast<const f16x8*>(f);
            al[rt] = *reinterpret_cast<const f16x8*>(f + PP);
        }
        __syncthreads();
    };
    produce(0);
    consume();
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        if (q + 1 < NQ) produce(q + 1);
        const f16x8 ch[2] = {ah[0], ah[1]}, cl[2] = {al[0], al[1]};
        for (int rt = 0; rt < 2; ++rt)
            for (int j = 0; j < 2; ++j) {
                const f16x8* b = j == 0 ? bq0[q & 1] : bq1[q & 1];
                f32x16 c = acc[rt][j];
                c = mh32(cl[rt], b[0], c);
                c = mh32(ch[rt], b[1], c);
                acc[rt][j] = mh32(ch[rt], b[0], c);
            }
        if (q + 1 < NQ) consume();
    }
}

template <bool STAMP>
__global__ __launch_bounds__(512, 1) void k_probe_w8(const float* rows, float* out, unsigned long long* stamps,
                                                     const f16x8* Bh, const float* colinv) {
    extern __shared__ __attribute__((aligned(16))) float act[];
    _Float16* stage = reinterpret_cast<_Float16*>(act + TM8 * SS);
    float* wmax = act + TM8 * SS + TM8 * 16;  // past the 2-plane stage (fp16: TM8*16*2*2 B)
    const int tid = threadIdx.x;
    const float* src = rows + (size_t)(blockIdx.x & 3) * TM8 * HP;
    float m = 0.f;
    for (int i = tid; i < TM8 * HP; i += 512) {
        act[(i / HP) * SS + i % HP] = src[i];
        m = fmaxf(m, fabsf(src[i]));
    }
    m = wave_max(m);
    if ((tid & 63) == 0) wmax[tid >> 6] = m;
    __syncthreads();
    if (STAMP && tid == 0) {
        stamps[blockIdx.x * 4 + 0] = __builtin_amdgcn_s_memtime();
        stamps[blockIdx.x * 4 + 1] = __builtin_amdgcn_s_memrealtime();
    }
    const int lane = tid & 63, wv = wave_id(), h = lane >> 5, l32 = lane & 31, ct = wv & 3, rh = wv >> 2;
    for (int L = 0; L < LAYERS; ++L) {
        float amax = 0.f;
        for (int w = 0; w < 8; ++w) amax = fmaxf(amax, wmax[w]);
        const float sa = pow2_scale(amax), inva = 1.f / sa;
        f32x16 acc[2][2];
        gemm32h_w8(act, Bh, stage, sa, acc);
        __syncthreads();
        float mm = 0.f;
        for (int j = 0; j < 2; ++j) {
            const float u = inva * colinv[(j == 0 ? ct : ct + 4) * 32 + l32];
            float* col = act + (j == 0 ? ct : ct + 4) * 32 + l32 + 4 * h * SS + rh * 64 * SS;
            for (int rt = 0; rt < 2; ++rt)
                for (int i = 0; i < 16; ++i) {
                    const float v = fmaxf(acc[rt][j][i] * u, 0.f);
                    col[(rt * 32 + (i & 3) + 8 * (i >> 2)) * SS] = v;
                    mm = fmaxf(mm, v);
                }
        }
        mm = wave_max(mm);
        if (lane == 0) wmax[wv] = mm;
        __syncthreads();
    }
    if (STAMP && tid == 0) {
        stamps[blockIdx.x * 4 + 2] = __builtin_amdgcn_s_memtime();
        stamps[blockIdx.x * 4 + 3] = __builtin_amdgcn_s_memrealtime();
    }
    if (blockIdx.x < 4)
        for (int i = tid; i < TM8 * HP; i += 512) out[(size_t)blockIdx.x * TM8 * HP + i] = act[(i / HP) * SS + i % HP];
}

// stamps[block][0..3] = memtime, memrealtime at the layer loop's start, then at its end
template <int SHAPE, bool STAMP>
__global__ __launch_bounds__(kBlock, 2) void k_probe(const float* rows, const bf16x8* Bs, float* out,
                                                     unsigned long long* stamps, const f16x8* Bh,
                                                     const float* colinv) {
    extern __shared__ __attribute__((aligned(16))) float act[];
    __bf16* stage = reinterpret_cast<__bf16*>(act + TM * SS);
    float* wmax = act + TM * SS + 3 * TM * 32 / 2;  // [4] wave maxima (past the largest stage)
    const int tid = threadIdx.x;
    const float* src = rows + (size_t)(blockIdx.x & 7) * TM * HP;
    float m = 0.f;
    for (int i = tid; i < TM * HP; i += kBlock) {
        act[(i / HP) * SS + i % HP] = src[i];
        m = fmaxf(m, fabsf(src[i]));
    }
    m = wave_max(m);
    if ((tid & 63) == 0) wmax[tid >> 6] = m;
    __syncthreads();
    float inv_next = 1.f;
    _Float16* planes = reinterpret_cast<_Float16*>(act) + 0;  // SHAPE 7: planes over the rows region
    if constexpr (SHAPE == 7) {
        // rows -> scaled planes (f32 rows of the probe input; the planes take 4 B per element)
        const float sa = pow2_scale(fmaxf(fmaxf(wmax[0], wmax[1]), fmaxf(wmax[2], wmax[3])));
        inv_next = 1.f / sa;
        float tmp[TM * HP / kBlock];
        for (int t = 0; t < TM * HP / kBlock; ++t) {
            const int i = tid + t * kBlock;
            tmp[t] = act[(i / HP) * SS + i % HP] * sa;
        }
        __syncthreads();
        for (int t = 0; t < TM * HP / kBlock; ++t) {
            const int i = tid + t * kBlock;
            const _Float16 hh = (_Float16)tmp[t];
            planes[(i / HP) * PS2 + i % HP] = hh;
            planes[(i / HP) * PS2 + i % HP + TM * PS2] = (_Float16)(tmp[t] - (float)hh);
        }
        __syncthreads();
    }
    if (STAMP && tid == 0) {
        stamps[blockIdx.x * 4 + 0] = __builtin_amdgcn_s_memtime();
        stamps[blockIdx.x * 4 + 1] = __builtin_amdgcn_s_memrealtime();
    }
    for (int L = 0; L < LAYERS; ++L) {
        if constexpr (SHAPE == 7) {
            f32x16 acc[2][2];
            gemm32h_pre(planes, Bh, acc);
            __syncthreads();  // every wave has read the planes
            store_planes_h(acc, planes, wmax, colinv, inv_next);
        } else if constexpr (SHAPE == 32) {
            f32x16 acc[2][2];
            gemm32(act, Bs, stage, acc);
            __syncthreads();
            store32(acc, act);
        } else if constexpr (SHAPE == 5) {
            const float amax = fmaxf(fmaxf(wmax[0], wmax[1]), fmaxf(wmax[2], wmax[3]));
            const float sa = pow2_scale(amax), inva = 1.f / sa;
            f32x4 acc[4][4];
            gemm16h(act, Bh, reinterpret_cast<_Float16*>(stage), sa, acc);
            __syncthreads();
            const int lane = tid & 63, wv = wave_id();
            float mm = 0.f;
            for (int c = 0; c < 4; ++c) {
                const float u = inva * colinv[wv * 64 + c * 16 + (lane & 15)];
                for (int rt = 0; rt < 4; ++rt)
                    for (int i = 0; i < 4; ++i) {
                        acc[rt][c][i] = fmaxf(acc[rt][c][i] * u, 0.f);
                        mm = fmaxf(mm, acc[rt][c][i]);
                    }
            }
            store16(acc, act);
            mm = wave_max(mm);
            if (lane == 0) wmax[wv] = mm;
        } else if constexpr (SHAPE == 3 || SHAPE == 4 || SHAPE == 6) {
            const float amax = fmaxf(fmaxf(wmax[0], wmax[1]), fmaxf(wmax[2], wmax[3]));
            const float sa = pow2_scale(amax), inva = 1.f / sa;  // exact: powers of two
            f32x16 acc[2][2];
            if constexpr (SHAPE == 3)
                gemm32h(act, Bh, reinterpret_cast<_Float16*>(stage), sa, acc);
            else if constexpr (SHAPE == 6)
                gemm32h_db(act, Bh, reinterpret_cast<_Float16*>(stage), sa, acc);
            else
                gemm32h_k32(act, Bh, reinterpret_cast<_Float16*>(stage), sa, acc);
            __syncthreads();
            const int lane = tid & 63, wv = wave_id();
            float mm = 0.f;
            for (int j = 0; j < 2; ++j) {
                const float u = inva * colinv[(j == 0 ? wv : wv + 4) * 32 + (lane & 31)];
                for (int rt = 0; rt < 2; ++rt)
                    for (int i = 0; i < 16; ++i) {
                        acc[rt][j][i] = fmaxf(acc[rt][j][i] * u, 0.f);
                        mm = fmaxf(mm, acc[rt][j][i]);
                    }
            }
            store32(acc, act);
            mm = wave_max(mm);
            if (lane == 0) wmax[wv] = mm;
        } else {
            f32x4 acc[4][4];
            gemm16(act, Bs, stage, acc);
            __syncthreads();
            store16(acc, act);
        }
        __syncthreads();
    }
    if (STAMP && tid == 0) {
        stamps[blockIdx.x * 4 + 2] = __builtin_amdgcn_s_memtime();
        stamps[blockIdx.x * 4 + 3] = __builtin_amdgcn_s_memrealtime();
    }
    if (blockIdx.x < 8) {
        if constexpr (SHAPE == 7) {
            for (int i = tid; i < TM * HP; i += kBlock) {
                const int o = (i / HP) * PS2 + i % HP;
                out[(size_t)blockIdx.x * TM * HP + i] =
                    ((float)planes[o] + (float)planes[o + TM * PS2]) * inv_next;
            }
        } else {
            for (int i = tid; i < TM * HP; i += kBlock) out[(size_t)blockIdx.x * TM * HP + i] = act[(i / HP) * SS + i % HP];
        }
    }
}

static uint16_t bf16_rn(float x) {
    uint32_t u;
    memcpy(&u, &x, 4);
    u += 0x7FFF + ((u >> 16) & 1);
    return (uint16_t)(u >> 16);
}
static float bf16_f(uint16_t b) {
    uint32_t u = (uint32_t)b << 16;
    float f;
    memcpy(&f, &u, 4);
    return f;
}

int main(int argc, char** argv) {
    const int blocks = argc > 1 ? atoi(argv[1]) : 512;  // 512 = two workgroups per CU, one wave
    const double warm_s = argc > 2 ? atof(argv[2]) : 2.0;
    const int data = argc > 3 ? atoi(argv[3]) : 0;
    std::vector<float> rows(8 * TM * HP), W(HP * HP);
    unsigned s = 12345;
    auto rnd = [&]() {
        s = s * 1664525u + 1013904223u;
        return ((s >> 8) & 0xffff) / 65536.0f * 2.f - 1.f;
    };
    for (auto& v : rows) v = rnd();
    if (data == 1)
        for (int r = 0; r < 8 * TM; ++r) {
            const float sc = expf(logf(1e-9f) + (rnd() * 0.5f + 0.5f) * (logf(6e-5f) - logf(1e-9f)));
            for (int k = 0; k < HP; ++k) rows[(size_t)r * HP + k] *= sc;
        }
    // weights scaled so the rows keep their magnitude through 8 ReLU layers (random mantissas in
    // every plane: the DVFS-relevant case)
    const float bound = sqrtf(6.f / HP) * 1.4f;
    for (auto& v : W) v = rnd() * bound;
    std::vector<uint16_t> Bs((size_t)3 * PL * 8);
    for (int k = 0; k < HP; ++k)
        for (int n = 0; n < HP; ++n) {
            const float x = W[(size_t)k * HP + n];
            const uint16_t hb = bf16_rn(x);
            const float r = x - bf16_f(hb);
            const uint16_t mb = bf16_rn(r);
            const uint16_t lb = bf16_rn(r - bf16_f(mb));
            const int q = k / 16, h = (k % 16) / 8, j = k % 8;
            for (int p = 0; p < 3; ++p)
                Bs[((((size_t)p * NQ + q) * 2 + h) * HP + n) * 8 + j] = p == 0 ? hb : p == 1 ? mb : lb;
        }
    // fp16 image: W[k][n] 2^sB_n in two planes, sB_n putting column n's max |W| in [2^13, 2^14)
    std::vector<_Float16> Bh((size_t)2 * PL * 8);
    std::vector<float> colinv(HP);
    for (int n = 0; n < HP; ++n) {
        float cm = 0.f;
        for (int k = 0; k < HP; ++k) cm = fmaxf(cm, fabsf(W[(size_t)k * HP + n]));
        int e;
        frexpf(cm, &e);
        const float sc = ldexpf(1.f, 14 - e);
        colinv[n] = 1.f / sc;
        for (int k = 0; k < HP; ++k) {
            const float x = W[(size_t)k * HP + n] * sc;
            const _Float16 hb = (_Float16)x;
            const _Float16 lb = (_Float16)(x - (float)hb);
            const int q = k / 16, h = (k % 16) / 8, j = k % 8;
            Bh[((((size_t)0 * NQ + q) * 2 + h) * HP + n) * 8 + j] = hb;
            Bh[((((size_t)1 * NQ + q) * 2 + h) * HP + n) * 8 + j] = lb;
        }
    }
    float *d_rows, *d_out, *d_colinv;
    f16x8* d_Bh;
    bf16x8* d_Bs;
    unsigned long long* d_st;
    hipMalloc(&d_rows, rows.size() * 4);
    hipMalloc(&d_Bs, Bs.size() * 2);
    hipMalloc(&d_out, (size_t)8 * TM * HP * 4);
    hipMalloc(&d_st, (size_t)blocks * 4 * 8);
    hipMemcpy(d_rows, rows.data(), rows.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(d_Bs, Bs.data(), Bs.size() * 2, hipMemcpyHostToDevice);
    hipMalloc(&d_Bh, Bh.size() * 2);
    hipMalloc(&d_colinv, HP * 4);
    hipMemcpy(d_Bh, Bh.data(), Bh.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(d_colinv, colinv.data(), HP * 4, hipMemcpyHostToDevice);
    std::vector<double> ref(TM * HP), nxt(TM * HP);
    for (int i = 0; i < TM * HP; ++i) ref[i] = rows[i];
    for (int L = 0; L < LAYERS; ++L) {
        for (int r = 0; r < TM; ++r)
            for (int n = 0; n < HP; ++n) {
                double a = 0;
                for (int k = 0; k < HP; ++k) a += ref[r * HP + k] * (double)W[(size_t)k * HP + n];
                nxt[r * HP + n] = a > 0 ? a : 0;
            }
        ref.swap(nxt);
    }
    const size_t lds32 = (size_t)TM * SS * 4 + 3 * TM * 32 * 2 + 16, lds16 = lds32;
    hipFuncSetAttribute((const void*)k_probe<32, false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds32);
    hipFuncSetAttribute((const void*)k_probe<32, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds32);
    hipFuncSetAttribute((const void*)k_probe<16, false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds16);
    hipFuncSetAttribute((const void*)k_probe<16, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds16);
    hipFuncSetAttribute((const void*)k_probe<3, false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds32);
    hipFuncSetAttribute((const void*)k_probe<3, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds32);
    for (auto kf : {(const void*)k_probe<4, false>, (const void*)k_probe<4, true>, (const void*)k_probe<5, false>,
                    (const void*)k_probe<5, true>, (const void*)k_probe<6, false>, (const void*)k_probe<6, true>,
                    (const void*)k_probe<7, false>, (const void*)k_probe<7, true>})
        hipFuncSetAttribute(kf, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds32);
    for (auto kf : {(const void*)k_probe_w8<false>, (const void*)k_probe_w8<true>})
        hipFuncSetAttribute(kf, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)((size_t)TM8 * SS * 4 + (size_t)TM8 * 16 * 2 * 2 + 64));
    for (int round = 0; round < 2; ++round)
        for (int shape : {3, 8, 5}) {
            // FLOPs the matrix cores issue: 6 products (bf16 split) or 3 (fp16 split)
            const double flop = 2.0 * TM * HP * HP * LAYERS * blocks * (shape >= 3 && shape <= 8 ? 3 : 6);
            auto launch = [&](bool stamp) {
#define L_(S, T) hipLaunchKernelGGL((k_probe<S, T>), dim3(blocks), dim3(kBlock), lds32, 0, d_rows, d_Bs, d_out, d_st, d_Bh, d_colinv)
                if (shape == 32) {
                    if (stamp) L_(32, true); else L_(32, false);
                } else if (shape == 16) {
                    if (stamp) L_(16, true); else L_(16, false);
                } else if (shape == 3) {
                    if (stamp) L_(3, true); else L_(3, false);
                } else if (shape == 4) {
                    if (stamp) L_(4, true); else L_(4, false);
                } else if (shape == 6) {
                    if (stamp) L_(6, true); else L_(6, false);
                } else if (shape == 7) {
                    if (stamp) L_(7, true); else L_(7, false);
                } else if (shape == 8) {
                    const size_t l8 = (size_t)TM8 * SS * 4 + (size_t)TM8 * 16 * 2 * 2 + 64;
                    if (stamp) hipLaunchKernelGGL((k_probe_w8<true>), dim3(blocks / 2), dim3(512), l8, 0, d_rows, d_out, d_st, d_Bh, d_colinv);
                    else hipLaunchKernelGGL((k_probe_w8<false>), dim3(blocks / 2), dim3(512), l8, 0, d_rows, d_out, d_st, d_Bh, d_colinv);
                } else {
                    if (stamp) L_(5, true); else L_(5, false);
                }
#undef L_
            };
            const auto t0 = std::chrono::steady_clock::now();
            int warm = 0;
            while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < warm_s) {
                for (int i = 0; i < 100; ++i) launch(false);
                hipDeviceSynchronize();
                warm += 100;
            }
            hipEvent_t e0, e1;
            hipEventCreate(&e0);
            hipEventCreate(&e1);
            const int reps = 200;
            hipEventRecord(e0);
            for (int r = 0; r < reps; ++r) launch(false);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            const double us = 1e3 * ms / reps;
            // stamped launches right behind (still under load): clock of the last one
            for (int r = 0; r < 50; ++r) launch(true);
            hipDeviceSynchronize();
            std::vector<unsigned long long> st((size_t)blocks * 4);
            hipMemcpy(st.data(), d_st, st.size() * 8, hipMemcpyDeviceToHost);
            std::vector<double> clk, cyc;
            for (int b = 0; b < (shape == 8 ? blocks / 2 : blocks); ++b) {
                const double dt = (double)(st[b * 4 + 2] - st[b * 4 + 0]);
                const double dr = (double)(st[b * 4 + 3] - st[b * 4 + 1]);
                if (dr > 0) {
                    clk.push_back(dt / dr * 100.0);  // MHz (s_memrealtime: 100 MHz)
                    cyc.push_back(dt);
                }
            }
            std::sort(clk.begin(), clk.end());
            std::sort(cyc.begin(), cyc.end());
            std::vector<float> o(TM * HP);
            hipMemcpy(o.data(), d_out, o.size() * 4, hipMemcpyDeviceToHost);
            double maxe = 0, maxr = 0;
            for (int i = 0; i < TM * HP; ++i) {
                maxe = fmax(maxe, fabs(o[i] - ref[i]));
                maxr = fmax(maxr, fabs(ref[i]));
            }
            printf("{\"round\": %d, \"shape\": \"%s\", \"blocks\": %d, \"warm_launches\": %d, \"us\": %.2f, "
                   "\"bf16_TFs\": %.1f, \"frac_spec\": %.4f, \"clock_mhz_median\": %.0f, \"clock_mhz_p10\": %.0f, "
                   "\"clock_mhz_p90\": %.0f, \"wg_cycles_median\": %.0f, \"frac_at_held_clock\": %.4f, "
                   "\"err_rel\": %.3e, \"data\": %d}\n",
                   round, shape == 32 ? "32x32x16" : shape == 16 ? "16x16x32" : shape == 3 ? "f16x3_32x32x16" : shape == 4 ? "f16x3_32x32x16_k32stage" : shape == 6 ? "f16x3_32x32x16_dbstage_1barrier" : shape == 7 ? "f16x3_32x32x16_presplit_planes" : shape == 8 ? "f16x3_32x32x16_128rows_8waves" : "f16x3_16x16x32", blocks, warm, us, flop / us / 1e6,
                   flop / us / 1e6 / 2516.6, clk[clk.size() / 2], clk[clk.size() / 10], clk[clk.size() * 9 / 10],
                   cyc[cyc.size() / 2], flop / us / 1e6 / (2516.6 * clk[clk.size() / 2] / 2400.0), maxe / maxr, data);
            fflush(stdout);
        }
    return 0;
}
