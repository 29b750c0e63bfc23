// Calibration probe (design decision only): the row kernels' hidden x hidden layer GEMM (64 LDS
// rows x 256 x 256 per 256-thread workgroup, B streamed from an L2-resident packed image) on
//   (f32)  v_mfma_f32_32x32x2_f32 — the current kernels' exact f32 path, and
//   (x6)   v_mfma_f32_32x32x16_bf16 on a 3-way bf16 split of both operands (x = xh + xm + xl
//          exactly; the six products hh, hm, mh, mm, hl, lh), B pre-split in its packed image, A
//          split in registers after each LDS read.
// Each workgroup runs LAYERS layers back to back (relu rows written back to LDS between layers).
// Prints time, TFLOP/s of the algorithmic f32 FLOPs, and the error of workgroup 0's output
// against an fp64 host reference for both paths.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probe/split_gemm_probe.hip -o build/split_gemm_probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int HP = 256, TM = 64, SS = HP + 4, NT = HP / 32, LAYERS = 8;
constexpr int kBlock = 256;

__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

// ---- f32 path (the current gemm_cols<8, 2>) ----
__device__ __forceinline__ void gemm_f32(const float* A, const float* Bp, f32x16 (&acc)[2][2]) {
    constexpr int nq = HP / 8;
    const int lane = threadIdx.x & 63, wv = wave_id(), h = lane >> 5, l32 = lane & 31;
    for (int rt = 0; rt < 2; ++rt)
        for (int j = 0; j < 2; ++j)
            for (int i = 0; i < 16; ++i) acc[rt][j][i] = 0.f;
    const float4* B0 = reinterpret_cast<const float4*>(Bp) + (size_t)h * HP + wv * 32 + l32;
    const float4* B1 = reinterpret_cast<const float4*>(Bp) + (size_t)h * HP + (wv + 4) * 32 + l32;
    constexpr size_t STEP = 2 * (size_t)HP;
    float4 p0 = B0[0], p1 = B0[STEP], r0 = B1[0], r1 = B1[STEP];
    const float* arow = A + l32 * SS + 4 * h;
    float4 a[2], an[2];
    for (int rt = 0; rt < 2; ++rt) a[rt] = *reinterpret_cast<const float4*>(arow + rt * 32 * SS);
#pragma unroll
    for (int q = 0; q < nq; ++q) {
        const float4 c0 = p0, c1 = r0;
        p0 = p1;
        r0 = r1;
        if (q + 2 < nq) {
            p1 = B0[(q + 2) * STEP];
            r1 = B1[(q + 2) * STEP];
        }
        if (q + 1 < nq)
            for (int rt = 0; rt < 2; ++rt)
                an[rt] = *reinterpret_cast<const float4*>(arow + rt * 32 * SS + 8 * (q + 1));
        __builtin_amdgcn_sched_barrier(0);
#define MF(S)                                                                                     \
    for (int rt = 0; rt < 2; ++rt) {                                                              \
        acc[rt][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[rt].S, c0.S, acc[rt][0], 0, 0, 0);    \
        acc[rt][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[rt].S, c1.S, acc[rt][1], 0, 0, 0);    \
    }
        MF(x) MF(y) MF(z) MF(w)
#undef MF
        __builtin_amdgcn_sched_barrier(0);
        for (int rt = 0; rt < 2; ++rt) a[rt] = an[rt];
    }
}

// ---- split path ----
struct Split3 {
    bf16x8 h, m, l;
};
__device__ __forceinline__ Split3 split8(float4 x0, float4 x1) {
    const float v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
    Split3 s;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const __bf16 hb = (__bf16)v[j];
        const float r = v[j] - (float)hb;
        const __bf16 mb = (__bf16)r;
        const float r2 = r - (float)mb;
        s.h[j] = hb;
        s.m[j] = mb;
        s.l[j] = (__bf16)r2;
    }
    return s;
}
__device__ __forceinline__ f32x16 mf16(bf16x8 a, bf16x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x16 mfma_x6b(const Split3& a, const bf16x8 (&b)[3], f32x16 c) {
    c = mf16(a.m, b[1], c);
    c = mf16(a.l, b[0], c);
    c = mf16(a.h, b[2], c);
    c = mf16(a.m, b[0], c);
    c = mf16(a.h, b[1], c);
    return mf16(a.h, b[0], c);
}
// B image: [plane 3][q = K/16][h 2][col HP] x 8 bf16 (16 B): lane (h, l32) of tile t reads entry
// (plane, q, h, t*32 + l32) = B[k = 16q + 8h + j][col], j = 0..7
template <bool SPLIT = true, bool BLOAD = true>
__device__ __forceinline__ void gemm_x6(const float* A, const bf16x8* Bs, f32x16 (&acc)[2][2]) {
    constexpr int nq = HP / 16;
    constexpr size_t PL = (size_t)nq * 2 * HP;  // entries per plane
    const int lane = threadIdx.x & 63, wv = wave_id(), h = lane >> 5, l32 = lane & 31;
    for (int rt = 0; rt < 2; ++rt)
        for (int j = 0; j < 2; ++j)
            for (int i = 0; i < 16; ++i) acc[rt][j][i] = 0.f;
    const bf16x8* B0 = Bs + (size_t)h * HP + wv * 32 + l32;
    const bf16x8* B1 = Bs + (size_t)h * HP + (wv + 4) * 32 + l32;
    constexpr size_t STEP = 2 * (size_t)HP;
    bf16x8 b0[3], b1[3], nb0[3], nb1[3];
    for (int p = 0; p < 3; ++p) {
        b0[p] = B0[p * PL];
        b1[p] = B1[p * PL];
    }
    const float* arow = A + l32 * SS + 8 * h;
    float4 a[2][2], an[2][2];
    for (int rt = 0; rt < 2; ++rt) {
        a[rt][0] = *reinterpret_cast<const float4*>(arow + rt * 32 * SS);
        a[rt][1] = *reinterpret_cast<const float4*>(arow + rt * 32 * SS + 4);
    }
#pragma unroll
    for (int q = 0; q < nq; ++q) {
        if (q + 1 < nq) {
            for (int p = 0; p < 3; ++p) {
                nb0[p] = BLOAD ? B0[p * PL + (q + 1) * STEP] : b0[(p + 1) % 3];
                nb1[p] = BLOAD ? B1[p * PL + (q + 1) * STEP] : b1[(p + 1) % 3];
            }
            for (int rt = 0; rt < 2; ++rt) {
                an[rt][0] = *reinterpret_cast<const float4*>(arow + rt * 32 * SS + 16 * (q + 1));
                an[rt][1] = *reinterpret_cast<const float4*>(arow + rt * 32 * SS + 16 * (q + 1) + 4);
            }
        }
#pragma unroll
        for (int rt = 0; rt < 2; ++rt) {
            Split3 s;
            if (SPLIT) {
                s = split8(a[rt][0], a[rt][1]);
            } else {
                s.h = __builtin_bit_cast(bf16x8, a[rt][0]);
                s.m = __builtin_bit_cast(bf16x8, a[rt][1]);
                s.l = s.h;
            }
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const bf16x8* b = j == 0 ? b0 : b1;
                f32x16 c = acc[rt][j];
                // small terms first
                c = mf16(s.m, b[1], c);
                c = mf16(s.l, b[0], c);
                c = mf16(s.h, b[2], c);
                c = mf16(s.m, b[0], c);
                c = mf16(s.h, b[1], c);
                c = mf16(s.h, b[0], c);
                acc[rt][j] = c;
            }
        }
        if (q + 1 < nq) {
            for (int p = 0; p < 3; ++p) {
                b0[p] = nb0[p];
                b1[p] = nb1[p];
            }
            for (int rt = 0; rt < 2; ++rt) {
                a[rt][0] = an[rt][0];
                a[rt][1] = an[rt][1];
            }
        }
    }
}

// x6 with the split of step q+1 software-pipelined under step q's MFMAs (sched_group_barrier
// pattern: 1 MFMA, then up to 4 VALU)
__device__ __forceinline__ void gemm_x6i(const float* A, const bf16x8* Bs, f32x16 (&acc)[2][2]) {
    constexpr int nq = HP / 16;
    constexpr size_t PL = (size_t)nq * 2 * HP;
    const int lane = threadIdx.x & 63, wv = wave_id(), h = lane >> 5, l32 = lane & 31;
    for (int rt = 0; rt < 2; ++rt)
        for (int j = 0; j < 2; ++j)
            for (int i = 0; i < 16; ++i) acc[rt][j][i] = 0.f;
    const bf16x8* B0 = Bs + (size_t)h * HP + wv * 32 + l32;
    const bf16x8* B1 = Bs + (size_t)h * HP + (wv + 4) * 32 + l32;
    constexpr size_t STEP = 2 * (size_t)HP;
    bf16x8 b0[3], b1[3], nb0[3], nb1[3];
    for (int p = 0; p < 3; ++p) {
        b0[p] = B0[p * PL];
        b1[p] = B1[p * PL];
    }
    const float* arow = A + l32 * SS + 8 * h;
    Split3 s[2], sn[2];
    for (int rt = 0; rt < 2; ++rt)
        s[rt] = split8(*reinterpret_cast<const float4*>(arow + rt * 32 * SS),
                       *reinterpret_cast<const float4*>(arow + rt * 32 * SS + 4));
#pragma unroll
    for (int q = 0; q < nq; ++q) {
        float4 an[2][2];
        if (q + 1 < nq) {
            for (int p = 0; p < 3; ++p) {
                nb0[p] = B0[p * PL + (q + 1) * STEP];
                nb1[p] = B1[p * PL + (q + 1) * STEP];
            }
            for (int rt = 0; rt < 2; ++rt) {
                an[rt][0] = *reinterpret_cast<const float4*>(arow + rt * 32 * SS + 16 * (q + 1));
                an[rt][1] = *reinterpret_cast<const float4*>(arow + rt * 32 * SS + 16 * (q + 1) + 4);
            }
        }
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const bf16x8* b = j == 0 ? b0 : b1;
                f32x16 c = acc[rt][j];
                c = mf16(s[rt].m, b[1], c);
                c = mf16(s[rt].l, b[0], c);
                c = mf16(s[rt].h, b[2], c);
                c = mf16(s[rt].m, b[0], c);
                c = mf16(s[rt].h, b[1], c);
                c = mf16(s[rt].h, b[0], c);
                acc[rt][j] = c;
            }
        if (q + 1 < nq) {
            for (int rt = 0; rt < 2; ++rt) sn[rt] = split8(an[rt][0], an[rt][1]);
#pragma unroll
            for (int k = 0; k < 24; ++k) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);
            }
            for (int p = 0; p < 3; ++p) {
                b0[p] = nb0[p];
                b1[p] = nb1[p];
            }
            for (int rt = 0; rt < 2; ++rt) s[rt] = sn[rt];
        }
    }
}

// x6 with explicit scheduling: the next step's loads fenced at the top of the step, then the
// MFMAs of this step interleaved (IL) with the split of the next step, or all MFMAs then the split
template <bool IL>
__device__ __forceinline__ void gemm_x6f(const float* A, const bf16x8* Bs, f32x16 (&acc)[2][2]) {
    constexpr int nq = HP / 16;
    constexpr size_t PL = (size_t)nq * 2 * HP;
    const int lane = threadIdx.x & 63, wv = wave_id(), h = lane >> 5, l32 = lane & 31;
    for (int rt = 0; rt < 2; ++rt)
        for (int j = 0; j < 2; ++j)
            for (int i = 0; i < 16; ++i) acc[rt][j][i] = 0.f;
    const bf16x8* B0 = Bs + (size_t)h * HP + wv * 32 + l32;
    const bf16x8* B1 = Bs + (size_t)h * HP + (wv + 4) * 32 + l32;
    constexpr size_t STEP = 2 * (size_t)HP;
    bf16x8 b0[3], b1[3];
    for (int p = 0; p < 3; ++p) {
        b0[p] = B0[p * PL];
        b1[p] = B1[p * PL];
    }
    const float* arow = A + l32 * SS + 8 * h;
    Split3 s[2];
    for (int rt = 0; rt < 2; ++rt)
        s[rt] = split8(*reinterpret_cast<const float4*>(arow + rt * 32 * SS),
                       *reinterpret_cast<const float4*>(arow + rt * 32 * SS + 4));
#pragma unroll
    for (int q = 0; q < nq; ++q) {
        bf16x8 nb0[3], nb1[3];
        float4 an[2][2];
        const int qn = q + 1 < nq ? q + 1 : q;
        for (int p = 0; p < 3; ++p) {
            nb0[p] = B0[p * PL + qn * STEP];
            nb1[p] = B1[p * PL + qn * STEP];
        }
        for (int rt = 0; rt < 2; ++rt) {
            an[rt][0] = *reinterpret_cast<const float4*>(arow + rt * 32 * SS + 16 * qn);
            an[rt][1] = *reinterpret_cast<const float4*>(arow + rt * 32 * SS + 16 * qn + 4);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[rt][j] = mfma_x6b(s[rt], j == 0 ? b0 : b1, acc[rt][j]);
        Split3 sn[2];
        for (int rt = 0; rt < 2; ++rt) sn[rt] = split8(an[rt][0], an[rt][1]);
        if (IL) {
#pragma unroll
            for (int k = 0; k < 22; ++k) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);
            }
            __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
        for (int rt = 0; rt < 2; ++rt) s[rt] = sn[rt];
        for (int p = 0; p < 3; ++p) {
            b0[p] = nb0[p];
            b1[p] = nb1[p];
        }
    }
}

// 128 rows per workgroup (one per CU), each wave 4 row tiles x 2 column tiles: half the B loads
// per MFMA of the 64-row form, the same A split per MFMA
constexpr int TM4 = 128;
__device__ __forceinline__ void gemm_x6_rt4(const float* A, const bf16x8* Bs, f32x16 (&acc)[4][2]) {
    constexpr int nq = HP / 16;
    constexpr size_t PL = (size_t)nq * 2 * HP;
    const int lane = threadIdx.x & 63, wv = wave_id(), h = lane >> 5, l32 = lane & 31;
    for (int rt = 0; rt < 4; ++rt)
        for (int j = 0; j < 2; ++j)
            for (int i = 0; i < 16; ++i) acc[rt][j][i] = 0.f;
    const bf16x8* B0 = Bs + (size_t)h * HP + wv * 32 + l32;
    const bf16x8* B1 = Bs + (size_t)h * HP + (wv + 4) * 32 + l32;
    constexpr size_t STEP = 2 * (size_t)HP;
    bf16x8 b0[3], b1[3], nb0[3], nb1[3];
    for (int p = 0; p < 3; ++p) {
        b0[p] = B0[p * PL];
        b1[p] = B1[p * PL];
    }
    const float* arow = A + l32 * SS + 8 * h;
    float4 a[4][2], an[4][2];
    for (int rt = 0; rt < 4; ++rt) {
        a[rt][0] = *reinterpret_cast<const float4*>(arow + rt * 32 * SS);
        a[rt][1] = *reinterpret_cast<const float4*>(arow + rt * 32 * SS + 4);
    }
#pragma unroll
    for (int q = 0; q < nq; ++q) {
        if (q + 1 < nq) {
            for (int p = 0; p < 3; ++p) {
                nb0[p] = B0[p * PL + (q + 1) * STEP];
                nb1[p] = B1[p * PL + (q + 1) * STEP];
            }
            for (int rt = 0; rt < 4; ++rt) {
                an[rt][0] = *reinterpret_cast<const float4*>(arow + rt * 32 * SS + 16 * (q + 1));
                an[rt][1] = *reinterpret_cast<const float4*>(arow + rt * 32 * SS + 16 * (q + 1) + 4);
            }
        }
#pragma unroll
        for (int rt = 0; rt < 4; ++rt) {
            const Split3 sp = split8(a[rt][0], a[rt][1]);
            acc[rt][0] = mfma_x6b(sp, b0, acc[rt][0]);
            acc[rt][1] = mfma_x6b(sp, b1, acc[rt][1]);
        }
        if (q + 1 < nq) {
            for (int p = 0; p < 3; ++p) {
                b0[p] = nb0[p];
                b1[p] = nb1[p];
            }
            for (int rt = 0; rt < 4; ++rt) {
                a[rt][0] = an[rt][0];
                a[rt][1] = an[rt][1];
            }
        }
    }
}

__global__ __launch_bounds__(256, 1) void k_probe_rt4(const float* rows, const bf16x8* Bs,
                                                      float* out) {
    extern __shared__ float act[];
    const int tid = threadIdx.x;
    const float* src = rows + (size_t)(blockIdx.x & 3) * TM4 * HP;
    for (int i = tid; i < TM4 * HP; i += kBlock) act[(i / HP) * SS + i % HP] = src[i];
    __syncthreads();
    f32x16 acc[4][2];
    const int lane = threadIdx.x & 63, wv = wave_id(), h = lane >> 5, l32 = lane & 31;
    for (int L = 0; L < LAYERS; ++L) {
        gemm_x6_rt4(act, Bs, acc);
        __syncthreads();
        for (int j = 0; j < 2; ++j) {
            const int t = j == 0 ? wv : wv + 4;
            float* col = act + t * 32 + l32 + 4 * h * SS;
            for (int rt = 0; rt < 4; ++rt)
                for (int i = 0; i < 16; ++i)
                    col[(rt * 32 + (i & 3) + 8 * (i >> 2)) * SS] = fmaxf(acc[rt][j][i], 0.f);
        }
        __syncthreads();
    }
    if (blockIdx.x < 4)
        for (int i = tid; i < TM4 * HP; i += kBlock)
            out[(size_t)blockIdx.x * TM4 * HP + i] = act[(i / HP) * SS + i % HP];
}

// cooperative split: per k step the workgroup's 256 threads split the step's 64 x 16 A values
// once (4 per thread) into an LDS stage of three bf16 planes (row stride 24 bf16: conflict-free
// 16-B reads), then every wave reads its fragments from the stage (2 barriers per step)
constexpr int STG = 24;
__device__ __forceinline__ void gemm_x6_coop(const float* A, __bf16* stage, const bf16x8* Bs,
                                             f32x16 (&acc)[2][2]) {
    constexpr int nq = HP / 16;
    constexpr size_t PL = (size_t)nq * 2 * HP;
    const int tid = threadIdx.x, lane = tid & 63, wv = wave_id(), h = lane >> 5, l32 = lane & 31;
    for (int rt = 0; rt < 2; ++rt)
        for (int j = 0; j < 2; ++j)
            for (int i = 0; i < 16; ++i) acc[rt][j][i] = 0.f;
    const bf16x8* B0 = Bs + (size_t)h * HP + wv * 32 + l32;
    const bf16x8* B1 = Bs + (size_t)h * HP + (wv + 4) * 32 + l32;
    constexpr size_t STEP = 2 * (size_t)HP;
    bf16x8 b0[3], b1[3], nb0[3], nb1[3];
    for (int p = 0; p < 3; ++p) {
        b0[p] = B0[p * PL];
        b1[p] = B1[p * PL];
    }
    const int sr = tid >> 2, sk = (tid & 3) * 4;  // this thread's 4 values of a step
    const float* src = A + sr * SS + sk;
    constexpr int PP = TM * STG;  // bf16 per plane
    float4 x = *reinterpret_cast<const float4*>(src);
#pragma unroll
    for (int q = 0; q < nq; ++q) {
        // split this thread's 4 values of step q into the stage
        {
            const float v[4] = {x.x, x.y, x.z, x.w};
            typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
            bf16x4 ph, pm, pl;
            for (int j = 0; j < 4; ++j) {
                const __bf16 hb = (__bf16)v[j];
                const float r = v[j] - (float)hb;
                const __bf16 mb = (__bf16)r;
                ph[j] = hb;
                pm[j] = mb;
                pl[j] = (__bf16)(r - (float)mb);
            }
            __bf16* d = stage + sr * STG + sk;
            *reinterpret_cast<bf16x4*>(d) = ph;
            *reinterpret_cast<bf16x4*>(d + PP) = pm;
            *reinterpret_cast<bf16x4*>(d + 2 * PP) = pl;
        }
        if (q + 1 < nq) {
            x = *reinterpret_cast<const float4*>(src + 16 * (q + 1));
            for (int p = 0; p < 3; ++p) {
                nb0[p] = B0[p * PL + (q + 1) * STEP];
                nb1[p] = B1[p * PL + (q + 1) * STEP];
            }
        }
        __syncthreads();
        Split3 sa[2];
        for (int rt = 0; rt < 2; ++rt) {
            const __bf16* f = stage + (rt * 32 + l32) * STG + 8 * h;
            sa[rt].h = *reinterpret_cast<const bf16x8*>(f);
            sa[rt].m = *reinterpret_cast<const bf16x8*>(f + PP);
            sa[rt].l = *reinterpret_cast<const bf16x8*>(f + 2 * PP);
        }
        __syncthreads();
#pragma unroll
        for (int rt = 0; rt < 2; ++rt) {
            acc[rt][0] = mfma_x6b(sa[rt], b0, acc[rt][0]);
            acc[rt][1] = mfma_x6b(sa[rt], b1, acc[rt][1]);
        }
        if (q + 1 < nq)
            for (int p = 0; p < 3; ++p) {
                b0[p] = nb0[p];
                b1[p] = nb1[p];
            }
    }
}

// A pre-split in LDS: planes [3][TM][HP + 8] bf16, written once per layer; 8 waves, wave w owns
// column tile w of both row tiles
constexpr int PS = HP + 8;  // plane row stride (bf16)
__device__ __forceinline__ void gemm_pl(const __bf16* P, const bf16x8* Bs, f32x16 (&acc)[2]) {
    constexpr int nq = HP / 16;
    constexpr size_t PL = (size_t)nq * 2 * HP;
    const int lane = threadIdx.x & 63, wv = wave_id(), h = lane >> 5, l32 = lane & 31;
    for (int rt = 0; rt < 2; ++rt)
        for (int i = 0; i < 16; ++i) acc[rt][i] = 0.f;
    const bf16x8* B0 = Bs + (size_t)h * HP + wv * 32 + l32;
    constexpr size_t STEP = 2 * (size_t)HP;
    bf16x8 b0[3], nb0[3];
    for (int p = 0; p < 3; ++p) b0[p] = B0[p * PL];
    const __bf16* arow = P + l32 * PS + 8 * h;
    constexpr size_t PP = (size_t)TM * PS;
    bf16x8 a[2][3], an[2][3];
    for (int rt = 0; rt < 2; ++rt)
        for (int p = 0; p < 3; ++p)
            a[rt][p] = *reinterpret_cast<const bf16x8*>(arow + p * PP + rt * 32 * PS);
#pragma unroll
    for (int q = 0; q < nq; ++q) {
        if (q + 1 < nq) {
            for (int p = 0; p < 3; ++p) nb0[p] = B0[p * PL + (q + 1) * STEP];
            for (int rt = 0; rt < 2; ++rt)
                for (int p = 0; p < 3; ++p)
                    an[rt][p] = *reinterpret_cast<const bf16x8*>(arow + p * PP + rt * 32 * PS +
                                                                 16 * (q + 1));
        }
#pragma unroll
        for (int rt = 0; rt < 2; ++rt) {
            f32x16 c = acc[rt];
            c = mf16(a[rt][1], b0[1], c);
            c = mf16(a[rt][2], b0[0], c);
            c = mf16(a[rt][0], b0[2], c);
            c = mf16(a[rt][1], b0[0], c);
            c = mf16(a[rt][0], b0[1], c);
            c = mf16(a[rt][0], b0[0], c);
            acc[rt] = c;
        }
        if (q + 1 < nq) {
            for (int p = 0; p < 3; ++p) b0[p] = nb0[p];
            for (int rt = 0; rt < 2; ++rt)
                for (int p = 0; p < 3; ++p) a[rt][p] = an[rt][p];
        }
    }
}

__device__ __forceinline__ void store_planes(const f32x16 (&acc)[2], __bf16* P) {
    const int lane = threadIdx.x & 63, wv = wave_id(), h = lane >> 5, l32 = lane & 31;
    constexpr size_t PP = (size_t)TM * PS;
    __bf16* col = P + wv * 32 + l32 + 4 * h * PS;
    for (int rt = 0; rt < 2; ++rt)
        for (int i = 0; i < 16; ++i) {
            const float x = fmaxf(acc[rt][i], 0.f);
            const __bf16 hb = (__bf16)x;
            const float r = x - (float)hb;
            const __bf16 mb = (__bf16)r;
            const int o = (rt * 32 + (i & 3) + 8 * (i >> 2)) * PS;
            col[o] = hb;
            col[PP + o] = mb;
            col[2 * PP + o] = (__bf16)(r - (float)mb);
        }
}

__global__ __launch_bounds__(512, 1) void k_probe_pl(const float* rows, const bf16x8* Bs,
                                                     float* out) {
    extern __shared__ __bf16 pl[];
    const int tid = threadIdx.x;
    constexpr size_t PP = (size_t)TM * PS;
    const float* src = rows + (size_t)(blockIdx.x & 7) * TM * HP;
    for (int i = tid; i < TM * HP; i += 512) {
        const float x = src[i];
        const __bf16 hb = (__bf16)x;
        const float r = x - (float)hb;
        const __bf16 mb = (__bf16)r;
        const int o = (i / HP) * PS + i % HP;
        pl[o] = hb;
        pl[PP + o] = mb;
        pl[2 * PP + o] = (__bf16)(r - (float)mb);
    }
    __syncthreads();
    f32x16 acc[2];
    for (int L = 0; L < LAYERS; ++L) {
        gemm_pl(pl, Bs, acc);
        __syncthreads();
        store_planes(acc, pl);
        __syncthreads();
    }
    if (blockIdx.x < 8)
        for (int i = tid; i < TM * HP; i += 512) {
            const int o = (i / HP) * PS + i % HP;
            out[(size_t)blockIdx.x * TM * HP + i] =
                ((float)pl[o] + (float)pl[PP + o]) + (float)pl[2 * PP + o];
        }
}

__device__ __forceinline__ void store_rows(const f32x16 (&acc)[2][2], float* act) {
    const int lane = threadIdx.x & 63, wv = wave_id(), h = lane >> 5, l32 = lane & 31;
    for (int j = 0; j < 2; ++j) {
        const int t = j == 0 ? wv : wv + 4;
        float* col = act + t * 32 + l32 + 4 * h * SS;
        for (int rt = 0; rt < 2; ++rt)
            for (int i = 0; i < 16; ++i)
                col[(rt * 32 + (i & 3) + 8 * (i >> 2)) * SS] = fmaxf(acc[rt][j][i], 0.f);
    }
}

template <int MODE>
__global__ __launch_bounds__(kBlock, 1) void k_probe(const float* rows, const float* Bf,
                                                     const bf16x8* Bs, float* out) {
    extern __shared__ float act[];
    const int tid = threadIdx.x;
    const float* src = rows + (size_t)(blockIdx.x & 7) * TM * HP;
    for (int i = tid; i < TM * HP; i += kBlock) act[(i / HP) * SS + i % HP] = src[i];
    __syncthreads();
    f32x16 acc[2][2];
    for (int L = 0; L < LAYERS; ++L) {
        if (MODE == 0)
            gemm_f32(act, Bf, acc);
        else if (MODE == 1)
            gemm_x6(act, Bs, acc);
        else if (MODE == 2)
            gemm_x6i(act, Bs, acc);
        else if (MODE == 4)
            gemm_x6<false, true>(act, Bs, acc);
        else if (MODE == 5)
            gemm_x6<true, false>(act, Bs, acc);
        else if (MODE == 10)
            gemm_x6_coop(act, reinterpret_cast<__bf16*>(act + TM * SS), Bs, acc);
        else if (MODE == 7)
            gemm_x6f<false>(act, Bs, acc);
        else if (MODE == 8)
            gemm_x6f<true>(act, Bs, acc);
        else
            gemm_x6<false, false>(act, Bs, acc);
        __syncthreads();
        store_rows(acc, act);
        __syncthreads();
    }
    if (blockIdx.x < 8)
        for (int i = tid; i < TM * HP; i += kBlock)
            out[(size_t)blockIdx.x * TM * HP + i] = act[(i / HP) * SS + i % HP];
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

int main() {
    const int blocks = 1024;
    std::vector<float> rows(8 * TM * HP), W(HP * HP);  // W[k][n]
    unsigned s = 12345;
    auto rnd = [&]() {
        s = s * 1664525u + 1013904223u;
        return ((s >> 8) & 0xffff) / 65536.0f * 2.f - 1.f;
    };
    for (auto& v : rows) v = rnd();
    const float bound = sqrtf(6.f / HP);
    for (auto& v : W) v = rnd() * bound;
    // f32 packed image [K/4][HP][4]
    std::vector<float> Bf((size_t)HP * HP);
    for (int k = 0; k < HP; ++k)
        for (int n = 0; n < HP; ++n) Bf[((size_t)(k >> 2) * HP + n) * 4 + (k & 3)] = W[(size_t)k * HP + n];
    // gemm_f32 reads lane half h at k = 8q + 4h + s: its image has (k>>2) = 2q + h, so entry
    // ((2q + h) * HP + n) * 4 + s — the layout above with the h offset folded in the pointer
    // split image [3][K/16][2][HP][8]
    const int nq = HP / 16;
    std::vector<uint16_t> Bs((size_t)3 * nq * 2 * HP * 8);
    for (int k = 0; k < HP; ++k)
        for (int n = 0; n < HP; ++n) {
            const float x = W[(size_t)k * HP + n];
            const uint16_t hb = bf16_rn(x);
            const float r = x - bf16_f(hb);
            const uint16_t mb = bf16_rn(r);
            const uint16_t lb = bf16_rn(r - bf16_f(mb));
            const int q = k / 16, h = (k % 16) / 8, j = k % 8;
            for (int p = 0; p < 3; ++p)
                Bs[((((size_t)p * nq + q) * 2 + h) * HP + n) * 8 + j] = p == 0 ? hb : p == 1 ? mb : lb;
        }
    float *d_rows, *d_Bf, *d_out;
    bf16x8* d_Bs;
    hipMalloc(&d_rows, rows.size() * 4);
    hipMalloc(&d_Bf, Bf.size() * 4);
    hipMalloc(&d_Bs, Bs.size() * 2);
    hipMalloc(&d_out, (size_t)8 * TM * HP * 4);
    hipMemcpy(d_rows, rows.data(), rows.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(d_Bf, Bf.data(), Bf.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(d_Bs, Bs.data(), Bs.size() * 2, hipMemcpyHostToDevice);
    const size_t lds = (size_t)TM * SS * 4 + (size_t)3 * TM * STG * 2;
    // fp64 reference of workgroup 0
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
    for (int mode = 0; mode < 11; ++mode) {
        auto k = mode == 0 ? k_probe<0> : mode == 1 ? k_probe<1> : mode == 2 ? k_probe<2> : mode == 4 ? k_probe<4> : mode == 5 ? k_probe<5> : mode == 6 ? k_probe<6> : mode == 7 ? k_probe<7> : k_probe<8>;
        if (mode == 9) k = k_probe<1>;
        if (mode == 10) k = k_probe<10>;
        const size_t lds_pl = (size_t)3 * TM * PS * 2;
        auto launch = [&]() {
            if (mode == 9)
                hipLaunchKernelGGL(k_probe_rt4, dim3(blocks / 2), dim3(kBlock), (size_t)TM4 * SS * 4, 0, d_rows, d_Bs, d_out);
            else if (mode != 3)
                hipLaunchKernelGGL(k, dim3(blocks), dim3(kBlock), lds, 0, d_rows, d_Bf, d_Bs, d_out);
            else
                hipLaunchKernelGGL(k_probe_pl, dim3(blocks), dim3(512), lds_pl, 0, d_rows, d_Bs, d_out);
        };
        hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipFuncSetAttribute((const void*)k_probe_pl, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_pl);
        hipFuncSetAttribute((const void*)k_probe_rt4, hipFuncAttributeMaxDynamicSharedMemorySize, (int)((size_t)TM4 * SS * 4));
        launch();
        hipDeviceSynchronize();
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        const int reps = 10;
        hipEventRecord(e0);
        for (int r = 0; r < reps; ++r) launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        const double us = 1e3 * ms / reps;
        const double flop = 2.0 * TM * HP * HP * LAYERS * blocks;
        std::vector<float> o(TM * HP);
        hipMemcpy(o.data(), d_out, o.size() * 4, hipMemcpyDeviceToHost);
        double maxe = 0, maxr = 0, sum2 = 0, ref2 = 0;
        for (int i = 0; i < TM * HP; ++i) {
            const double e = fabs(o[i] - ref[i]);
            maxe = fmax(maxe, e);
            maxr = fmax(maxr, fabs(ref[i]));
            sum2 += e * e;
            ref2 += ref[i] * ref[i];
        }
        printf("{\"mode\": \"%s\", \"us\": %.1f, \"TFs\": %.1f, \"max_abs_err\": %.3e, "
               "\"max_ref\": %.3e, \"rel_rms_err\": %.3e}\n",
               mode == 0 ? "f32" : mode == 1 ? "bf16x6" : mode == 2 ? "bf16x6_interleaved" : mode == 3 ? "bf16x6_lds_planes_8w" : mode == 4 ? "x6_nosplit" : mode == 5 ? "x6_noBload" : mode == 6 ? "x6_nosplit_noBload" : mode == 7 ? "x6_fenced" : mode == 8 ? "x6_fenced_interleaved" : mode == 9 ? "x6_rt4_128rows_1wg" : "x6_coop_split_stage", us, flop / us / 1e6, maxe, maxr, sqrt(sum2 / ref2));
    }
    return 0;
}
