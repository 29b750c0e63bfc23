// mlp_common.h — the device MLP layout (include/navenv.h nav_mlp) and the fragment helpers
// shared by the row kernels (mlp_kernels.hip) and the learner kernels (learner_kernels.hip).
#pragma once
#include <stdlib.h>

#include "nav_device.h"

using namespace nav;

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kMaxLayers = 9;
// workgroups hold RT row tiles of 32 rows (RT = 2; RT = 1 for small batches, row_tiles_for)

struct MlpDev {
    const float* params;
    const float* packed;
    int d_in, d_out, hp, n_hidden;
    int64_t count;
    int64_t w_off[kMaxLayers], b_off[kMaxLayers];
};

inline int64_t r4(int64_t x) { return (x + 3) & ~(int64_t)3; }

bool make_dev(const nav_mlp* n, MlpDev* d) {
    if (!n || n->d_in < 1 || n->d_in > 4 || n->d_out < 1 || n->d_out > 2 || n->hidden_pad < 32 ||
        n->hidden_pad > 256 || (n->hidden_pad & 31) || n->n_hidden < 1 ||
        n->n_hidden >= kMaxLayers || !n->params || (n->n_hidden > 1 && !n->packed) ||
        n->hidden < 1 || n->hidden > n->hidden_pad)
        return false;
    const int hp = n->hidden_pad;
    d->params = n->params;
    d->packed = n->packed;
    d->d_in = n->d_in;
    d->d_out = n->d_out;
    d->hp = hp;
    d->n_hidden = n->n_hidden;
    int64_t o = 0;
    for (int l = 0; l <= n->n_hidden; ++l) {
        const int64_t in = l == 0 ? n->d_in : hp, out = l == n->n_hidden ? n->d_out : hp;
        d->w_off[l] = o;
        o += r4(in * out);
        d->b_off[l] = o;
        o += r4(out);
    }
    d->count = o;
    return true;
}

// Edge-gradient layout: every parameter except the hidden x hidden weights W_1 .. W_{nh-1}, in
// the flat order with those segments cut out (W0 | b0 | b1 .. b_{nh-1} | Wo | bo). The forward /
// backward kernels sum these per row block while the operands sit in LDS (edge slabs
// [blocks][edge_count]); nav_grad_reduce folds them and the weight-gradient slabs into the flat
// gradient.
__host__ __device__ inline int64_t hidden_w_count(const MlpDev& d) {
    return (int64_t)(d.n_hidden - 1) * d.hp * d.hp;
}
__host__ __device__ inline int64_t edge_count(const MlpDev& d) { return d.count - hidden_w_count(d); }
// edge index of b_L (L < n_hidden), of Wo and of bo
__host__ __device__ inline int64_t e_b(const MlpDev& d, int L) {
    return d.b_off[L] - (int64_t)L * d.hp * d.hp;
}
__host__ __device__ inline int64_t e_wo(const MlpDev& d) { return d.w_off[d.n_hidden] - hidden_w_count(d); }
__host__ __device__ inline int64_t e_bo(const MlpDev& d) { return d.b_off[d.n_hidden] - hidden_w_count(d); }
// flat parameter index of edge index e
__host__ __device__ inline int64_t edge_to_flat(const MlpDev& d, int64_t e) {
    const int nh = d.n_hidden;
    if (nh == 1 || e < d.w_off[1]) return e;
    if (e >= e_wo(d)) return e + hidden_w_count(d);
    const int64_t L = (e - d.w_off[1]) / d.hp + 1;  // inside the b_L run
    return e + L * d.hp * d.hp;
}

inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

// ReLU as an integer max of the bit pattern: one v_max_i32 (fmaxf costs a NaN-quieting
// v_max_f32 x, x first). Negative values and -0 give +0; finite results equal fmaxf(v, 0).
NAV_DEV float relu(float v) { return __int_as_float(max(__float_as_int(v), 0)); }

// On post-ReLU values (v >= +0, so the bit patterns order like the values): the ReLU bit as
// min(bits, 1) (every positive float's pattern is >= 1; +0's is 0) and the running max as an
// integer max (fmaxf quiets both operands first), one VALU each
#ifndef NAV_NNBITS
#define NAV_NNBITS 1
#endif
NAV_DEV uint32_t pos_bit(float v) {
    return NAV_NNBITS ? min((uint32_t)__float_as_int(v), 1u) : (v > 0.f ? 1u : 0u);
}
NAV_DEV float max_nn(float m, float v) {
    return NAV_NNBITS ? __int_as_float(max(__float_as_int(m), __float_as_int(v))) : fmaxf(m, v);
}

// One hidden unit of layer 0 (K = d_in <= 4; absent inputs and weights are 0). The forward and the
// weight-gradient kernel's recompute of h_0 share this fma order, so both produce the same bits.
NAV_DEV float layer0_unit(float4 x, float w0, float w1, float w2, float w3, float b) {
    float v = b;
    v = fmaf(x.x, w0, v);
    v = fmaf(x.y, w1, v);
    v = fmaf(x.z, w2, v);
    v = fmaf(x.w, w3, v);
    return relu(v);
}

// dL/dz of the top hidden layer before its ReLU mask: dy . Wo[:, n] (d_out <= 2; absent = 0).
// Shared by the backward and the weight-gradient recompute of dz_{nh-1}.
NAV_DEV float top_unit(float g0, float g1, float w0, float w1) { return fmaf(g1, w1, g0 * w0); }

NAV_DEV f32x16 mfma(float a, float b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// Entry (plane p, k step q = k / 16, lane half h = (k / 8) & 1, column n) of a 16-bit B-operand
// image of one hp x hp matrix B[k][n] (k = the product's K): the 8 values of plane p of
// B[16q + 8h + j][n], j = 0..7 — one 16-B load per lane per plane and k step, 32 lanes of a
// half-wave on 512 consecutive bytes.
__host__ __device__ inline int64_t split_entry(int hp, int p, int k, int n) {
    return ((((int64_t)p * (hp / 16) + (k >> 4)) * 2 + ((k >> 3) & 1)) * hp + n) * 8 + (k & 7);
}

// ---- fp32 GEMMs on the fp16 matrix cores (the row kernels' hidden x hidden products) ----
// Both f32 operands carry a power-of-two scale and are split EXACTLY-to-22-bits into two fp16
// planes: x 2^e = hi + lo + r, hi = fp16(x 2^e), lo = fp16(x 2^e - hi) (the remainder exact in
// f32), |r| <= 2^-22 |x 2^e| (11 + 11 significant bits). sum_k a_k b_k is formed from the three
// products lo.hi + hi.lo + hi.hi on v_mfma_f32_32x32x16_f16 (fp16 x fp16 is exact in the f32
// accumulator); the dropped lo.lo is below 2^-22 |a||b|. The scales keep both planes out of fp16
// overflow and the lo plane's absolute precision (2^-24 in scaled units, the fp16 subnormal step)
// at 2^-37 of the operand's max: A (the LDS rows) per 32-row tile and GEMM, from the tile's
// max |a| that the producing epilogue publishes (publish_amax); B per column n, from the
// column's max |b|, stored with the image. The accumulators are unscaled by ldexp(acc, -(ea +
// e_n)), exact. Half the MFMAs of round 4's three-plane bf16 split (six products) at a smaller error
// (probe tools/probe/mfma_shape_probe.hip: 6.6e-7 vs 7.9e-7 relative to fp64 on uniform rows,
// 2.7e-7 vs 3.9e-7 on dz-like rows spanning 1e-9 .. 6e-5; 99 vs 156 us per 8-layer launch).
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));

NAV_DEV f32x16 mfma_h(f16x8 a, f16x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

struct Split2 {
    f16x8 h, l;
};

// acc += a . b over one 16-deep k step, the three products smallest first
NAV_DEV f32x16 mfma_x3(const Split2& a, const f16x8 (&b)[2], f32x16 c) {
    c = mfma_h(a.l, b[0], c);
    c = mfma_h(a.h, b[1], c);
    return mfma_h(a.h, b[0], c);
}

// the same with both operands split in registers: a.lo b.hi + a.hi b.lo + a.hi b.hi
NAV_DEV f32x16 mfma_x3s(const Split2& a, const Split2& b, f32x16 c) {
    c = mfma_h(a.l, b.h, c);
    c = mfma_h(a.h, b.l, c);
    return mfma_h(a.h, b.h, c);
}

// max |v| over the wave (every lane gets it)
NAV_DEV float wave_max_abs(float v) {
    v = fabsf(v);
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) v = fmaxf(v, __shfl_xor(v, m, 64));
    return v;
}

// The hi plane of a split is converted ONCE and lo is formed from those very bits: without the
// barrier the compiler may form the stored hi with v_cvt_pk_f16_f32 and rematerialise the hi
// that lo subtracts with v_cvt_f16_f32, and the two round an fp16 tie differently (hi + lo then
// misses x by one fp16 ulp of hi: tools/probe/cvt_probe.hip, a 7.8e-4 error at a tie).
template <typename T>
NAV_DEV void pin_value(T& v) {
    asm volatile("" : "+v"(v));
}

// 8 scaled f32 values -> the two fp16 fragments
NAV_DEV Split2 split2_8(const float (&v)[8]) {
    Split2 s;
#pragma unroll
    for (int j = 0; j < 8; ++j) s.h[j] = (_Float16)v[j];
    pin_value(s.h);
#pragma unroll
    for (int j = 0; j < 8; ++j) s.l[j] = (_Float16)(v[j] - (float)s.h[j]);
    return s;
}

// Exponent e with max_abs 2^e in [2^(top-1), 2^top) (0 for max_abs 0 or not finite), clamped so
// that 2^e and 2^-e are normal floats.
__host__ __device__ inline int pow2_exp_to(float max_abs, int top) {
    if (!(max_abs > 0.f) || !(max_abs < 3.0e38f)) return 0;
    int E;
    (void)frexpf(max_abs, &E);  // max_abs = m 2^E, m in [0.5, 1)
    int e = top - E;
    return e > 126 ? 126 : e < -126 ? -126 : e;
}
// an operand's scale: its max |x| 2^e in [2^13, 2^14), so products of two scaled operands and
// their K-sums stay far inside f32 and both fp16 planes inside fp16's range
__host__ __device__ inline int pow2_exp(float max_abs) { return pow2_exp_to(max_abs, 14); }

// The fp16 B image of one hp x hp matrix: planes [2][hp/16][2][hp] x 8 fp16 (split_entry), then
// the per-column exponents e_n (int32[hp]): hp^2 + hp floats.
__host__ __device__ constexpr int64_t split_image_floats(int hp) { return (int64_t)hp * hp + hp; }
NAV_DEV const int* image_exps(const float* image, int hp) {
    return reinterpret_cast<const int*>(image + (int64_t)hp * hp);
}

NAV_DEV int acc_row(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }

// Column tiles of a wave: wave w owns 32-column tiles t = w and w + 4 (when < NT) of every
// 128-row block, for all 4 row tiles: acc[rt][j] is the 32x32 tile (rows rt*32.., cols t_j*32..).
// Wave index as a scalar: the compiler then treats per-wave tile ownership as uniform control
// flow (s_cbranch) instead of exec-masked vector branches with pointer selects.
NAV_DEV int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

// ReLU masks: one 16-bit word per (row tile, column tile, lane) holding the lane's 16 C-layout
// elements' (value > 0) bits; [n_hidden][row tiles][NT][64]. The backward reads 2 bytes per 16
// elements instead of the 64 bytes of saved activations.
NAV_DEV size_t mask_idx(int64_t rowtile, int NT_, int t, int lane) {
    return ((size_t)rowtile * NT_ + t) * 64 + lane;
}

constexpr int kWaves = kBlock / 64;

#ifndef NAV_PHASE_FENCE
#define NAV_PHASE_FENCE 1
#endif
// Phase timing probe (variant builds with -DNAV_PHASE_TRACE only; tools/phase_trace.py): s_memtime
// at numbered marks, per wave of 4 traced workgroups of the row kernels.
#ifdef NAV_PHASE_TRACE
#ifdef NAV_TRACE_WIDE
// NAV_TRACE_WIDE: blocks 0, 8, 16, ... (64 of them: one XCD's share of a 512-block grid)
constexpr int kTraced = 64;
#define NAV_TRACED_SLOT() (blockIdx.x % 8 == 0 && blockIdx.x / 8 < kTraced ? (int)blockIdx.x / 8 : -1)
#else
constexpr int kTraced = 4;
// (grid row 0 only: split twins would race on the slots)
#define NAV_TRACED_SLOT()                                                                      \
    (blockIdx.y != 0 ? -1 : blockIdx.x == 0 ? 0 : blockIdx.x == 1 ? 1 : blockIdx.x == 200 ? 2   \
                          : blockIdx.x == 511 ? 3 : -1)
#endif
__device__ unsigned long long g_phase_trace[kTraced][kBlock / 64][64];
#define NAV_MARK(k)                                                                            \
    do {                                                                                       \
        const int tw_ = NAV_TRACED_SLOT();                                                     \
        if (tw_ >= 0 && (threadIdx.x & 63) == 0 && (k) >= 0 && (k) < 64)                        \
            g_phase_trace[tw_][threadIdx.x >> 6][(k)] = __builtin_readcyclecounter();          \
    } while (0)
// marks that exist only in the trace build (no scheduling fence in the product build)
#define NAV_TRACE_MARK(k) NAV_MARK(k)
#define NAV_TICK_MK 52
#elif NAV_PHASE_FENCE
// The phase marks are scheduling fences: the scheduler may not move code across a phase boundary
// (layer 0, the GEMM, the output layer, the epilogues). Without them it spreads one phase's
// loads and VALU into the next phase's MFMA loop, and the 256-VGPR actor program runs 30 %
// slower (profiles/r03zc: actor_rows 137 vs 101 us, the whole step 0.698 vs 0.668 ms).
#define NAV_MARK(k) __builtin_amdgcn_sched_barrier(0)
#else
#define NAV_MARK(k) \
    do {            \
    } while (0)
#endif
#ifndef NAV_PHASE_TRACE
#define NAV_TRACE_MARK(k) \
    do {                  \
    } while (0)
#define NAV_TICK_MK -64
#endif

// Held-clock probe (variant builds with -DNAV_CLOCK_STAMP only; tools/clock_probe.py): thread 0 of
// each of the first kClockBlocks workgroups stamps s_memtime (shader clock) and s_memrealtime
// (100 MHz) at the kernel's start and end; kernel ids: 0 critic_rows, 1 actor_rows, 2 the tick
// launch. The stamps go only to this buffer (MI355X_MICROARCH.md 'DVFS give-back' 6).
#ifdef NAV_CLOCK_STAMP
constexpr int kClockBlocks = 1024;
__device__ unsigned long long g_clock_stamp[3][kClockBlocks][4];
#define NAV_CLOCK(kid, at)                                                                     \
    do {                                                                                       \
        if (threadIdx.x == 0 && blockIdx.y == 0 && blockIdx.x < kClockBlocks) {                \
            g_clock_stamp[kid][blockIdx.x][2 * (at)] = __builtin_amdgcn_s_memtime();           \
            g_clock_stamp[kid][blockIdx.x][2 * (at) + 1] = __builtin_amdgcn_s_memrealtime();   \
        }                                                                                      \
    } while (0)
#else
#define NAV_CLOCK(kid, at) \
    do {                   \
    } while (0)
#endif

// Mask image row-tile count: independent of the workgroup height, so any RT reads what any RT
// wrote (row tile = global row / 32; layers strided by ceil(M/128)*4 tiles).
__host__ __device__ inline int64_t mask_rowtiles(int64_t M) { return ((M + 127) / 128) * 4; }

}  // namespace
