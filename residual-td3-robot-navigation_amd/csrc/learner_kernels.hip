// learner_kernels.hip — the cross-row half of the residual-TD3 learner (robot.py:236-310) on
// gfx950: hidden x hidden weight gradients on MFMA, the fixed-order gradient reduce fused with
// torch's Adam, multi-net Adam for the shared-policy bucket, Polyak soft updates (all refreshing
// the packed MFMA weight images), and the replay sampling / copy glue. The row-local half
// (forward, row backward, the fused train_critic / train_actor row programs) is mlp_kernels.hip.
#include "mlp_common.h"

namespace {

// ---------------- hidden x hidden weight gradients (split-M partial slabs) ----------------
// dW_L = dz_L^T h_{L-1} for L = 1 .. nh-1 over the rows of each split. The thin layers' gradients
// (W0, every bias, Wo, bo) are edge partials of the forward / backward kernels instead.
//
// Work decomposition: one workgroup = 8 waves = one tn x 64 output tile (n0.., k0..) of one
// layer of one network over the rows of one split; each wave takes 1/8 of the split's rows and
// keeps the tile in 32 x 32 accumulators (the MFMA K dimension is the batch row), the 8 partial
// tiles are summed through LDS in a fixed order and the workgroup writes ONE partial slab tile.
// 256 workgroups (one per CU, 2 waves per SIMD) fill the chip, so the slabs are 4-8 MB per
// launch and the reduce reads 8-16 slabs.
// 2-hidden-layer networks with whole tiles (the bench shape) take the factored path
// (wgrad_rows_fact: the ReLU bit as an exact bf16 A operand, Wo applied after the sum, tn = 128
// for d_out = 1). Every other shape takes the f32 MFMA path below (tn = 64).
// Operands come straight from registers, no panel staging and no barrier in the row loop: for
// the batch rows (2 per MFMA step: lane half h = row parity) every lane forms its own A element
// P[row][n0 + 32 i + lane] and B element Q[row][k0 + 32 j + lane]. P = dz of the top hidden
// layer is recomputed as top_unit(dy row, Wo column) under the forward's ReLU bit; Q = h_0 as
// layer0_unit(x row, W0 row, b0) — the same bits the backward / forward produced, so a 2-hidden-
// layer network reads only its input rows, dy rows and 1 bit per element. The row data (x, dy)
// of 64 rows is loaded coalesced (lane = row), parked in a wave-private LDS slot and read back
// as a broadcast per lane half; saved panels of deeper networks are read per element.
struct WgradArgs {
    MlpDev net[2];          // 1 or 2 networks, same shapes, same input rows
    int64_t M;
    const float* in;        // layer-0 input rows: h_0 is recomputed (layer0_unit)
    int ld_in, in_col;
    const float* acts[2];   // [nh][M][hp]: saved h_L, 1 <= L <= nh-2
    const float* dz[2];     // [nh][M][hp]: saved dz_L, 1 <= L <= nh-2
    const float* dy[2];     // dz_{nh-1} is recomputed: top_unit(dy row, Wo) under the ReLU bit
    int ld_dy;
    const uint16_t* masks[2];  // the forward's ReLU bit image
    float* slabs[2];        // [splits][(nh-1) hp hp]
    int splits;
    int TT;                 // 64-wide tiles across hp (the k side of a tile)
    int tn;                 // tile height on the n side: 64, or 128 (wgrad_tile_fact, d_out = 1)
    int TN;                 // tn-high tiles across hp
    int n_hid;              // tile jobs per network = (nh - 1) * TN * TT
    int fact;               // 1: the factored-Wo path (wgrad_tile_fact) for every tile
    int64_t per_split;      // rows per split (multiple of 32)
    int64_t per_wave;       // rows per wave (multiple of 32)
    int64_t skew;           // rows moved from each of waves 4-7 to its SIMD partner wave w - 4
};

// Phase probe of the weight-gradient kernels (variant builds with -DNAV_WGRAD_TRACE only;
// tools/wgrad_trace.py): s_memtime per wave at numbered marks of 4 workgroups (blocks 0, 1, 128,
// 255) per kernel (0 k_wgrad_fact, 1 k_wgrad); the last launch of each kernel wins.
#ifdef NAV_WGRAD_TRACE
__device__ unsigned long long g_wgrad_trace[2][4][8][8];
#define WG_MARK(kid, k)                                                                        \
    do {                                                                                       \
        const int b_ = blockIdx.x == 0 ? 0 : blockIdx.x == 1 ? 1 : blockIdx.x == 128 ? 2         \
                       : blockIdx.x == 255 ? 3 : -1;                                           \
        if (b_ >= 0 && (threadIdx.x & 63) == 0)                                                \
            g_wgrad_trace[kid][b_][threadIdx.x >> 6][k] = __builtin_readcyclecounter();         \
    } while (0)
#else
#define WG_MARK(kid, k) \
    do {                \
    } while (0)
#endif

constexpr int WG_WAVES = 8;
#ifndef NAV_WG_SKEW_FACT
#define NAV_WG_SKEW_FACT 64
#endif
#ifndef NAV_WG_SKEW_OPND
#define NAV_WG_SKEW_OPND 128
#endif
constexpr int WG_TOTAL = 256;  // workgroups that fill the chip (one 8-wave workgroup per CU)
constexpr int WG_THREADS = WG_WAVES * 64;
constexpr int WG_TILE = 64;
constexpr int WG_CHUNK = 64;  // rows per staged chunk (lane = row)
// LDS: 8 partial 64 x 64 tiles for the in-workgroup reduction + per wave 64 rows of (x[4], dy[2])
constexpr int WG_STAGE_FLOATS = WG_CHUNK * 6;  // one slot; 2 slots per wave (double buffer)
inline size_t wgrad_lds_bytes() {
    return ((size_t)WG_WAVES * WG_TILE * WG_TILE + (size_t)WG_WAVES * 2 * WG_STAGE_FLOATS) * 4;
}
// The factored path's tile height: 128 rows of n for d_out = 1 when hp allows (NI = 4 column
// tiles per wave at 128 accumulator registers), else 64. The path itself needs a 2-hidden-layer
// network with whole 64 x 64 tiles.
__host__ __device__ inline bool wgrad_fact_ok(int hp, int n_hidden) {
    return n_hidden == 2 && hp % WG_TILE == 0;
}
__host__ __device__ inline int wgrad_tile_n(int d_out, int hp, int n_hidden) {
    return wgrad_fact_ok(hp, n_hidden) && d_out == 1 && hp % 128 == 0 ? 128 : WG_TILE;
}

// rows [r_lo, r_hi) of one wave into acc (tile n0.., k0.. of layer L of net y)
// RA (k_wgrad_gen): the chunk's saved dz / h row values are loaded into registers before its
// products (loaded at their use inside the product they exposed one memory round trip per row
// pair: ~20 k cycles for 32 rows at config 1's shape, profiles/r06zj); k_wgrad, whose MFMA-operand
// path holds 254 registers, keeps the loads at their use
template <bool PR, bool QR, bool RA_ = false>
NAV_DEV void wgrad_rows(const WgradArgs& a, int y, int L, int n0, int k0, int64_t r_lo,
                        int64_t r_hi, float* stage, f32x16 (&acc)[2][2]) {
    const MlpDev& net = a.net[y];
    const int hp = net.hp, nh = net.n_hidden, d_in = net.d_in, d_out = net.d_out;
    const int lane = threadIdx.x & 63, h = lane >> 5, l32 = lane & 31;
    const int64_t M = a.M, MH = M * hp;
    // 32-column sub-tiles inside hp (wave-uniform); absent columns read a clamped valid column
    const bool nv1 = n0 + 32 < hp, kv1 = k0 + 32 < hp;
    const int cn[2] = {n0 + l32, nv1 ? n0 + 32 + l32 : n0 + l32};
    const int ck[2] = {k0 + l32, kv1 ? k0 + 32 + l32 : k0 + l32};
    float wo[2][2] = {{0.f, 0.f}, {0.f, 0.f}}, w0[2][4] = {}, b0[2] = {0.f, 0.f};
    if (PR) {
        const float* Wo = net.params + net.w_off[nh];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            wo[i][0] = Wo[cn[i]];
            wo[i][1] = d_out > 1 ? Wo[hp + cn[i]] : 0.f;
        }
    }
    if (QR) {
        const float* W0 = net.params + net.w_off[0];
        const float* bb = net.params + net.b_off[0];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
#pragma unroll
            for (int k = 0; k < 4; ++k) w0[j][k] = k < d_in ? W0[ck[j] * d_in + k] : 0.f;
            b0[j] = bb[ck[j]];
        }
    }
    // one saved operand only (two would not fit next to the accumulators), HS row pairs at a time
    constexpr bool RA = RA_ && (PR != QR);
    constexpr int HS = WG_CHUNK / 8;  // row pairs per register window
    const int NTm = hp >> 5;
    const uint16_t* mk = PR ? a.masks[y] + (size_t)(nh - 1) * mask_rowtiles(M) * NTm * 64 : nullptr;
    const int tm0 = n0 >> 5, tm1 = nv1 ? tm0 + 1 : tm0;
    const float* Psv = PR ? nullptr : a.dz[y] + (int64_t)L * MH;
    const float* Qsv = QR ? nullptr : a.acts[y] + (int64_t)(L - 1) * MH;
    float* xs = stage;                  // [64][4]
    float* gs = stage + WG_CHUNK * 4;   // [64][2]

    // one chunk's row data in registers: x row (QR), dy row (PR), and the ReLU words of the
    // chunk's 2 row tiles x 2 column tiles (PR): bits of rows with (row & 4) == 0 in the low half
    float4 cx = make_float4(0.f, 0.f, 0.f, 0.f);
    float2 cg = make_float2(0.f, 0.f);
    uint32_t cm[2][2] = {{0u, 0u}, {0u, 0u}};
    auto load = [&](int64_t rb) {
        const int64_t r = rb + lane;
        const bool ok = r < r_hi;
        const int64_t rc = ok ? r : r_lo;
        if (QR) {
            const float* x = a.in + rc * a.ld_in + a.in_col;
            cx.x = ok ? x[0] : 0.f;
            cx.y = ok && d_in > 1 ? x[1] : 0.f;
            cx.z = ok && d_in > 2 ? x[2] : 0.f;
            cx.w = ok && d_in > 3 ? x[3] : 0.f;
        }
        if (PR) {
            const float* g = a.dy[y] + rc * a.ld_dy;
            cg.x = ok ? g[0] : 0.f;
            cg.y = ok && d_out > 1 ? g[1] : 0.f;
            const int64_t rt0 = rb >> 5;
            const bool t1 = rb + 32 < r_hi;  // a range may end after the chunk's first tile
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int t = 0; t < 2; ++t) {
                    const uint16_t* w = mk + ((rt0 + (t && t1)) * NTm + (i ? tm1 : tm0)) * 64 + l32;
                    cm[i][t] = t && !t1 ? 0u : (uint32_t)w[0] | ((uint32_t)w[32] << 16);
                }
        }
    };
    auto park = [&]() {
        if (QR) *reinterpret_cast<float4*>(xs + lane * 4) = cx;
        if (PR) *reinterpret_cast<float2*>(gs + lane * 2) = cg;
    };
    if (r_lo >= r_hi) return;
    load(r_lo);
    park();
    uint32_t mw[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int t = 0; t < 2; ++t) mw[i][t] = cm[i][t] >> h;  // the lane half's row parity
    for (int64_t rb = r_lo; rb < r_hi; rb += WG_CHUNK) {
        const bool more = rb + WG_CHUNK < r_hi;
        if (more) load(rb + WG_CHUNK);  // next chunk in flight under this one
        float ps[RA && !PR ? HS : 1][2], qs[RA && !QR ? HS : 1][2];
        auto window = [&](int s0) {  // the saved row values of row pairs s0 .. s0 + HS - 1
#pragma unroll
            for (int u = 0; u < HS; ++u) {
                const int64_t r = rb + 2 * (s0 + u) + h;
                const bool ok = r < r_hi;
                const int64_t rc = ok ? r : r_lo;
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    if constexpr (!PR) ps[u][i] = ok ? Psv[rc * hp + cn[i]] : 0.f;
                    if constexpr (!QR) qs[u][i] = ok ? Qsv[rc * hp + ck[i]] : 0.f;
                }
            }
        };
#pragma unroll
        for (int s = 0; s < WG_CHUNK / 2; ++s) {
            // wave-uniform: a range's last chunk may be short (RA stops at a window boundary: the
            // window's rows past r_hi add exact zeros, and its row registers stay static)
            if ((!RA || s % HS == 0) && rb + 2 * s >= r_hi) break;
            if constexpr (RA) {
                if (s % HS == 0) window(s);
            }
            const int rr = 2 * s + h;  // row of this lane half inside the chunk
            float p[2], q[2];
            if (PR) {
                const float2 g = *reinterpret_cast<const float2*>(gs + rr * 2);
                // bit of row rr in the C-layout mask word: element (rr & 3) + 4 (rr >> 3 & 3) of
                // lane half (rr >> 2) & 1 (the +h of rr was folded into mw)
                const int sh = 16 * ((s >> 1) & 1) + 2 * (s & 1) + 4 * ((s & 15) >> 2);
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    const uint32_t bit = (mw[i][s >> 4] >> sh) & 1u;
                    p[i] = bit ? top_unit(g.x, g.y, wo[i][0], wo[i][1]) : 0.f;
                }
            } else if constexpr (RA) {
#pragma unroll
                for (int i = 0; i < 2; ++i) p[i] = ps[RA && !PR ? s % HS : 0][i];
            } else {
                const int64_t r = rb + rr;
                const bool ok = r < r_hi;
                const float* src = Psv + (ok ? r : r_lo) * hp;
#pragma unroll
                for (int i = 0; i < 2; ++i) p[i] = ok ? src[cn[i]] : 0.f;
            }
            if (QR) {
                const float4 x = *reinterpret_cast<const float4*>(xs + rr * 4);
#pragma unroll
                for (int j = 0; j < 2; ++j) q[j] = layer0_unit(x, w0[j][0], w0[j][1], w0[j][2], w0[j][3], b0[j]);
            } else if constexpr (RA) {
#pragma unroll
                for (int j = 0; j < 2; ++j) q[j] = qs[RA && !QR ? s % HS : 0][j];
            } else {
                const int64_t r = rb + rr;
                const bool ok = r < r_hi;
                const float* src = Qsv + (ok ? r : r_lo) * hp;
#pragma unroll
                for (int j = 0; j < 2; ++j) q[j] = ok ? src[ck[j]] : 0.f;
            }
            acc[0][0] = mfma(p[0], q[0], acc[0][0]);
            if (kv1) acc[0][1] = mfma(p[0], q[1], acc[0][1]);
            if (nv1) acc[1][0] = mfma(p[1], q[0], acc[1][0]);
            if (nv1 && kv1) acc[1][1] = mfma(p[1], q[1], acc[1][1]);
        }
        if (more) {
            park();  // this wave's reads of the slot were issued above: LDS keeps them in order
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int t = 0; t < 2; ++t) mw[i][t] = cm[i][t] >> h;
        }
    }
}

// Wave-uniform max |dy_d| (d < d_out) and max |x_i| (i < d_in) over the wave's rows [r_lo, r_hi):
// the bounds behind the fp16 operand scales of the weight-gradient products (a bound within a
// few binades of the true max costs nothing: the lo plane's absolute step stays 2^-24 of the
// scaled bound).
NAV_DEV void row_maxima(const WgradArgs& a, int y, int64_t r_lo, int64_t r_hi, float (&G)[2],
                        float (&X)[4]) {
    const int lane = threadIdx.x & 63, d_in = a.net[y].d_in, d_out = a.net[y].d_out;
    float g0 = 0.f, g1 = 0.f, x0 = 0.f, x1 = 0.f, x2 = 0.f, x3 = 0.f;
    // RU rows per lane per trip, every load of a trip issued before the first max (one memory
    // round trip per 64 RU rows), whole-row vector loads where the layout allows (the rows are
    // 32 B apart in the learner's batch: one load instruction per row instead of d_in)
    constexpr int RU = 4;
    const float* xin = a.in + a.in_col;
    const bool xv4 = d_in == 4 && (a.ld_in & 3) == 0 && ((uintptr_t)xin & 15) == 0;
    const bool xv2 = d_in == 2 && (a.ld_in & 1) == 0 && ((uintptr_t)xin & 7) == 0;
    const bool gv2 = d_out == 2 && (a.ld_dy & 1) == 0 && ((uintptr_t)a.dy[y] & 7) == 0;
    for (int64_t rb = r_lo; rb < r_hi; rb += 64 * RU) {
        float gv[RU][2], xv[RU][4];
#pragma unroll
        for (int u = 0; u < RU; ++u) {
            gv[u][0] = gv[u][1] = 0.f;
            xv[u][0] = xv[u][1] = xv[u][2] = xv[u][3] = 0.f;
            if (rb + 64 * u >= r_hi) continue;  // wave-uniform
            const int64_t r = rb + 64 * u + lane;
            if (r >= r_hi) continue;
            const float* g = a.dy[y] + r * a.ld_dy;
            const float* x = xin + r * a.ld_in;
            if (gv2) {
                const float2 v = *reinterpret_cast<const float2*>(g);
                gv[u][0] = v.x;
                gv[u][1] = v.y;
            } else {
                gv[u][0] = g[0];
                if (d_out > 1) gv[u][1] = g[1];
            }
            if (xv4) {
                const float4 v = *reinterpret_cast<const float4*>(x);
                xv[u][0] = v.x; xv[u][1] = v.y; xv[u][2] = v.z; xv[u][3] = v.w;
            } else if (xv2) {
                const float2 v = *reinterpret_cast<const float2*>(x);
                xv[u][0] = v.x; xv[u][1] = v.y;
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    if (d_in > i) xv[u][i] = x[i];
            }
        }
#pragma unroll
        for (int u = 0; u < RU; ++u) {
            g0 = fmaxf(g0, fabsf(gv[u][0]));
            g1 = fmaxf(g1, fabsf(gv[u][1]));
            x0 = fmaxf(x0, fabsf(xv[u][0]));
            x1 = fmaxf(x1, fabsf(xv[u][1]));
            x2 = fmaxf(x2, fabsf(xv[u][2]));
            x3 = fmaxf(x3, fabsf(xv[u][3]));
        }
    }
    // wave-uniform: scalar registers
    auto su = [](float v) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(wave_max_abs(v)))); };
    G[0] = su(g0);
    G[1] = su(g1);
    X[0] = su(x0);
    X[1] = su(x1);
    X[2] = su(x2);
    X[3] = su(x3);
}

// Bound on |h_0[r][c]| = relu(b0[c] + sum_i x_ri W0[c][i]) for the column c of this lane from the
// lane half's constants (inputs h and 2 + h; the bias on h = 0): sum_i X_i |W0[c][i]| + |b0[c]|.
NAV_DEV float h0_bound(const float (&X)[4], float wa, float wb, float bias) {
    const int h = (threadIdx.x & 63) >> 5;
    const float part = (h ? X[1] : X[0]) * fabsf(wa) + (h ? X[3] : X[2]) * fabsf(wb) + fabsf(bias);
    return part + __shfl_xor(part, 32, 64);
}

// The largest exponent <= e at which a constant of magnitude <= m stays finite when scaled by
// 2^e (m 2^e < 2^126). The h_0 scale comes from the bound above, which is tiny when the inputs
// and the bias are: the layer-0 weights scaled by it would overflow to inf and a zero input row
// then give 0 * inf = NaN in the operand MFMA. Binds only in that degenerate case (the bound's
// own 2^14 target keeps e below it otherwise), so normal results are unchanged.
NAV_DEV int cap_exp_finite(int e, float m) {
    if (!(m > 0.f)) return e;
    int E;
    (void)frexpf(m, &E);  // m = f 2^E, f in [0.5, 1)
    return min(e, 126 - E);
}

// The MFMA-operand path for a full 64 x 64 tile of a 2-hidden-layer network with d_out = 2 (the
// actor; d_out = 1 takes the factored path below).
// The operands are produced by MFMAs too: per 32-row tile, dz = dy . Wo (K = d_out <= 2, one
// v_mfma_f32_32x32x2_f32 per 32 columns) and h_0 = x . W0^T + b0 (K = d_in <= 4, two MFMAs on
// the bias as C) land in the C layout, where lane (l32, h) register e holds row
// acc_row(e, h) of column l32. Taking the weight-gradient MFMA's K (batch-row) order as
// step e <-> rows {acc_row(e, 0), acc_row(e, 1)}, register e of those tiles IS the A / B operand
// of step e, and bit e of the lane's own ReLU mask word (the forward's C-layout image) is the
// ReLU derivative of exactly that element. Per 64 weight-gradient MFMAs a wave issues 6 operand
// MFMAs and ~100 VALU (mask, relu) instead of ~320 VALU: the f32 MFMA shares the SIMD's issue
// with the VALU, so the VALU count per MFMA is what sets the rate. No LDS, no barrier in the
// row loop. h_0 and dz are the forward's / backward's values as fused f32 chains in the same
// order (layer0_unit: b + x0 w0 + x1 w1 + ..., top_unit: g0 w0 + g1 w1).
NAV_DEV void wgrad_rows_mfma(const WgradArgs& a, int y, int n0, int k0, int64_t r_lo,
                             int64_t r_hi, f32x16 (&acc)[2][2]) {
    const MlpDev& net = a.net[y];
    const int hp = net.hp, nh = net.n_hidden, d_in = net.d_in, d_out = net.d_out;
    const int lane = threadIdx.x & 63, h = lane >> 5, l32 = lane & 31;
    const int64_t M = a.M;
    const int NTm = hp >> 5;
    // constant B operands of the operand MFMAs: Wo rows (k = output j = h), W0 columns (k = h,
    // then 2 + h), and the bias through a K = 2 MFMA of (1, 0) x (b, 0): the C tile starts at b
    // exactly, so h_0 accumulates in layer0_unit's order b + x0 w0 + x1 w1 + x2 w2 + x3 w3
    float wob[2], w0b[2][2], bob[2];
    {
        const float* Wo = net.params + net.w_off[nh];
        const float* W0 = net.params + net.w_off[0];
        const float* bb = net.params + net.b_off[0];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            wob[i] = h < d_out ? Wo[h * hp + n0 + 32 * i + l32] : 0.f;
            const int c = k0 + 32 * i + l32;
            w0b[i][0] = h < d_in ? W0[c * d_in + h] : 0.f;
            w0b[i][1] = 2 + h < d_in ? W0[c * d_in + 2 + h] : 0.f;
            bob[i] = h == 0 ? bb[c] : 0.f;
        }
    }
    if (r_lo >= r_hi) return;
    const uint16_t* mk = a.masks[y] + (size_t)(nh - 1) * mask_rowtiles(M) * NTm * 64 +
                         (size_t)(n0 >> 5) * 64 + lane;
    const size_t mstride = (size_t)NTm * 64;
    const float* dyp = a.dy[y];
    const int ld_dy = a.ld_dy, ld_in = a.ld_in;
    const float* xin = a.in + a.in_col;
    // raw loads of a 32-row tile (A operands: lane l32 = row, h = k; the lane's 2 mask words),
    // in tile order through running per-lane pointers (a 64-bit add per stream and tile: the
    // address math is VALU, which the f32 MFMA waits for); a partial last tile reads clamped rows,
    // and what does not exist is zeroed where it is used
    const int gk = h < d_out ? h : 0, xk0 = h < d_in ? h : 0, xk1 = 2 + h < d_in ? 2 + h : 0;
    struct Raw {
        float g, x0, x1;
        uint32_t m0, m1;
    };
    const float* gp = dyp + (r_lo + l32) * ld_dy + gk;
    const float* xp = xin + (r_lo + l32) * ld_in;
    const uint16_t* mp = mk + (size_t)(r_lo >> 5) * mstride;
    const int64_t gstep = 32 * (int64_t)ld_dy, xstep = 32 * (int64_t)ld_in;
    int64_t rl = r_lo;  // first row of the next tile to load
    auto load = [&](int64_t) {
        Raw v;
        if (rl + 32 <= r_hi) {
            v.g = *gp;
            v.x0 = xp[xk0];
            v.x1 = xp[xk1];
            v.m0 = mp[0];
            v.m1 = mp[64];
        } else {  // rows past r_hi read row r_lo (the values are not used)
            const bool ok = rl + l32 < r_hi;
            const float* g = ok ? gp : dyp + r_lo * ld_dy + gk;
            const float* x = ok ? xp : xin + r_lo * ld_in;
            v.g = *g;
            v.x0 = x[xk0];
            v.x1 = x[xk1];
            v.m0 = mp[0];
            v.m1 = mp[64];
        }
        gp += gstep;
        xp += xstep;
        mp += mstride;
        rl += 32;
        return v;
    };
    // operand MFMAs of one tile (results in the C layout, masked later by finish())
    // the h_0 tiles start at the (scaled) bias of their column, set by VALU: the same C operand
    // the K = 2 bias MFMA of (1, 0) x (b, 0) produced (exactly b), one f32 MFMA fewer per column
    // half and tile; inputs 2, 3 only exist for d_in > 2 (the actor has 2)
    float bc[2];  // set below, after the scales
    const bool x23 = d_in > 2;
    auto issue = [&](int64_t rt, const Raw& v, f32x16 (&P)[2], f32x16 (&Q)[2]) {
        const bool ok = rt + l32 < r_hi && h < d_out;  // rows past r_hi: dz = 0, add nothing
        const float g = ok ? v.g : 0.f;
        const float x0 = h < d_in ? v.x0 : 0.f, x1 = 2 + h < d_in ? v.x1 : 0.f;
        const f32x16 zero = {};
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            P[i] = mfma(g, wob[i], zero);
            f32x16 b;
#pragma unroll
            for (int e = 0; e < 16; ++e) b[e] = bc[i];
            Q[i] = mfma(x0, w0b[i][0], b);
        }
        if (x23) {
#pragma unroll
            for (int i = 0; i < 2; ++i) Q[i] = mfma(x1, w0b[i][1], Q[i]);
        }
    };
    // ReLU derivative of the top layer on P (bit e of the lane's word as an all-ones mask) and
    // the layer-0 ReLU on Q (an integer max of the bit pattern: one v_max_i32)
    auto finish = [&](const Raw& v, f32x16 (&P)[2], f32x16 (&Q)[2]) {
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            // v_bfe_i32 of one bit: 0 or all ones
            P[0][e] = __int_as_float(__float_as_int(P[0][e]) & __builtin_amdgcn_sbfe((int)v.m0, e, 1));
            P[1][e] = __int_as_float(__float_as_int(P[1][e]) & __builtin_amdgcn_sbfe((int)v.m1, e, 1));
            Q[0][e] = __int_as_float(max(__float_as_int(Q[0][e]), 0));
            Q[1][e] = __int_as_float(max(__float_as_int(Q[1][e]), 0));
        }
    };
    // per 32-row tile: the operand MFMAs, their ReLU epilogue, then the tile's two 16-deep k steps
    // of the fp16 product (the partner wave on the SIMD keeps the matrix pipe busy while this one
    // waits for its operand MFMAs; double-buffering the operand tiles would not fit the 256
    // registers of two waves per SIMD next to the split fragments). The raw loads run two tiles
    // ahead.
    Raw cur = load(r_lo);
    Raw nxt = cur;
    if (r_lo + 32 < r_hi) nxt = load(r_lo + 32);
    // (the first two tiles' loads are in flight under the bound pre-pass)
    // fp16 operand scales (mlp_common.h), folded into the operand MFMAs' constants (a power of two
    // commutes with every rounding of the f32 chains): P column tile i by 2^ep[i] from the bound
    // sum_d max|g_d| |Wo[d][n]| (max over the tile's 32 n), Q column k by 2^eq[j] from h0_bound
    int ep[2], eq[2];
    {
        float G[2], X[4];
        WG_MARK(1, 2);
        row_maxima(a, y, r_lo, r_hi, G, X);
        WG_MARK(1, 3);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            float b = G[h] * fabsf(wob[i]);
            b += __shfl_xor(b, 32, 64);
#pragma unroll
            for (int m = 1; m < 32; m <<= 1) b = fmaxf(b, __shfl_xor(b, m, 64));
            ep[i] = pow2_exp(b);
            wob[i] = ldexpf(wob[i], ep[i]);
            float wm = fmaxf(fmaxf(fabsf(w0b[i][0]), fabsf(w0b[i][1])), fabsf(bob[i]));
            wm = fmaxf(wm, __shfl_xor(wm, 32, 64));
            eq[i] = cap_exp_finite(pow2_exp(h0_bound(X, w0b[i][0], w0b[i][1], bob[i])), wm);
            w0b[i][0] = ldexpf(w0b[i][0], eq[i]);
            w0b[i][1] = ldexpf(w0b[i][1], eq[i]);
            bob[i] = ldexpf(bob[i], eq[i]);
            bc[i] = bob[i] + __shfl_xor(bob[i], 32, 64);  // the column's scaled bias, both halves
        }
    }
    for (int64_t rt = r_lo; rt < r_hi; rt += 32) {
        Raw nn = nxt;
        if (rt + 64 < r_hi) nn = load(rt + 64);
        f32x16 P[2], Q[2];
        issue(rt, cur, P, Q);
        finish(cur, P, Q);
        // registers 8s .. 8s+7 of the C-layout operands are k step s (rows 16s + 8(j>>2) + 4h +
        // (j&3), the same for P and Q), each (already scaled) split into two fp16 planes right
        // before its three products
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
            Split2 sp[2], sq[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                float vp[8], vq[8];
#pragma unroll
                for (int t = 0; t < 8; ++t) {
                    vp[t] = P[i][8 * s2 + t];
                    vq[t] = Q[i][8 * s2 + t];
                }
                sp[i] = split2_8(vp);
                sq[i] = split2_8(vq);
            }
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[i][j] = mfma_x3s(sp[i], sq[j], acc[i][j]);
        }
        cur = nxt;
        nxt = nn;
    }
    WG_MARK(1, 4);
    // unscale: tile (i, j) by 2^-(ep[i] + eq[j]) (eq per lane column), exact
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = ldexpf(acc[i][j][e], -(ep[i] + eq[j]));
}

// ---- the factored form for 2-hidden-layer networks (the bench shape) ----
// With e the forward's ReLU bit of the top hidden layer and g_d = dL/dy_d,
//   dz_1[r][n] = e[r][n] sum_d g_d[r] Wo[d][n]        (robot.py:355-363 autograd, d < d_out)
//   dW_1[n][k] = sum_r dz_1[r][n] h_0[r][k] = sum_d Wo[d][n] S_d[n][k],
//   S_d[n][k]  = sum_r e[r][n] Q_d[r][k],   Q_d[r][k] = g_d[r] h_0[r][k].
// The A operand of S_d is the ReLU bit itself, exact in fp16 (as 2.0, the 0.5 goes into Wo; 8
// bits of a mask word become an A fragment by one 16-B read of a 256-entry LDS table — fp16 2.0
// and bf16 2.0 share the bit pattern 0x4000), and only the B operand Q_d is split: scaled by a
// power of two (h_0 per column k into [2^6, 2^7) through the layer-0 constants, g_d per wave into
// [2^7, 2^8) from the wave's max |g_d|) and cut into two fp16 planes, so the product carries f32
// accuracy with 2 MFMAs per 16-deep k step and 32 x 32 tile (the three-plane bf16 form: 3), and
// nothing per element on the n side. That frees a wave to own NI = 4 column tiles of n
// (128 x 64) at D = 1 — the twin critics — for 128 accumulator registers.


// GV: dy rows packed (ld_dy = D) and 16-B aligned (float4 loads at fixed offsets); XV: x rows of 4
// floats, 16-B aligned (one float4 load per row). Both are launch-uniform: the full-tile loop is
// compiled per form, with running row pointers and no per-tile branch on the layout.
template <int NI, int D, bool GV, bool XV>
NAV_DEV void wgrad_rows_fact(const WgradArgs& a, int y, int n0, int k0, int64_t r_lo,
                             int64_t r_hi, const char* tab, f32x16 (&out)[NI][2]) {
    const MlpDev& net = a.net[y];
    const int hp = net.hp, d_in = net.d_in;
    const int lane = threadIdx.x & 63, h = lane >> 5, l32 = lane & 31;
    const int64_t M = a.M;
    const int NTm = hp >> 5;
    f32x16 acc[D][NI][2];
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int e = 0; e < 16; ++e) acc[d][i][j][e] = 0.f;
    // h_0 = relu(x . W0^T + b0) by f32 MFMAs in the C layout, where lane (l32, h) register e
    // holds row acc_row(e, h) of column l32. Constant B operands: W0 columns (k = h, then 2 + h),
    // and the bias through a K = 2 MFMA of (1, 0) x (b, 0), so the C tile starts at b exactly and
    // h_0 accumulates in layer0_unit's order b + x0 w0 + x1 w1 + x2 w2 + x3 w3
    float w0b[2][2], bob[2];
    {
        const float* W0 = net.params + net.w_off[0];
        const float* bb = net.params + net.b_off[0];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int c = k0 + 32 * j + l32;
            w0b[j][0] = h < d_in ? W0[c * d_in + h] : 0.f;
            w0b[j][1] = 2 + h < d_in ? W0[c * d_in + 2 + h] : 0.f;
            bob[j] = h == 0 ? bb[c] : 0.f;
        }
    }
    int eh[2], eg[D];  // the fp16 operand scales (below, under the first tile's loads)
    float sg[D];
    float bcj[2];      // the scaled bias of the lane's column per half (below, with the scales)
    const bool x23 = d_in > 2;
    const size_t mstride = (size_t)NTm * 64;
    const uint16_t* mp = a.masks[y] + (size_t)mask_rowtiles(M) * mstride +  // layer 1's bits
                         (size_t)(n0 >> 5) * 64 + lane + (size_t)(r_lo >> 5) * mstride;
    const float* dyp = a.dy[y];
    const int ld_dy = a.ld_dy, ld_in = a.ld_in;
    const int xk0 = h < d_in ? h : 0, xk1 = 2 + h < d_in ? 2 + h : 0;
    // the tile's own A operands (x row of lane l32, inputs k = h and 2 + h) and the lane's NI
    // mask words; the main loop keeps the next full tile's in flight
    struct Raw {
        float x0, x1;
        uint32_t m[NI];
    };
    // the x row as one 16-B load when it is 4 aligned floats (both lane halves read the row)
    const bool xrow4 = d_in == 4 && (ld_in & 3) == 0 && (((uintptr_t)(a.in + a.in_col)) & 15) == 0;
    auto load_raw = [&](int64_t rt, Raw& v) {
        const int64_t rx = rt + l32 < r_hi ? rt + l32 : r_lo;  // absent rows read row r_lo
        const float* x = a.in + a.in_col + rx * ld_in;
        if (xrow4) {
            const float4 u = *reinterpret_cast<const float4*>(x);
            v.x0 = h ? u.y : u.x;
            v.x1 = h ? u.w : u.z;
        } else {
            v.x0 = x[xk0];
            v.x1 = x[xk1];
        }
        const uint16_t* m = mp + (size_t)((rt - r_lo) >> 5) * mstride;
#pragma unroll
        for (int i = 0; i < NI; ++i) v.m[i] = m[i * 64];
    };
    // one 32-row tile: h_0 by the f32 MFMAs, Q_d = relu(h_0) g_d split per k step, 2 MFMAs per
    // (i, j, d) and step. gs[s2][d][t]: g_d (scaled) of the row of register e = 8 s2 + t
    auto tile = [&](const Raw& cur, const float (&gs)[2][D][8]) {
        const float x0 = h < d_in ? cur.x0 : 0.f, x1 = 2 + h < d_in ? cur.x1 : 0.f;
        // one 32-column half j of the k side at a time (16 registers of h_0 live)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            // the C operand starts at the column's scaled bias (exactly what the K = 2 bias MFMA
            // of (1, 0) x (b, 0) produced), set by VALU: one f32 MFMA fewer per half and tile
            f32x16 Z;
#pragma unroll
            for (int e = 0; e < 16; ++e) Z[e] = bcj[j];
            Z = mfma(x0, w0b[j][0], Z);
            if (x23) Z = mfma(x1, w0b[j][1], Z);
            // registers 8s .. 8s+7 of the C layout are k step s (rows 16s + 8(t>>2) + 4h +
            // (t&3)), the same rows as bits 8s .. 8s+7 of the lane's mask words
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
                for (int d = 0; d < D; ++d) {
                    float q[8];
#pragma unroll
                    for (int t = 0; t < 8; ++t)
                        q[t] = __int_as_float(max(__float_as_int(Z[8 * s2 + t]), 0)) * gs[s2][d][t];
                    const Split2 sq = split2_8(q);
#pragma unroll
                    for (int i = 0; i < NI; ++i) {
                        // the fragment of byte s2 of the mask word, read from the table right
                        // before its 3 MFMAs (the opaque offset keeps the compiler from holding
                        // all NI x 2 fragments live across the passes over j)
                        uint32_t ta = (s2 == 0 ? cur.m[i] << 4 : cur.m[i] >> 4) & 0xFF0u;
                        asm volatile("" : "+v"(ta));
                        const f16x8 pi = *reinterpret_cast<const f16x8*>(tab + ta);
                        acc[d][i][j] = mfma_h(pi, sq.l, acc[d][i][j]);
                        acc[d][i][j] = mfma_h(pi, sq.h, acc[d][i][j]);
                    }
                }
        }
    };
    const int64_t r_full = r_lo + ((r_hi - r_lo) & ~(int64_t)31);
    constexpr int LDG = GV ? D : 0;  // the compile-time dy row stride of the GV form
    const int ldg = GV ? LDG : ld_dy;
    // the g values of rows rt + 4h + 16 s2 + 8 qq + t (register e = 8 s2 + 4 qq + t of the C
    // layout) from the row pointer g0 = dy + (rt + 4h) ldg
    auto load_g_at = [&](const float* gp, float (&gs)[2][D][8]) {
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
            for (int qq = 0; qq < 2; ++qq) {
                const float* g = gp + (16 * s2 + 8 * qq) * ldg;
                if (GV && D == 1) {
                    const float4 u = *reinterpret_cast<const float4*>(g);
                    gs[s2][0][4 * qq] = u.x; gs[s2][0][4 * qq + 1] = u.y;
                    gs[s2][0][4 * qq + 2] = u.z; gs[s2][0][4 * qq + 3] = u.w;
                } else if (GV) {
                    const float4 u0 = *reinterpret_cast<const float4*>(g);
                    const float4 u1 = *reinterpret_cast<const float4*>(g + 4);
                    gs[s2][0][4 * qq] = u0.x; gs[s2][D - 1][4 * qq] = u0.y;
                    gs[s2][0][4 * qq + 1] = u0.z; gs[s2][D - 1][4 * qq + 1] = u0.w;
                    gs[s2][0][4 * qq + 2] = u1.x; gs[s2][D - 1][4 * qq + 2] = u1.y;
                    gs[s2][0][4 * qq + 3] = u1.z; gs[s2][D - 1][4 * qq + 3] = u1.w;
                } else {
#pragma unroll
                    for (int t = 0; t < 4; ++t)
#pragma unroll
                        for (int d = 0; d < D; ++d) gs[s2][d][4 * qq + t] = g[t * ldg + d];
                }
            }
    };
    // the g scales on the loaded values (D = 2; D = 1 folds them into the layer-0 constants)
    auto scale_g = [&](float (&gs)[2][D][8]) {
        if (D == 1) return;
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
            for (int d = 0; d < D; ++d)
#pragma unroll
                for (int t = 0; t < 8; ++t) gs[s2][d][t] *= sg[d];
    };
    // full tiles: running per-lane pointers (x row, mask words, g rows), every row in range, so no
    // clamp; d_out = 1 loads its g values one tile ahead with the rest (d_out = 2 at the tile: its
    // 32 prefetched values do not fit the registers)
    constexpr bool GPF = D == 1;
    const int64_t nfull = (r_full - r_lo) >> 5;
    const float* xq = a.in + a.in_col + (r_lo + l32) * (int64_t)ld_in;
    const uint16_t* mq = mp;
    const float* gq = dyp + (r_lo + 4 * h) * (int64_t)ldg;
    const int64_t xstep = 32 * (int64_t)ld_in, gstep = 32 * (int64_t)ldg;
    auto load_full = [&](Raw& v, float (&gs)[2][D][8]) {
        if (XV) {
            const float4 u = *reinterpret_cast<const float4*>(xq);
            v.x0 = h ? u.y : u.x;
            v.x1 = h ? u.w : u.z;
        } else {
            v.x0 = xq[xk0];
            v.x1 = xq[xk1];
        }
#pragma unroll
        for (int i = 0; i < NI; ++i) v.m[i] = mq[i * 64];
        if (GPF) load_g_at(gq, gs);
        xq += xstep;
        mq += mstride;
        gq += gstep;
    };
    Raw c0, c1;
    float g0[2][D][8], g1[2][D][8];
    if (nfull > 0) load_full(c0, g0);
    // the scales, computed under the first tile's loads: h_0 column half j by 2^eh[j] (folded into
    // the layer-0 constants: a power of two commutes with the fma chain's roundings), g_d by
    // 2^eg[d] (D = 1: folded into the same constants, so the g rows are used as loaded; D = 2:
    // applied to the loaded g values)
    {
        float G[2], X[4];
        WG_MARK(0, 2);
        row_maxima(a, y, r_lo, r_hi, G, X);
        WG_MARK(0, 3);
#pragma unroll
        for (int d = 0; d < D; ++d) {
            eg[d] = pow2_exp_to(G[d], 8);
            sg[d] = D == 1 ? 1.f : ldexpf(1.f, eg[d]);
        }
        // per 32-column half (wave-uniform, scalar registers: the 128-accumulator program has no
        // vector register to spare)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            eh[j] = __builtin_amdgcn_readfirstlane(
                pow2_exp_to(wave_max_abs(h0_bound(X, w0b[j][0], w0b[j][1], bob[j])), 7));
            // (the sum capped at 2^120: Z = h_0 2^eh stays finite for every finite h_0 bound)
            if (D == 1) eh[j] = min(max(eh[j] + eg[0], -126), 120);
            eh[j] = __builtin_amdgcn_readfirstlane(cap_exp_finite(
                eh[j], wave_max_abs(fmaxf(fmaxf(fabsf(w0b[j][0]), fabsf(w0b[j][1])),
                                          fabsf(bob[j])))));
            w0b[j][0] = ldexpf(w0b[j][0], eh[j]);
            w0b[j][1] = ldexpf(w0b[j][1], eh[j]);
            bob[j] = ldexpf(bob[j], eh[j]);
            bcj[j] = bob[j] + __shfl_xor(bob[j], 32, 64);  // the column's scaled bias, both halves
        }
        if (D == 1) eg[0] = 0;
    }
    for (int64_t t = 0; t < nfull; ++t) {
        if (t + 1 < nfull) load_full(c1, g1);
        if (!GPF) load_g_at(dyp + (r_lo + 32 * t + 4 * h) * (int64_t)ldg, g0);
        scale_g(g0);
        tile(c0, g0);
        c0 = c1;
        if (GPF) {
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
                for (int d = 0; d < D; ++d)
#pragma unroll
                    for (int e = 0; e < 8; ++e) g0[s2][d][e] = g1[s2][d][e];
        }
    }
    WG_MARK(0, 4);
    if (r_full < r_hi) {  // the last, partial tile of the rows (M % 32 rows)
        Raw cur;
        load_raw(r_full, cur);
        float gs[2][D][8];
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int64_t r = r_full + acc_row(e, h);
#pragma unroll
            for (int d = 0; d < D; ++d) gs[e >> 3][d][e & 7] = r < r_hi ? dyp[r * ld_dy + d] * sg[d] : 0.f;
        }
        tile(cur, gs);
    }
    // dW tile = sum_d (Wo[d][n] / 2) S_d: register e of tile (i, j) is row n = n0 + 32 i +
    // acc_row(e, h)
    const float* Wo = net.params + net.w_off[net.n_hidden];
#pragma unroll
    for (int i = 0; i < NI; ++i) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int n = n0 + 32 * i + 8 * q + 4 * h;
            float4 wv[D];
#pragma unroll
            for (int d = 0; d < D; ++d) {
                const float* w = Wo + d * hp + n;
                wv[d] = make_float4(w[0], w[1], w[2], w[3]);
            }
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int e = 4 * q + t;
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const float w0 = (t == 0 ? wv[0].x : t == 1 ? wv[0].y : t == 2 ? wv[0].z : wv[0].w) * 0.5f;
                    float v = w0 * ldexpf(acc[0][i][j][e], -(eh[j] + eg[0]));
                    if (D > 1) {
                        const float w1 = (t == 0 ? wv[D - 1].x : t == 1 ? wv[D - 1].y
                                          : t == 2 ? wv[D - 1].z : wv[D - 1].w) * 0.5f;
                        v = fmaf(w1, ldexpf(acc[D - 1][i][j][e], -(eh[j] + eg[D - 1])), v);
                    }
                    out[i][j][e] = v;
                }
            }
        }
    }
}

// The NI tiles of each wave summed across the 8 waves through LDS (R slots of NI*32 x 64 floats
// in 128 KB: waves w and w + R share slot w % R, in wave order) and written as one slab tile.
// Slot layout: per 32 x 32 block (i, j) and lane, the lane's 16 accumulator values contiguous
// (16-B LDS accesses, 4 per block instead of 16 single-dword ones), the 4 chunks of a lane
// rotated by (lane >> 2) & 3 so the 8 lanes of one LDS cycle hit distinct banks. The final pass
// gives wave w the blocks w, w + 8, ...: 16 values per lane summed over the slots in slot order
// (the same order as p_0 + p_R + p_1 + ... of a row-major slot), each stored to 32 consecutive
// columns of a slab row per lane half.
template <int NI>
NAV_DEV void wgrad_reduce_write(const WgradArgs& a, int y, int split, int L, int n0, int k0,
                                const f32x16 (&acc)[NI][2], float* red) {
    constexpr int T = NI * 32 * WG_TILE;
    constexpr int R = (WG_WAVES * WG_TILE * WG_TILE) / T < WG_WAVES
                          ? (WG_WAVES * WG_TILE * WG_TILE) / T : WG_WAVES;
    const MlpDev& net = a.net[y];
    const int hp = net.hp;
    const int wv = wave_id(), lane = threadIdx.x & 63, h = lane >> 5, l32 = lane & 31;
    const int rot = (lane >> 2) & 3;
    float4* mine = reinterpret_cast<float4*>(red + (wv % R) * T);
#pragma unroll
    for (int round = 0; round < WG_WAVES / R; ++round) {
        if (wv / R == round) {
#pragma unroll
            for (int i = 0; i < NI; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    float4* p = mine + ((i * 2 + j) * 64 + lane) * 4;
#pragma unroll
                    for (int c = 0; c < 4; ++c) {
                        float4 v = make_float4(acc[i][j][4 * c], acc[i][j][4 * c + 1],
                                               acc[i][j][4 * c + 2], acc[i][j][4 * c + 3]);
                        if (round) {
                            const float4 o = p[c ^ rot];
                            v = make_float4(o.x + v.x, o.y + v.y, o.z + v.z, o.w + v.w);
                        }
                        p[c ^ rot] = v;
                    }
                }
        }
        __syncthreads();
    }
    float* o = a.slabs[y] + (int64_t)split * hidden_w_count(net) + (int64_t)(L - 1) * hp * hp;
    const float4* slots = reinterpret_cast<const float4*>(red);
    for (int b = wv; b < NI * 2; b += WG_WAVES) {
        const int i = b >> 1, j = b & 1;
        float v[16];
#pragma unroll
        for (int w = 0; w < R; ++w) {
            const float4* p = slots + (size_t)w * (T / 4) + (b * 64 + lane) * 4;
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const float4 u = p[c ^ rot];
                if (w == 0) {
                    v[4 * c] = u.x; v[4 * c + 1] = u.y; v[4 * c + 2] = u.z; v[4 * c + 3] = u.w;
                } else {
                    v[4 * c] += u.x; v[4 * c + 1] += u.y; v[4 * c + 2] += u.z; v[4 * c + 3] += u.w;
                }
            }
        }
        const int col = k0 + 32 * j + l32;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int n = n0 + 32 * i + acc_row(e, h);
            if (n < hp && col < hp) o[(int64_t)n * hp + col] = v[e];
        }
    }
}

// One workgroup's tile job: network y, hidden layer L, output tile (n0.., k0..), row split.
// Workgroups b of a grid of `total`: nets x tile jobs x splits. Block order is XCD-grouped
// (blocks b and b + 8 share an XCD's L2): the tile jobs of one (net, split) — which read the same
// rows — are consecutive in the virtual order v and land on one XCD.
struct TileJob {
    int y, job, split, L, n0, k0;
};
NAV_DEV TileJob wgrad_job(const WgradArgs& a, int b, int total) {
    const int v = (total % 8 == 0) ? (b % 8) * (total / 8) + b / 8 : b;
    const int grp = v / a.n_hid, TT = a.TT, TN = a.TN;
    TileJob t;
    t.job = v % a.n_hid;
    t.y = grp / a.splits;
    t.split = grp % a.splits;
    t.L = t.job / (TN * TT) + 1;
    t.n0 = ((t.job % (TN * TT)) / TT) * a.tn;
    t.k0 = (t.job % TT) * WG_TILE;
    return t;
}

// split s's rows for wave wv: [r_lo, r_hi). Waves w and w + 4 share a SIMD, and its arbiter
// issues the older wave first: with equal rows the second wave of every SIMD reached the LDS
// reduce ~9 k cycles after the first and ran that tail alone (profiles/r05z). `skew` rows (a
// multiple of 32: whole tiles) move from wave w + 4 to wave w, so the pair finishes together.
NAV_DEV void wave_rows(const WgradArgs& a, int split, int wv, int64_t skew, int64_t& r_lo,
                       int64_t& r_hi) {
    const int64_t M = a.M;
    const int64_t s_lo = (int64_t)split * a.per_split < M ? (int64_t)split * a.per_split : M;
    const int64_t s_hi = s_lo + a.per_split < M ? s_lo + a.per_split : M;
    const int64_t pa = a.per_wave + skew, pb = a.per_wave - skew;  // waves 0-3, 4-7
    const int64_t off = wv < WG_WAVES / 2 ? wv * pa : (WG_WAVES / 2) * pa + (wv - WG_WAVES / 2) * pb;
    const int64_t len = wv < WG_WAVES / 2 ? pa : pb;
    r_lo = s_lo + off < s_hi ? s_lo + off : s_hi;
    r_hi = r_lo + len < s_hi ? r_lo + len : s_hi;
}

template <int NI, int D>
NAV_DEV void wgrad_tile_fact(const WgradArgs& a, const TileJob& t, float* smem, uint4* tab) {
    WG_MARK(0, 0);
    // the bits -> A fragment table (a static LDS array: its address is a constant, so a fragment
    // read is one ds_read_b128 at the entry's offset): entry b, dword d holds fp16 2.0 (0x4000)
    // in its low half when bit 2d of b is set and in its high half when bit 2d + 1 is
    if (threadIdx.x < 256) {
        const uint32_t b = threadIdx.x;
        uint32_t w[4];
#pragma unroll
        for (int d = 0; d < 4; ++d)
            w[d] = ((b >> (2 * d)) & 1u ? 0x4000u : 0u) | ((b >> (2 * d + 1)) & 1u ? 0x40000000u : 0u);
        tab[b] = make_uint4(w[0], w[1], w[2], w[3]);
    }
    __syncthreads();
    WG_MARK(0, 1);
    int64_t r_lo, r_hi;
    wave_rows(a, t.split, wave_id(), a.skew, r_lo, r_hi);
    f32x16 out[NI][2];
    const char* tb = reinterpret_cast<const char*>(tab);
    const bool gv = a.ld_dy == D && ((uintptr_t)a.dy[t.y] & 15) == 0;
    const bool xv = a.net[t.y].d_in == 4 && (a.ld_in & 3) == 0 &&
                    ((uintptr_t)(a.in + a.in_col) & 15) == 0;
    if (gv && xv) wgrad_rows_fact<NI, D, true, true>(a, t.y, t.n0, t.k0, r_lo, r_hi, tb, out);
    else if (gv) wgrad_rows_fact<NI, D, true, false>(a, t.y, t.n0, t.k0, r_lo, r_hi, tb, out);
    else if (xv) wgrad_rows_fact<NI, D, false, true>(a, t.y, t.n0, t.k0, r_lo, r_hi, tb, out);
    else wgrad_rows_fact<NI, D, false, false>(a, t.y, t.n0, t.k0, r_lo, r_hi, tb, out);
    WG_MARK(0, 5);
    wgrad_reduce_write<NI>(a, t.y, t.split, t.L, t.n0, t.k0, out, smem);
    WG_MARK(0, 6);
}

// The tile job's partial over its split's rows, written as one slab tile (8 waves' partials
// summed in wave order). GEN (k_wgrad_gen, networks of >= 3 hidden layers, whose tiles never take
// the MFMA-operand path): the generic rows only, with their saved rows loaded ahead (RA)
template <bool GEN>
NAV_DEV void wgrad_tile(const WgradArgs& a, const TileJob& t, float* smem) {
    WG_MARK(1, 0);
    const int y = t.y, split = t.split, L = t.L, n0 = t.n0, k0 = t.k0;
    const int nh = a.net[y].n_hidden;
    const int wv = wave_id();
    const bool pr = L == nh - 1, qr = L == 1;
    const bool full = n0 + WG_TILE <= a.net[y].hp && k0 + WG_TILE <= a.net[y].hp;
    const bool opnd = pr && qr && full;  // the MFMA-operand path (32-row tiles: skew allowed)
    int64_t r_lo, r_hi;
    wave_rows(a, split, wv, opnd ? a.skew : 0, r_lo, r_hi);
    float* red = smem;                                          // [8][64][64]
    float* stage = smem + WG_WAVES * WG_TILE * WG_TILE + wv * 2 * WG_STAGE_FLOATS;
    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
    if constexpr (GEN) {
        if (pr && qr) wgrad_rows<true, true, true>(a, y, L, n0, k0, r_lo, r_hi, stage, acc);
        else if (pr) wgrad_rows<true, false, true>(a, y, L, n0, k0, r_lo, r_hi, stage, acc);
        else if (qr) wgrad_rows<false, true, true>(a, y, L, n0, k0, r_lo, r_hi, stage, acc);
        else wgrad_rows<false, false, true>(a, y, L, n0, k0, r_lo, r_hi, stage, acc);
    } else {
        if (opnd) wgrad_rows_mfma(a, y, n0, k0, r_lo, r_hi, acc);
        else if (pr && qr) wgrad_rows<true, true>(a, y, L, n0, k0, r_lo, r_hi, stage, acc);
        else if (pr) wgrad_rows<true, false>(a, y, L, n0, k0, r_lo, r_hi, stage, acc);
        else if (qr) wgrad_rows<false, true>(a, y, L, n0, k0, r_lo, r_hi, stage, acc);
        else wgrad_rows<false, false>(a, y, L, n0, k0, r_lo, r_hi, stage, acc);
    }
    // the 8 partial tiles meet in LDS, summed in wave order
    WG_MARK(1, 5);
    wgrad_reduce_write<2>(a, y, split, L, n0, k0, acc, red);
    WG_MARK(1, 6);
}

// grid: nets x tile jobs x splits workgroups of 8 waves (one kernel per path: each gets its own
// register allocation)
__global__ __launch_bounds__(WG_THREADS) void k_wgrad(WgradArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    wgrad_tile<false>(a, wgrad_job(a, blockIdx.x, gridDim.x), smem);
}
__global__ __launch_bounds__(WG_THREADS) void k_wgrad_gen(WgradArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    wgrad_tile<true>(a, wgrad_job(a, blockIdx.x, gridDim.x), smem);
}
template <int NI, int D>
__global__ __launch_bounds__(WG_THREADS) void k_wgrad_fact(WgradArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    __shared__ uint4 tab[256];
    wgrad_tile_fact<NI, D>(a, wgrad_job(a, blockIdx.x, gridDim.x), smem, tab);
}

// ---------------- optimizer / target update, refreshing the packed images ----------------
struct PackInfo {
    int hp, n_hidden, d_out;
    int64_t w_off[kMaxLayers];
    float* packed;
};

// The fp16 B images (mlp_common.h) of every hidden x hidden weight of up to 8 networks, rebuilt
// from the f32 parameters after each writer (Adam, Polyak, pack). One workgroup per (network,
// hidden layer, image, 16-column group): thread (c = t & 15, kq = t >> 4) holds the 16 values
// B[16 kq .. 16 kq + 15][16 g + c] in registers; the column's max |B| meets in LDS, then every
// thread writes its two 8-k entries of both planes and the kq = 0 thread the exponent e_n. The
// forward image's column n is W_L's row n (B[k][n] = W_L[n][k]: float4 reads along the row), the
// backward image's is W_L's column n (B[k][n] = W_L[k][n]: 16 lanes on 64 consecutive bytes).
// hp / 16 <= 16 k chunks: one load round trip and no second pass over W.
// For d_out = 1 the TOP hidden layer's backward image holds Wt[k][n] = Wo[k] * W_L[k][n] (f32
// products) instead of W_L: the row backward's top GEMM then takes the forward's ReLU bits as
// its exact fp16 A operand and applies dL/dq per row after the sum (mlp_kernels.hip gemm_bits).
struct PackJob {
    const float* p;
    PackInfo pk;
};
struct PackArgs {
    PackJob j[8];
    int n, per_net, cg;
};

__global__ __launch_bounds__(kBlock) void k_pack_img(PackArgs a) {
    __shared__ float cmax[16][16];
    int b = blockIdx.x;
    const int jn = b / a.per_net;
    b -= jn * a.per_net;
    const PackJob& J = a.j[jn];
    const int hp = J.pk.hp;
    const int g = b % a.cg;
    b /= a.cg;
    const int which = b & 1, L = (b >> 1) + 1;
    if (L >= J.pk.n_hidden || g * 16 >= hp) return;  // workgroup-uniform
    const float* W = J.p + J.pk.w_off[L];
    float* img = J.pk.packed + (int64_t)(L - 1) * 2 * split_image_floats(hp) +
                 which * split_image_floats(hp);
    const int c = threadIdx.x & 15, kq = threadIdx.x >> 4;
    const int n = g * 16 + c, k0 = 16 * kq;
    const bool on = k0 < hp;  // hp is a multiple of 32 (and n < hp: whole 16-column groups)
    float v[16];
    float m = 0.f;
    if (on) {
        if (which == 0) {
            const float4* r = reinterpret_cast<const float4*>(W + (int64_t)n * hp + k0);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float4 u = r[q];
                v[4 * q] = u.x; v[4 * q + 1] = u.y; v[4 * q + 2] = u.z; v[4 * q + 3] = u.w;
            }
        } else {
#pragma unroll
            for (int t = 0; t < 16; ++t) v[t] = W[(int64_t)(k0 + t) * hp + n];
            if (J.pk.d_out == 1 && L == J.pk.n_hidden - 1) {  // workgroup-uniform
                const float* Wo = J.p + J.pk.w_off[J.pk.n_hidden];
#pragma unroll
                for (int t = 0; t < 16; ++t) v[t] = Wo[k0 + t] * v[t];
            }
        }
#pragma unroll
        for (int t = 0; t < 16; ++t) m = fmaxf(m, fabsf(v[t]));
    }
    cmax[kq][c] = m;
    __syncthreads();
    if (!on) return;
#pragma unroll
    for (int q = 0; q < 16; ++q) m = fmaxf(m, cmax[q][c]);
    const int e = pow2_exp(m);
    const float sc = ldexpf(1.f, e);
    _Float16* h16 = reinterpret_cast<_Float16*>(img);
#pragma unroll
    for (int half = 0; half < 2; ++half) {
        float xs[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) xs[t] = v[8 * half + t] * sc;
        const Split2 sp = split2_8(xs);
        const int k = k0 + 8 * half;
        *reinterpret_cast<f16x8*>(h16 + split_entry(hp, 0, k, n)) = sp.h;
        *reinterpret_cast<f16x8*>(h16 + split_entry(hp, 1, k, n)) = sp.l;
    }
    if (kq == 0) reinterpret_cast<int*>(img + (int64_t)hp * hp)[n] = e;
}

NAV_DEV float adam1(float& p, float g, float& m, float& v, float b1w, float b2, float omb2,
                    float eps, float step_size, float bc2s) {
    // torch 2.10 _single_tensor_adam: m.lerp_(g, 1-b1); v.mul_(b2).addcmul_(g, g, 1-b2);
    // denom = v.sqrt()/bc2_sqrt + eps; p.addcdiv_(m, denom, -step_size)
    m = fmaf(b1w, g - m, m);
    v = v * b2 + (omb2 * g) * g;
    const float denom = sqrtf(v) / bc2s + eps;
    p = p + (-step_size) * (m / denom);
    return p;
}

// ---------------- gradient reduce (+ fused Adam) ----------------
// grad = hidden-W entries: sum of the weight-gradient split slabs (block = 64 float4 columns x 4
// split groups, the group sums added in order through LDS); every other entry: sum of the
// per-row-block edge slabs (one wave per float4, lanes take blocks b = lane, lane + 64, ..., a
// fixed xor tree adds the lanes). Deterministic: the same order on every run. With ADAM the
// finished gradient goes straight into torch's Adam update (robot.py:236-239) of the parameter
// it belongs to and the packed MFMA images are refreshed; up to 2 networks per launch.
// robot.py:293-310 soft update of up to 4 (target, source) pairs in one launch
struct PolyPair {
    float4* t;
    const float4* s;
    int64_t n4;
};
struct PolyArgs {
    PolyPair q[4];
    int n;
    int64_t total4;
    float omt, tau;
};

struct RedNet {
    MlpDev net;
    const float4* hs;
    const float4* es;
    float4* grad;  // nullable with ADAM
    float4* p;
    float4* m;
    float4* v;
    float step_size, bc2s;
    int nbh, nbe;
    float4* tgt;   // nullable: this net's target, soft-updated from the new parameters
};

struct RedArgs {
    RedNet n[2];
    int splits;
    int64_t nblk;
    float b1w, b2, omb2, eps;
    // the soft updates of the launch (robot.py:283-285): the nets' own targets in red_out, the
    // extra (target, source) pairs by the blocks past the reduce blocks
    PolyArgs poly;
    int red_blocks;
};

// Adam on the float4 of parameters at flat4 with its finished gradient g and the net's own
// target (when soft-updated in the launch); the packed images follow in k_pack_img
NAV_DEV void adam_out(const RedArgs& a, const RedNet& rn, int64_t flat4, float4 g) {
    float4 pp = rn.p[flat4], mm = rn.m[flat4], vv = rn.v[flat4];
    adam1(pp.x, g.x, mm.x, vv.x, a.b1w, a.b2, a.omb2, a.eps, rn.step_size, rn.bc2s);
    adam1(pp.y, g.y, mm.y, vv.y, a.b1w, a.b2, a.omb2, a.eps, rn.step_size, rn.bc2s);
    adam1(pp.z, g.z, mm.z, vv.z, a.b1w, a.b2, a.omb2, a.eps, rn.step_size, rn.bc2s);
    adam1(pp.w, g.w, mm.w, vv.w, a.b1w, a.b2, a.omb2, a.eps, rn.step_size, rn.bc2s);
    rn.p[flat4] = pp;
    rn.m[flat4] = mm;
    rn.v[flat4] = vv;
    if (rn.tgt) {  // robot.py:309 on the parameter just stepped (k_polyak's expression)
        float4 t = rn.tgt[flat4];
        t.x = t.x * a.poly.omt + pp.x * a.poly.tau;
        t.y = t.y * a.poly.omt + pp.y * a.poly.tau;
        t.z = t.z * a.poly.omt + pp.z * a.poly.tau;
        t.w = t.w * a.poly.omt + pp.w * a.poly.tau;
        rn.tgt[flat4] = t;
    }
}

template <bool ADAM>
NAV_DEV void red_out(const RedArgs& a, const RedNet& rn, int64_t flat4, float4 g) {
    if (rn.grad) rn.grad[flat4] = g;
    if (ADAM) adam_out(a, rn, flat4, g);
}

// soft update of element i of the pairs' concatenation (k_polyak_multi's body)
NAV_DEV void polyak_elem(const PolyArgs& a, int64_t i) {
    int64_t j = i;
    int k = 0;
    while (k < a.n - 1 && j >= a.q[k].n4) j -= a.q[k++].n4;
    const PolyPair& q = a.q[k];
    float4 t = q.t[j];
    const float4 s = q.s[j];
    // robot.py:309 target*(1-tau) + source*tau (two products, one sum)
    t.x = t.x * a.omt + s.x * a.tau;
    t.y = t.y * a.omt + s.y * a.tau;
    t.z = t.z * a.omt + s.z * a.tau;
    t.w = t.w * a.omt + s.w * a.tau;
    q.t[j] = t;
}

template <bool ADAM>
__global__ __launch_bounds__(kBlock) void k_grad_reduce(RedArgs a) {
    __shared__ float4 part[4][64];
    const int c = threadIdx.x & 63, g = threadIdx.x >> 6;
    int b = blockIdx.x;
    if (b >= a.red_blocks) {  // the extra soft-update pairs (block-uniform)
        for (int64_t i = (int64_t)(b - a.red_blocks) * kBlock + threadIdx.x; i < a.poly.total4;
             i += (int64_t)(gridDim.x - a.red_blocks) * kBlock)
            polyak_elem(a.poly, i);
        return;
    }
    const bool second = b >= a.n[0].nbh + a.n[0].nbe;
    const RedNet& rn = second ? a.n[1] : a.n[0];
    if (second) b -= a.n[0].nbh + a.n[0].nbe;
    const MlpDev& net = rn.net;
    if (b < rn.nbh) {
        const int64_t hw4 = hidden_w_count(net) / 4;
        const int64_t i = (int64_t)b * 64 + c;
        float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
        if (i < hw4) {
#pragma unroll 4
            for (int k = g; k < a.splits; k += 4) {
                const float4 v = rn.hs[(int64_t)k * hw4 + i];
                s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
            }
        }
        part[g][c] = s;
        __syncthreads();
        if (g != 0 || i >= hw4) return;
        float4 r = part[0][c];
#pragma unroll
        for (int q = 1; q < 4; ++q) {
            r.x += part[q][c].x; r.y += part[q][c].y; r.z += part[q][c].z; r.w += part[q][c].w;
        }
        const int64_t per = (int64_t)net.hp * net.hp / 4;
        const int L = (int)(i / per) + 1;
        red_out<ADAM>(a, rn, net.w_off[L] / 4 + i % per, r);
        return;
    }
    // edge entries: one block = 16 float4 columns x 16 groups of edge blocks; thread (column
    // t & 15, group t >> 4) sums blocks g, g + 16, g + 32, ... in order (a wave instruction reads
    // 4 block rows x 256 contiguous bytes), then the 16 group sums meet in group order in LDS
    const int64_t e4 = edge_count(net) / 4;
    const int ec = threadIdx.x & 15, eg = threadIdx.x >> 4;
    const int64_t o = (int64_t)(b - rn.nbh) * 16 + ec;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    if (o < e4) {
        // 16 loads in flight per trip: a thread's 32 blocks (the bench's 512 / 16 groups) in two
        // memory round trips instead of eight (the launch's critical path)
        const float4* col = rn.es + o;
        int64_t k = eg;
#pragma unroll 1
        for (; k + 240 < a.nblk; k += 256) {
            float4 v[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) v[u] = col[(k + 16 * u) * e4];
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                s.x += v[u].x; s.y += v[u].y; s.z += v[u].z; s.w += v[u].w;
            }
        }
        for (; k < a.nblk; k += 16) {
            const float4 v = col[k * e4];
            s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
        }
    }
    float4* gp = &part[0][0];  // [16 groups][16 columns]
    gp[eg * 16 + ec] = s;
    __syncthreads();
    if (eg != 0 || o >= e4) return;
    float4 r = gp[ec];
#pragma unroll
    for (int q = 1; q < 16; ++q) {
        const float4 v = gp[q * 16 + ec];
        r.x += v.x; r.y += v.y; r.z += v.z; r.w += v.w;
    }
    red_out<ADAM>(a, rn, edge_to_flat(net, 4 * o) / 4, r);
}

__global__ __launch_bounds__(kBlock) void k_adam(float4* __restrict__ p,
                                                 const float4* __restrict__ g, float4* m,
                                                 float4* v, int64_t n4, float b1w, float b2,
                                                 float omb2, float eps, float ss, float bc2s) {
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n4;
         i += (int64_t)gridDim.x * kBlock) {
        float4 pp = p[i], gg = g[i], mm = m[i], vv = v[i];
        adam1(pp.x, gg.x, mm.x, vv.x, b1w, b2, omb2, eps, ss, bc2s);
        adam1(pp.y, gg.y, mm.y, vv.y, b1w, b2, omb2, eps, ss, bc2s);
        adam1(pp.z, gg.z, mm.z, vv.z, b1w, b2, omb2, eps, ss, bc2s);
        adam1(pp.w, gg.w, mm.w, vv.w, b1w, b2, omb2, eps, ss, bc2s);
        p[i] = pp; m[i] = mm; v[i] = vv;
    }
}

// torch.optim.Adam of up to 2 networks in one launch from flat gradients that a collective
// produced (shared policy: the SUM all-reduce of the bucket); g / grad_div is the averaged
// gradient (grad_div 1: the plain step, bit-identical to k_adam). With the soft updates (a
// policy epoch, nav_adam_polyak_multi): each net's own target follows its stepped parameters
// (k_polyak's expression, as in the fused reduce), and the extra (target, source) pairs run on
// the blocks past the Adam blocks — the hook path's counterpart of nav_grad_reduce_adam_polyak.
struct AdamNet {
    float4* p;
    const float4* g;
    float4* m;
    float4* v;
    int64_t n4;
    float step_size, bc2s;
    float4* tgt;  // nullable: this net's target, soft-updated from the new parameters
};
struct AdamArgs {
    AdamNet q[2];
    int n;
    int64_t total4;
    float b1w, b2, omb2, eps, gdiv;
    PolyArgs poly;
    int adam_blocks;
};

__global__ __launch_bounds__(kBlock) void k_adam_multi(AdamArgs a) {
    if ((int)blockIdx.x >= a.adam_blocks) {  // the extra soft-update pairs (block-uniform)
        for (int64_t i = (int64_t)(blockIdx.x - a.adam_blocks) * kBlock + threadIdx.x;
             i < a.poly.total4; i += (int64_t)(gridDim.x - a.adam_blocks) * kBlock)
            polyak_elem(a.poly, i);
        return;
    }
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < a.total4;
         i += (int64_t)a.adam_blocks * kBlock) {
        const bool second = a.n > 1 && i >= a.q[0].n4;
        const AdamNet& q = second ? a.q[1] : a.q[0];
        const int64_t j = second ? i - a.q[0].n4 : i;
        float4 pp = q.p[j], gg = q.g[j], mm = q.m[j], vv = q.v[j];
        gg.x = gg.x / a.gdiv; gg.y = gg.y / a.gdiv; gg.z = gg.z / a.gdiv; gg.w = gg.w / a.gdiv;
        adam1(pp.x, gg.x, mm.x, vv.x, a.b1w, a.b2, a.omb2, a.eps, q.step_size, q.bc2s);
        adam1(pp.y, gg.y, mm.y, vv.y, a.b1w, a.b2, a.omb2, a.eps, q.step_size, q.bc2s);
        adam1(pp.z, gg.z, mm.z, vv.z, a.b1w, a.b2, a.omb2, a.eps, q.step_size, q.bc2s);
        adam1(pp.w, gg.w, mm.w, vv.w, a.b1w, a.b2, a.omb2, a.eps, q.step_size, q.bc2s);
        q.p[j] = pp; q.m[j] = mm; q.v[j] = vv;
        if (q.tgt) {  // robot.py:309 on the parameter just stepped
            float4 t = q.tgt[j];
            t.x = t.x * a.poly.omt + pp.x * a.poly.tau;
            t.y = t.y * a.poly.omt + pp.y * a.poly.tau;
            t.z = t.z * a.poly.omt + pp.z * a.poly.tau;
            t.w = t.w * a.poly.omt + pp.w * a.poly.tau;
            q.tgt[j] = t;
        }
    }
}

__global__ __launch_bounds__(kBlock) void k_polyak(float4* __restrict__ t,
                                                   const float4* __restrict__ s, int64_t n4,
                                                   float omt, float tau) {
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n4;
         i += (int64_t)gridDim.x * kBlock) {
        float4 a = t[i];
        const float4 b = s[i];
        // robot.py:309 target*(1-tau) + source*tau (two products, one sum)
        a.x = a.x * omt + b.x * tau;
        a.y = a.y * omt + b.y * tau;
        a.z = a.z * omt + b.z * tau;
        a.w = a.w * omt + b.w * tau;
        t[i] = a;
    }
}

__global__ __launch_bounds__(kBlock) void k_polyak_multi(PolyArgs a) {
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < a.total4;
         i += (int64_t)gridDim.x * kBlock)
        polyak_elem(a, i);
}

// ---------------- TD3 glue ----------------
__global__ __launch_bounds__(kBlock) void k_replay_sample(const float4* __restrict__ rows,
                                                          int64_t size, int64_t B,
                                                          const int64_t* __restrict__ idx,
                                                          uint32_t s0, uint32_t s1, uint32_t ctr,
                                                          float4* __restrict__ batch) {
    const int64_t b = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (b >= B) return;
    int64_t k;
    if (idx) {
        k = idx[b];
    } else {
        const uint4 w = philox((uint32_t)b, 0u, NAV_TAG_SAMPLE, ctr, s0, s1);
        k = (int64_t)(((uint64_t)w.x * (uint64_t)size) >> 32);
    }
    batch[2 * b] = rows[2 * k];
    batch[2 * b + 1] = rows[2 * k + 1];
}

__global__ __launch_bounds__(kBlock) void k_fill(float* x, int64_t n, float v) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n) x[i] = v;
}

__global__ __launch_bounds__(kBlock) void k_strided_copy(const float* __restrict__ src, int lds,
                                                         int cs, float* __restrict__ dst, int ldd,
                                                         int cd, int64_t rows, int cols) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= rows * cols) return;
    const int64_t r = i / cols;
    const int c = (int)(i % cols);
    dst[r * ldd + cd + c] = src[r * lds + cs + c];
}

inline int blocks_for(int64_t n) { return (int)((n + kBlock - 1) / kBlock); }
inline int grid_stride_blocks(int64_t n) {
    const int64_t b = (n + kBlock - 1) / kBlock;
    return (int)(b < 2048 ? (b > 0 ? b : 1) : 2048);
}

PackInfo pack_info(const MlpDev& d, float* packed) {
    PackInfo pk;
    pk.hp = d.hp;
    pk.n_hidden = d.n_hidden;
    pk.d_out = d.d_out;
    for (int l = 0; l < kMaxLayers; ++l) pk.w_off[l] = l <= d.n_hidden ? d.w_off[l] : 0;
    pk.packed = d.n_hidden > 1 ? packed : nullptr;
    return pk;
}

// The networks whose packed images a launch changed; launch() rebuilds them (k_pack_img) on the
// same stream right after the writer.
struct PackSet {
    PackArgs a{};
    bool add(const nav_mlp* net) {
        MlpDev d;
        if (!net || !make_dev(net, &d)) return false;
        if (d.n_hidden < 2) return true;
        if (a.n >= 8) return false;
        a.j[a.n].p = net->params;
        a.j[a.n].pk = pack_info(d, net->packed);
        ++a.n;
        return true;
    }
    int launch(hipStream_t st) {
        if (a.n == 0) return 0;
        int hp = 0, nh = 0;
        for (int i = 0; i < a.n; ++i) {
            hp = a.j[i].pk.hp > hp ? a.j[i].pk.hp : hp;
            nh = a.j[i].pk.n_hidden > nh ? a.j[i].pk.n_hidden : nh;
        }
        a.cg = (hp + 15) / 16;
        a.per_net = (nh - 1) * 2 * a.cg;
        hipLaunchKernelGGL(k_pack_img, dim3((unsigned)(a.n * a.per_net)), dim3(kBlock), 0, st, a);
        NAV_CHECK_LAUNCH();
        return 0;
    }
};

bool red_net(const nav_mlp* net, const float* hs, int splits, const float* es, float* grad,
             RedNet* rn) {
    if (!make_dev(net, &rn->net)) return false;
    if (rn->net.n_hidden > 1 && (!hs || splits < 1)) return false;
    rn->hs = reinterpret_cast<const float4*>(hs);
    rn->es = reinterpret_cast<const float4*>(es);
    rn->grad = reinterpret_cast<float4*>(grad);
    rn->nbh = (int)((hidden_w_count(rn->net) / 4 + 63) / 64);
    rn->nbe = (int)((edge_count(rn->net) / 4 + 15) / 16);
    return true;
}


}  // namespace

extern "C" {

int32_t nav_mlp_wgrad_splits(int32_t n_nets, int32_t d_out, int32_t hidden_pad, int32_t n_hidden,
                             int64_t M) {
    if (n_nets < 1 || n_nets > 2 || d_out < 1 || d_out > 2 || hidden_pad < 32 ||
        hidden_pad > 256 || (hidden_pad & 31) || n_hidden < 1 || M < 0)
        return NAV_EINVAL;
    if (n_hidden < 2) return 1;
    const int TT = (hidden_pad + WG_TILE - 1) / WG_TILE;
    const int tn = wgrad_tile_n(d_out, hidden_pad, n_hidden);
    const int TN = (hidden_pad + tn - 1) / tn;
    const int64_t jobs = (int64_t)n_nets * (n_hidden - 1) * TN * TT;
    // WG_TOTAL workgroups (256: one 8-wave workgroup per CU), at least 512 rows per split
    int64_t s = WG_TOTAL / jobs;
    const int64_t by_rows = (M + 511) / 512;
    if (s > by_rows) s = by_rows;
    return (int32_t)(s < 1 ? 1 : s);
}

static int wgrad_args(const nav_mlp* nets, int32_t n_nets, int64_t M, const float* in,
                      int32_t ld_in, int32_t in_col, const float* const* acts,
                      const float* const* dz, const float* const* dy, int32_t ld_dy,
                      const uint16_t* const* masks, float* const* slabs, int32_t splits,
                      WgradArgs& a) {
    if (!nets || n_nets < 1 || n_nets > 2 || M < 1 || splits < 1 || !in || !dy || ld_dy < 0 ||
        !masks || !slabs)
        return NAV_EINVAL;
    for (int i = 0; i < n_nets; ++i) {
        if (!make_dev(&nets[i], &a.net[i]) || !dy[i] || !masks[i] || !slabs[i]) return NAV_EINVAL;
        if (a.net[i].hp != a.net[0].hp || a.net[i].d_in != a.net[0].d_in ||
            a.net[i].n_hidden != a.net[0].n_hidden || a.net[i].d_out != a.net[0].d_out)
            return NAV_EINVAL;
        a.acts[i] = acts ? acts[i] : nullptr;
        a.dz[i] = dz ? dz[i] : nullptr;
        if (a.net[i].n_hidden > 2 && (!a.acts[i] || !a.dz[i])) return NAV_EINVAL;
        a.dy[i] = dy[i];
        a.masks[i] = masks[i];
        a.slabs[i] = slabs[i];
    }
    if (in_col < 0 || in_col + a.net[0].d_in > ld_in) return NAV_EINVAL;
    a.M = M;
    a.in = in;
    a.ld_in = ld_in;
    a.in_col = in_col;
    a.ld_dy = ld_dy;
    a.splits = splits;
    const int hp = a.net[0].hp, nh = a.net[0].n_hidden;
    a.TT = (hp + WG_TILE - 1) / WG_TILE;
    a.tn = wgrad_tile_n(a.net[0].d_out, hp, nh);
    a.TN = (hp + a.tn - 1) / a.tn;
    a.n_hid = (nh - 1) * a.TN * a.TT;
    // the factored path for the critics (d_out = 1); the actor's d_out = 2 would need two
    // accumulator sets and two splits per element (measured slower than wgrad_rows_mfma: 40 vs
    // 34 us at 2x256 on bf16, profiles/r04c; on the fp16 split 31.9 vs 25.4 us, r06r)
    a.fact = wgrad_fact_ok(hp, nh) && a.net[0].d_out == 1;
    // 32-row aligned splits and per-wave ranges: a chunk's mask row tiles start on a tile
    // boundary (at 64-row granularity a 100-row batch ran on 2 of the 8 waves: config 1's k_wgrad
    // 19.7 us, the generic path's rows loop ~30 k cycles, profiles/r06zf)
    a.per_split = ((M + splits - 1) / splits + 31) / 32 * 32;
    a.per_wave = ((a.per_split + WG_WAVES - 1) / WG_WAVES + 31) / 32 * 32;
    // whole 32-row tiles moved to the first wave of each SIMD pair, per 256 rows of a wave
    // (tools/wgrad_bench.py, profiles/r05ad_ab_wgrad_skew.txt: 0 / 32 / 64 / 96 rows for the
    // factored kernel -> 32.5 / 32.0 / 31.8 / 33.0 us, 0 / 64 / 96 / 128 for the operand path ->
    // 27.4 / 27.4 / 27.1 / 26.8 us)
    a.skew = (a.per_wave / 256) * (a.fact ? NAV_WG_SKEW_FACT : NAV_WG_SKEW_OPND);
    if ((int64_t)n_nets * a.n_hid * splits > ((int64_t)1 << 30)) return NAV_EINVAL;
    return 0;
}

int nav_mlp_wgrad(const nav_mlp* nets, int32_t n_nets, int64_t M, const float* in,
                  int32_t ld_in, int32_t in_col, const float* const* acts,
                  const float* const* dz, const float* const* dy, int32_t ld_dy,
                  const uint16_t* const* masks, float* const* slabs, int32_t splits,
                  void* stream) {
    WgradArgs a{};
    const int rc = wgrad_args(nets, n_nets, M, in, ld_in, in_col, acts, dz, dy, ld_dy, masks,
                              slabs, splits, a);
    if (rc) return rc;
    if (a.net[0].n_hidden < 2) return 0;
    const int64_t blocks = (int64_t)n_nets * a.n_hid * splits;
    // the factored kernel: its 4 KB fragment table is static, the dynamic part the reduce slots
    const size_t lds = a.fact ? (size_t)WG_WAVES * WG_TILE * WG_TILE * 4 : wgrad_lds_bytes();
    // >= 3 hidden layers: no tile is both the top and the first layer (no operand path)
    void (*k)(WgradArgs) = a.fact                  ? (a.tn == 128 ? k_wgrad_fact<4, 1> : k_wgrad_fact<2, 1>)
                           : a.net[0].n_hidden >= 3 ? k_wgrad_gen
                                                    : k_wgrad;
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(k, dim3((unsigned)blocks), dim3(WG_THREADS), lds, S(stream), a);
    NAV_CHECK_LAUNCH();
    return 0;
}

int nav_grad_reduce(const nav_mlp* net, const float* hidden_slabs, int32_t splits,
                    const float* edge_slabs, int64_t edge_blocks, float* grad, void* stream) {
    RedArgs a{};
    if (!grad || !edge_slabs || edge_blocks < 1 || splits < 0 ||
        !red_net(net, hidden_slabs, splits, edge_slabs, grad, &a.n[0]))
        return NAV_EINVAL;
    a.splits = splits;
    a.nblk = edge_blocks;
    a.red_blocks = a.n[0].nbh + a.n[0].nbe;
    hipLaunchKernelGGL(k_grad_reduce<false>, dim3((unsigned)a.red_blocks), dim3(kBlock), 0,
                       S(stream), a);
    NAV_CHECK_LAUNCH();
    return 0;
}

int nav_grad_reduce_multi(const nav_mlp* nets, int32_t n_nets, const float* const* hidden_slabs,
                          int32_t splits, const float* const* edge_slabs, int64_t edge_blocks,
                          float* const* grads, void* stream) {
    RedArgs a{};
    if (!nets || n_nets < 1 || n_nets > 2 || !hidden_slabs || !edge_slabs || edge_blocks < 1 ||
        splits < 0 || !grads)
        return NAV_EINVAL;
    int blocks = 0;
    for (int i = 0; i < n_nets; ++i) {
        if (!edge_slabs[i] || !grads[i] ||
            !red_net(&nets[i], hidden_slabs[i], splits, edge_slabs[i], grads[i], &a.n[i]))
            return NAV_EINVAL;
        if (a.n[i].net.hp != a.n[0].net.hp || a.n[i].net.n_hidden != a.n[0].net.n_hidden)
            return NAV_EINVAL;
        blocks += a.n[i].nbh + a.n[i].nbe;
    }
    a.splits = splits;
    a.nblk = edge_blocks;
    a.red_blocks = blocks;
    hipLaunchKernelGGL(k_grad_reduce<false>, dim3((unsigned)blocks), dim3(kBlock), 0, S(stream),
                       a);
    NAV_CHECK_LAUNCH();
    return 0;
}

static int adam_multi_impl(const nav_mlp* nets, int32_t n_nets, const float* const* grads,
                           float* const* m, float* const* v, float beta1, float beta2, float eps,
                           const float* step_size, const float* bc2_sqrt, float grad_div,
                           const nav_mlp* net_targets, const nav_mlp* targets,
                           const nav_mlp* sources, int32_t n_pairs, float tau, void* stream) {
    AdamArgs a{};
    PackSet ps;
    if (!nets || n_nets < 1 || n_nets > 2 || !grads || !m || !v || !step_size || !bc2_sqrt ||
        !(grad_div > 0.f) || n_pairs < 0 || n_pairs > 4 || (n_pairs && (!targets || !sources)))
        return NAV_EINVAL;
    for (int i = 0; i < n_nets; ++i) {
        MlpDev d;
        if (!make_dev(&nets[i], &d) || !grads[i] || !m[i] || !v[i]) return NAV_EINVAL;
        AdamNet& q = a.q[i];
        q.p = reinterpret_cast<float4*>(nets[i].params);
        q.g = reinterpret_cast<const float4*>(grads[i]);
        q.m = reinterpret_cast<float4*>(m[i]);
        q.v = reinterpret_cast<float4*>(v[i]);
        q.n4 = d.count / 4;
        q.step_size = step_size[i];
        q.bc2s = bc2_sqrt[i];
        if (!ps.add(&nets[i])) return NAV_EINVAL;
        if (net_targets) {
            MlpDev dt;
            if (!make_dev(&net_targets[i], &dt) || dt.count != d.count || dt.hp != d.hp ||
                dt.n_hidden != d.n_hidden || !ps.add(&net_targets[i]))
                return NAV_EINVAL;
            q.tgt = reinterpret_cast<float4*>(net_targets[i].params);
        }
        a.total4 += q.n4;
    }
    for (int i = 0; i < n_pairs; ++i) {
        MlpDev dt, ds;
        if (!make_dev(&targets[i], &dt) || !make_dev(&sources[i], &ds) || dt.count != ds.count ||
            dt.hp != ds.hp || dt.n_hidden != ds.n_hidden || !ps.add(&targets[i]))
            return NAV_EINVAL;
        a.poly.q[i].t = reinterpret_cast<float4*>(targets[i].params);
        a.poly.q[i].s = reinterpret_cast<const float4*>(sources[i].params);
        a.poly.q[i].n4 = dt.count / 4;
        a.poly.total4 += a.poly.q[i].n4;
    }
    a.poly.n = n_pairs;
    a.poly.omt = 1.0f - tau;
    a.poly.tau = tau;
    a.n = n_nets;
    a.b1w = 1.0f - beta1;
    a.b2 = beta2;
    a.omb2 = 1.0f - beta2;
    a.eps = eps;
    a.gdiv = grad_div;
    a.adam_blocks = grid_stride_blocks(a.total4);
    int blocks = a.adam_blocks;
    if (n_pairs) blocks += (int)((a.poly.total4 + kBlock - 1) / kBlock < 256
                                     ? (a.poly.total4 + kBlock - 1) / kBlock : 256);
    hipLaunchKernelGGL(k_adam_multi, dim3((unsigned)blocks), dim3(kBlock), 0, S(stream), a);
    NAV_CHECK_LAUNCH();
    return ps.launch(S(stream));
}

int nav_adam_multi(const nav_mlp* nets, int32_t n_nets, const float* const* grads,
                   float* const* m, float* const* v, float beta1, float beta2, float eps,
                   const float* step_size, const float* bc2_sqrt, float grad_div, void* stream) {
    return adam_multi_impl(nets, n_nets, grads, m, v, beta1, beta2, eps, step_size, bc2_sqrt,
                           grad_div, nullptr, nullptr, nullptr, 0, 0.f, stream);
}

int nav_adam_polyak_multi(const nav_mlp* nets, int32_t n_nets, const float* const* grads,
                          float* const* m, float* const* v, float beta1, float beta2, float eps,
                          const float* step_size, const float* bc2_sqrt, float grad_div,
                          const nav_mlp* net_targets, const nav_mlp* targets,
                          const nav_mlp* sources, int32_t n_pairs, float tau, void* stream) {
    if (!net_targets) return NAV_EINVAL;
    return adam_multi_impl(nets, n_nets, grads, m, v, beta1, beta2, eps, step_size, bc2_sqrt,
                           grad_div, net_targets, targets, sources, n_pairs, tau, stream);
}

// RedArgs of the reduce (+ Adam when m is non-NULL, + the soft updates): *blocks = the reduce
// blocks of k_grad_reduce (a.red_blocks) plus its soft-update blocks
static int red_args(const nav_mlp* nets, int32_t n_nets, const float* const* hidden_slabs,
                    int32_t splits, const float* const* edge_slabs, int64_t edge_blocks,
                    float* const* grads, float* const* m, float* const* v, float beta1,
                    float beta2, float eps, const float* step_size, const float* bc2_sqrt,
                    const nav_mlp* net_targets, const nav_mlp* targets, const nav_mlp* sources,
                    int32_t n_pairs, float tau, RedArgs& a, int* blocks_out, PackSet* ps) {
    const bool adam = m != nullptr;
    if (!nets || n_nets < 1 || n_nets > 2 || !hidden_slabs || !edge_slabs || edge_blocks < 1 ||
        splits < 0 || (adam && (!v || !step_size || !bc2_sqrt)) || n_pairs < 0 || n_pairs > 4 ||
        (n_pairs && (!targets || !sources)) || (!adam && (n_pairs || net_targets || !grads)))
        return NAV_EINVAL;
    int blocks = 0;
    for (int i = 0; i < n_nets; ++i) {
        RedNet& rn = a.n[i];
        if (!edge_slabs[i] || (adam && (!m[i] || !v[i])) || (!adam && !grads[i]) ||
            !red_net(&nets[i], hidden_slabs[i], splits, edge_slabs[i], grads ? grads[i] : nullptr,
                     &rn))
            return NAV_EINVAL;
        if (rn.net.hp != a.n[0].net.hp || rn.net.n_hidden != a.n[0].net.n_hidden)
            return NAV_EINVAL;
        if (adam) {
            rn.p = reinterpret_cast<float4*>(nets[i].params);
            rn.m = reinterpret_cast<float4*>(m[i]);
            rn.v = reinterpret_cast<float4*>(v[i]);
            rn.step_size = step_size[i];
            rn.bc2s = bc2_sqrt[i];
            if (ps && !ps->add(&nets[i])) return NAV_EINVAL;
        }
        if (net_targets) {
            MlpDev dt;
            if (!make_dev(&net_targets[i], &dt) || dt.count != rn.net.count ||
                dt.hp != rn.net.hp || dt.n_hidden != rn.net.n_hidden)
                return NAV_EINVAL;
            rn.tgt = reinterpret_cast<float4*>(net_targets[i].params);
            if (ps && !ps->add(&net_targets[i])) return NAV_EINVAL;
        }
        blocks += rn.nbh + rn.nbe;
    }
    for (int i = 0; i < n_pairs; ++i) {
        MlpDev dt, ds;
        if (!make_dev(&targets[i], &dt) || !make_dev(&sources[i], &ds) || dt.count != ds.count ||
            dt.hp != ds.hp || dt.n_hidden != ds.n_hidden)
            return NAV_EINVAL;
        a.poly.q[i].t = reinterpret_cast<float4*>(targets[i].params);
        a.poly.q[i].s = reinterpret_cast<const float4*>(sources[i].params);
        a.poly.q[i].n4 = dt.count / 4;
        if (ps && !ps->add(&targets[i])) return NAV_EINVAL;
        a.poly.total4 += a.poly.q[i].n4;
    }
    a.poly.n = n_pairs;
    a.poly.omt = 1.0f - tau;
    a.poly.tau = tau;
    a.red_blocks = blocks;
    if (n_pairs) blocks += (int)((a.poly.total4 + kBlock - 1) / kBlock < 256
                                     ? (a.poly.total4 + kBlock - 1) / kBlock : 256);
    a.splits = splits;
    a.nblk = edge_blocks;
    a.b1w = 1.0f - beta1;
    a.b2 = beta2;
    a.omb2 = 1.0f - beta2;
    a.eps = eps;
    *blocks_out = blocks;
    return 0;
}

static int grad_reduce_adam_impl(const nav_mlp* nets, int32_t n_nets, const float* const* hidden_slabs,
                          int32_t splits, const float* const* edge_slabs, int64_t edge_blocks,
                          float* const* grads, float* const* m, float* const* v, float beta1,
                          float beta2, float eps, const float* step_size, const float* bc2_sqrt,
                          const nav_mlp* net_targets, const nav_mlp* targets,
                          const nav_mlp* sources, int32_t n_pairs, float tau, void* stream) {
    RedArgs a{};
    PackSet ps;
    int blocks = 0;
    if (!m) return NAV_EINVAL;
    const int rc = red_args(nets, n_nets, hidden_slabs, splits, edge_slabs, edge_blocks, grads, m,
                            v, beta1, beta2, eps, step_size, bc2_sqrt, net_targets, targets,
                            sources, n_pairs, tau, a, &blocks, &ps);
    if (rc) return rc;
    hipLaunchKernelGGL(k_grad_reduce<true>, dim3((unsigned)blocks), dim3(kBlock), 0, S(stream),
                       a);
    NAV_CHECK_LAUNCH();
    return ps.launch(S(stream));
}

int nav_grad_reduce_adam(const nav_mlp* nets, int32_t n_nets, const float* const* hidden_slabs,
                         int32_t splits, const float* const* edge_slabs, int64_t edge_blocks,
                         float* const* grads, float* const* m, float* const* v, float beta1,
                         float beta2, float eps, const float* step_size, const float* bc2_sqrt,
                         void* stream) {
    return grad_reduce_adam_impl(nets, n_nets, hidden_slabs, splits, edge_slabs, edge_blocks,
                                 grads, m, v, beta1, beta2, eps, step_size, bc2_sqrt, nullptr,
                                 nullptr, nullptr, 0, 0.f, stream);
}

int nav_grad_reduce_adam_polyak(const nav_mlp* nets, int32_t n_nets,
                                const float* const* hidden_slabs, int32_t splits,
                                const float* const* edge_slabs, int64_t edge_blocks,
                                float* const* grads, float* const* m, float* const* v,
                                float beta1, float beta2, float eps, const float* step_size,
                                const float* bc2_sqrt, const nav_mlp* net_targets,
                                const nav_mlp* targets, const nav_mlp* sources, int32_t n_pairs,
                                float tau, void* stream) {
    if (!net_targets) return NAV_EINVAL;
    return grad_reduce_adam_impl(nets, n_nets, hidden_slabs, splits, edge_slabs, edge_blocks,
                                 grads, m, v, beta1, beta2, eps, step_size, bc2_sqrt, net_targets,
                                 targets, sources, n_pairs, tau, stream);
}

int nav_polyak_multi(const nav_mlp* targets, const nav_mlp* sources, int32_t n, float tau,
                     void* stream) {
    PolyArgs a{};
    PackSet ps;
    if (!targets || !sources || n < 1 || n > 4) return NAV_EINVAL;
    for (int i = 0; i < n; ++i) {
        MlpDev dt, ds;
        if (!make_dev(&targets[i], &dt) || !make_dev(&sources[i], &ds) || dt.count != ds.count ||
            dt.hp != ds.hp || dt.n_hidden != ds.n_hidden)
            return NAV_EINVAL;
        a.q[i].t = reinterpret_cast<float4*>(targets[i].params);
        a.q[i].s = reinterpret_cast<const float4*>(sources[i].params);
        a.q[i].n4 = dt.count / 4;
        if (!ps.add(&targets[i])) return NAV_EINVAL;
        a.total4 += a.q[i].n4;
    }
    a.n = n;
    a.omt = 1.0f - tau;
    a.tau = tau;
    hipLaunchKernelGGL(k_polyak_multi, dim3(grid_stride_blocks(a.total4)), dim3(kBlock), 0,
                       S(stream), a);
    NAV_CHECK_LAUNCH();
    return ps.launch(S(stream));
}

int nav_adam(const nav_mlp* net, const float* grad, float* m, float* v, float beta1, float beta2,
             float eps, float step_size, float bc2_sqrt, void* stream) {
    MlpDev d;
    if (!make_dev(net, &d) || !grad || !m || !v) return NAV_EINVAL;
    const int64_t n4 = d.count / 4;
    hipLaunchKernelGGL(k_adam, dim3(grid_stride_blocks(n4)), dim3(kBlock), 0, S(stream),
                       reinterpret_cast<float4*>(net->params),
                       reinterpret_cast<const float4*>(grad), reinterpret_cast<float4*>(m),
                       reinterpret_cast<float4*>(v), n4, 1.0f - beta1, beta2, 1.0f - beta2, eps,
                       step_size, bc2_sqrt);
    NAV_CHECK_LAUNCH();
    PackSet ps;
    ps.add(net);
    return ps.launch(S(stream));
}

int nav_polyak(const nav_mlp* target, const nav_mlp* source, float tau, void* stream) {
    MlpDev dt, ds;
    if (!make_dev(target, &dt) || !make_dev(source, &ds) || dt.count != ds.count ||
        dt.hp != ds.hp || dt.n_hidden != ds.n_hidden)
        return NAV_EINVAL;
    const int64_t n4 = dt.count / 4;
    hipLaunchKernelGGL(k_polyak, dim3(grid_stride_blocks(n4)), dim3(kBlock), 0, S(stream),
                       reinterpret_cast<float4*>(target->params),
                       reinterpret_cast<const float4*>(source->params), n4, 1.0f - tau, tau);
    NAV_CHECK_LAUNCH();
    PackSet ps;
    ps.add(target);
    return ps.launch(S(stream));
}

int nav_mlp_pack(const nav_mlp* net, void* stream) {
    MlpDev d;
    if (!make_dev(net, &d)) return NAV_EINVAL;
    if (d.n_hidden < 2) return 0;
    if (!net->packed) return NAV_EINVAL;
    PackSet ps;
    ps.add(net);
    return ps.launch(S(stream));
}

int nav_replay_sample(const nav_replay* replay, int64_t size, int64_t B, const int64_t* idx,
                      uint32_t seed_lo, uint32_t seed_hi, uint32_t counter, float* batch,
                      void* stream) {
    if (!replay || !replay->rows || size < 1 || size > replay->capacity ||
        size > ((int64_t)1 << 32) || B < 0 || !batch)
        return NAV_EINVAL;
    if (B == 0) return 0;
    hipLaunchKernelGGL(k_replay_sample, dim3(blocks_for(B)), dim3(kBlock), 0, S(stream),
                       reinterpret_cast<const float4*>(replay->rows), size, B, idx, seed_lo,
                       seed_hi, counter, reinterpret_cast<float4*>(batch));
    NAV_CHECK_LAUNCH();
    return 0;
}

int nav_fill(float* x, int64_t n, float value, void* stream) {
    if (n < 0 || (n && !x)) return NAV_EINVAL;
    if (n == 0) return 0;
    hipLaunchKernelGGL(k_fill, dim3(blocks_for(n)), dim3(kBlock), 0, S(stream), x, n, value);
    NAV_CHECK_LAUNCH();
    return 0;
}

int nav_strided_copy(const float* src, int32_t ld_src, int32_t col_src, float* dst,
                     int32_t ld_dst, int32_t col_dst, int64_t rows, int32_t cols, void* stream) {
    if (rows < 0 || cols < 0 || (rows && cols && (!src || !dst))) return NAV_EINVAL;
    if (rows == 0 || cols == 0) return 0;
    hipLaunchKernelGGL(k_strided_copy, dim3(blocks_for(rows * cols)), dim3(kBlock), 0, S(stream),
                       src, ld_src, col_src, dst, ld_dst, col_dst, rows, cols);
    NAV_CHECK_LAUNCH();
    return 0;
}

}  // extern "C"

#ifdef NAV_WGRAD_TRACE
extern "C" int nav_wgrad_trace_read(unsigned long long* host, int n) {
    const size_t bytes = sizeof(g_wgrad_trace);
    if (!host || (size_t)n * sizeof(unsigned long long) < bytes) return NAV_EINVAL;
    const hipError_t e = hipMemcpyFromSymbol(host, HIP_SYMBOL(g_wgrad_trace), bytes);
    return e == hipSuccess ? 0 : -(int)e;
}
#endif
