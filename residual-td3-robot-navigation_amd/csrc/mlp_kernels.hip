// mlp_kernels.hip — the residual-TD3 actor/critic MLPs (robot.py:128-206) and their learner
// (robot.py:209-398) on gfx950.
//
// Forward / row-backward: one 256-thread workgroup = 4 waves = a 128-row block kept in LDS (fp32,
// row stride hp+4 so b128 fragment reads are conflict-free) across all layers. Hidden x hidden
// layers run on v_mfma_f32_32x32x2_f32 (exact fp32): every wave owns 1-2 32-column tiles of all
// 128 rows; A fragments come from the shared LDS rows, B fragments stream from the L2-resident
// pre-packed weight image with a 2-step register prefetch, so the K loop has no barrier. The thin
// input layer (K = 2 or 4) and output layer (N = 1 or 2) run on the VALU; ReLU derivatives travel
// from forward to backward as C-layout bit masks. Weight gradients: one launch per network over
// row splits writing deterministic partial slabs, reduced in a fixed order.
#include <stdlib.h>

#include "nav_device.h"

using namespace nav;

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kMaxLayers = 9;
// workgroups hold RT row tiles of 32 rows (RT = 2 or 4; NAV_MLP_RT)

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

inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

NAV_DEV f32x16 mfma(float a, float b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

NAV_DEV int acc_row(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }

// Column tiles of a wave: wave w owns 32-column tiles t = w and w + 4 (when < NT) of every
// 128-row block, for all 4 row tiles: acc[rt][j] is the 32x32 tile (rows rt*32.., cols t_j*32..).
// Wave index as a scalar: the compiler then treats per-wave tile ownership as uniform control
// flow (s_cbranch) instead of exec-masked vector branches with pointer selects.
NAV_DEV int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

template <int NT>
struct WaveCols {
    int t0, t1;
    bool has0, has1;
    NAV_DEV WaveCols(int wv) : t0(wv), t1(wv + 4), has0(NT >= 4 || wv < NT), has1(NT >= 8 || wv + 4 < NT) {}
};

// acc[rt][j] = A[128 rows][hp] (LDS, row stride S_) x B[hp][tile t_j], B from a packed image in
// global memory [hp/4][hp][4] (element (k, n) at ((k>>2)*hp + n)*4 + (k&3)) — L2-resident, read
// once per workgroup, prefetched two K-steps ahead in registers. No barrier inside the K loop:
// the LDS rows are read-only during the product. K order inside an 8-deep step is permuted the
// same way for A and B (lane half h covers k = 8q + 4h + s at MFMA s).
template <int NT, int RT>
NAV_DEV void gemm_cols(const float* __restrict__ A, int S_, const float* __restrict__ Bp,
                       f32x16 (&acc)[RT][2]) {
    constexpr int hp = NT * 32;
    constexpr int nq = hp / 8;
    const int lane = threadIdx.x & 63, wv = wave_id(), h = lane >> 5, l32 = lane & 31;
    const WaveCols<NT> wc(wv);
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[rt][j][i] = 0.f;
    if (!wc.has0) return;  // wave-uniform (scalar) branch
    // A wave without a second tile re-reads its first tile's B (same cache lines) so every load
    // is unconditional; its second-tile MFMAs are skipped by a scalar branch.
    const int t1 = wc.has1 ? wc.t1 : wc.t0;
    const float4* B0 = reinterpret_cast<const float4*>(Bp) + (size_t)h * hp + wc.t0 * 32 + l32;
    const float4* B1 = reinterpret_cast<const float4*>(Bp) + (size_t)h * hp + t1 * 32 + l32;
    constexpr size_t STEP = 2 * (size_t)hp;  // float4 per 8-deep K step
    constexpr size_t S1 = nq > 1 ? STEP : 0;
    float4 p0 = B0[0], p1 = B0[S1];
    float4 r0 = B1[0], r1 = B1[S1];
    const float* arow = A + l32 * S_ + 4 * h;
    float4 a[RT], an[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) a[rt] = *reinterpret_cast<const float4*>(arow + rt * 32 * S_);
#pragma unroll
    for (int q = 0; q < nq; ++q) {
        const float4 c0 = p0, c1 = r0;
        p0 = p1;
        r0 = r1;
        // issue step q+2's B (L2) and step q+1's A (LDS) before step q's MFMAs; the scheduling
        // fences keep the compiler from sinking the loads next to their uses
        if (q + 2 < nq) {
            p1 = B0[(q + 2) * STEP];
            r1 = B1[(q + 2) * STEP];
        }
        if (q + 1 < nq) {
#pragma unroll
            for (int rt = 0; rt < RT; ++rt)
                an[rt] = *reinterpret_cast<const float4*>(arow + rt * 32 * S_ + 8 * (q + 1));
        }
        __builtin_amdgcn_sched_barrier(0);
#define NAV_MF(S, C)                                                                     \
    _Pragma("unroll") for (int rt = 0; rt < RT; ++rt) {                                 \
        acc[rt][0] = mfma(a[rt].S, c0.S, acc[rt][0]);                                   \
        if (NT >= 8 || wc.has1) acc[rt][1] = mfma(a[rt].S, c1.S, acc[rt][1]);           \
    }
        NAV_MF(x, 0) NAV_MF(y, 1) NAV_MF(z, 2) NAV_MF(w, 3)
#undef NAV_MF
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) a[rt] = an[rt];
    }
}

enum { IN_F32 = 0, IN_BASELINE = 1 };
enum { OUT_F32 = 0, OUT_TARGET = 1, OUT_ACT = 2 };

// ReLU masks: one 16-bit word per (row tile, column tile, lane) holding the lane's 16 C-layout
// elements' (value > 0) bits; [n_hidden][row tiles][NT][64]. The backward reads 2 bytes per 16
// elements instead of the 64 bytes of saved activations.
NAV_DEV size_t mask_idx(int64_t rowtile, int NT_, int t, int lane) {
    return ((size_t)rowtile * NT_ + t) * 64 + lane;
}

struct FwdArgs {
    MlpDev net[2];
    int64_t M;
    const float* in;
    int ld_in, in_col;
    float* out[2];
    int ld_out, out_col;
    float* acts[2];
    uint16_t* masks[2];
    // OUT_TARGET
    const float* eps;
    float policy_noise, noise_clip, max_action;
    uint32_t seed_lo, seed_hi, counter;
    // IN_BASELINE / OUT_ACT
    const double* state;
    const double* goal;
    const double* noise_scale;
    const double* noise_z;
    uint32_t step;
    int act_mode;
    double max_action_d;
    double* action_out;
};

// rows [tm][hp+4] + input/dy staging [tm][4] + output-layer partial sums [2][kBlock]
inline size_t lds_bytes(int hp, int tm) {
    return ((size_t)tm * (hp + 4) + tm * 4 + 2 * kBlock) * 4;
}

// Mask image row-tile count: independent of the workgroup height, so any RT reads what any RT
// wrote (row tile = global row / 32; layers strided by ceil(M/128)*4 tiles).
__host__ __device__ inline int64_t mask_rowtiles(int64_t M) { return ((M + 127) / 128) * 4; }

// Store a layer's C-layout result into the LDS rows (the next layer's A operand) and its ReLU
// mask bits. Global copies of the rows are written afterwards by copy_rows (coalesced).
template <int NT, int RT>
NAV_DEV void store_layer(f32x16 (&acc)[RT][2], float* act, int S_, uint16_t* mask, int64_t rt0) {
    const int lane = threadIdx.x & 63, wv = wave_id(), h = lane >> 5, l32 = lane & 31;
    const WaveCols<NT> wc(wv);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        if (!(j == 0 ? wc.has0 : wc.has1)) continue;
        const int t = j == 0 ? wc.t0 : wc.t1;
        float* col = act + t * 32 + l32 + 4 * h * S_;
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
            uint32_t bits = 0;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const float v = acc[rt][j][i];
                col[(rt * 32 + (i & 3) + 8 * (i >> 2)) * S_] = v;
                bits |= (v > 0.f ? 1u : 0u) << i;
            }
            if (mask) mask[mask_idx(rt0 + rt, NT, t, lane)] = (uint16_t)bits;
        }
    }
}

// 128 LDS rows -> global [M][hp] rows row0.., float4 per lane (1 KiB per wave instruction).
template <int NT, int RT>
NAV_DEV void copy_rows(const float* act, int S_, float* g, int64_t row0, int64_t M) {
    constexpr int hp = NT * 32, Q4 = hp / 4;
    for (int idx = threadIdx.x; idx < RT * 32 * Q4; idx += kBlock) {
        const int r = idx / Q4, c4 = idx - r * Q4;
        if (row0 + r < M)
            *reinterpret_cast<float4*>(g + (row0 + r) * hp + 4 * c4) =
                *reinterpret_cast<const float4*>(act + r * S_ + 4 * c4);
    }
}

template <int NT, int RT, int IN_MODE, int OUT_MODE>
__global__ __launch_bounds__(kBlock, 1) void k_mlp_fwd(FwdArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    constexpr int hp = NT * 32, SS = hp + 4, TM = RT * 32;
    const int tid = threadIdx.x, lane = tid & 63, wv = wave_id(), h = lane >> 5, l32 = lane & 31;
    const MlpDev& net = a.net[blockIdx.y];
    float* act_save = a.acts[blockIdx.y];
    uint16_t* masks = a.masks[blockIdx.y];
    const int64_t M = a.M;
    const int64_t row0 = (int64_t)blockIdx.x * TM;
    const int64_t rt0 = (int64_t)blockIdx.x * RT;
    const int64_t n_rt = mask_rowtiles(M);
    float* act = smem;
    float* xin = smem + TM * SS;  // [TM][4]
    const int d_in = net.d_in, d_out = net.d_out, nh = net.n_hidden;
    const WaveCols<NT> wc(wv);

    // ---- input rows -> xin
    if (tid < TM) {
        const int64_t r = row0 + tid;
        float x[4] = {0.f, 0.f, 0.f, 0.f};
        if (r < M) {
            if (IN_MODE == IN_F32) {
                const float* src = a.in + r * a.ld_in + a.in_col;
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (k < d_in) x[k] = src[k];
            } else {
                // robot.py:556 baseline = state - goal, then torch.FloatTensor (f64 -> f32)
                const double2 s = reinterpret_cast<const double2*>(a.state)[r];
                const double2 g = reinterpret_cast<const double2*>(a.goal)[r];
                x[0] = (float)(s.x - g.x);
                x[1] = (float)(s.y - g.y);
            }
        }
        *reinterpret_cast<float4*>(xin + tid * 4) = make_float4(x[0], x[1], x[2], x[3]);
    }
    __syncthreads();

    // ---- layer 0 (K = d_in) on the VALU, written in the C layout of the wave's column tiles
    {
        const float* W0 = net.params + net.w_off[0];
        const float* b0 = net.params + net.b_off[0];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            if (!(j == 0 ? wc.has0 : wc.has1)) continue;
            const int t = j == 0 ? wc.t0 : wc.t1;
            const int c = t * 32 + l32;
            float w[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (k < d_in) w[k] = W0[c * d_in + k];
            const float b = b0[c];
            float* col = act + c + 4 * h * SS;
            const float* xr = xin + 4 * h * 4;
#pragma unroll 1
            for (int rt = 0; rt < RT; ++rt) {
                uint32_t bits = 0;
                // all 16 input rows first: the LDS stores below may alias them for the compiler,
                // which would otherwise wait on every read
                float4 xs[16];
#pragma unroll
                for (int i = 0; i < 16; ++i)
                    xs[i] = *reinterpret_cast<const float4*>(xr + (rt * 32 + (i & 3) + 8 * (i >> 2)) * 4);
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const int ro = rt * 32 + (i & 3) + 8 * (i >> 2);
                    const float4 x = xs[i];
                    float v = b;
                    v = fmaf(x.x, w[0], v);
                    v = fmaf(x.y, w[1], v);
                    v = fmaf(x.z, w[2], v);
                    v = fmaf(x.w, w[3], v);
                    v = fmaxf(v, 0.f);
                    col[ro * SS] = v;
                    bits |= (v > 0.f ? 1u : 0u) << i;
                }
                if (masks) masks[mask_idx(rt0 + rt, NT, t, lane)] = (uint16_t)bits;
            }
        }
    }
    __syncthreads();
    if (act_save) copy_rows<NT, RT>(act, SS, act_save, row0, M);

    // ---- hidden x hidden layers on MFMA
    for (int L = 1; L < nh; ++L) {
        f32x16 acc[RT][2];
        gemm_cols<NT, RT>(act, SS, net.packed + (int64_t)(L - 1) * 2 * hp * hp, acc);
        const float* bL = net.params + net.b_off[L];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            if (!(j == 0 ? wc.has0 : wc.has1)) continue;
            const float b = bL[(j == 0 ? wc.t0 : wc.t1) * 32 + l32];
#pragma unroll
            for (int rt = 0; rt < RT; ++rt)
#pragma unroll
                for (int i = 0; i < 16; ++i) acc[rt][j][i] = fmaxf(acc[rt][j][i] + b, 0.f);
        }
        __syncthreads();  // every wave has finished reading the layer's input rows
        store_layer<NT, RT>(acc, act, SS, masks ? masks + (size_t)L * n_rt * NT * 64 : nullptr,
                            rt0);
        __syncthreads();
        if (act_save) copy_rows<NT, RT>(act, SS, act_save + (int64_t)L * M * hp, row0, M);
    }

    // ---- output layer (N = d_out <= 2) on the VALU: every thread takes one row and one K slice
    // of hp / PARTS; the slices' partial sums meet in LDS and add up in a fixed order
    {
        constexpr int PARTS = kBlock / TM, KP = hp / PARTS;
        const int rl = tid % TM, part = tid / TM;
        const float* ar = act + rl * SS + part * KP;
        const float* Wo = net.params + net.w_off[nh] + part * KP;
        float s0 = 0.f, s1 = 0.f;
#pragma unroll 4
        for (int k = 0; k < KP; k += 4) {
            const float4 x = *reinterpret_cast<const float4*>(ar + k);
            const float4 w0 = *reinterpret_cast<const float4*>(Wo + k);
            s0 = fmaf(x.x, w0.x, s0); s0 = fmaf(x.y, w0.y, s0);
            s0 = fmaf(x.z, w0.z, s0); s0 = fmaf(x.w, w0.w, s0);
            if (d_out > 1) {
                const float4 w1 = *reinterpret_cast<const float4*>(Wo + hp + k);
                s1 = fmaf(x.x, w1.x, s1); s1 = fmaf(x.y, w1.y, s1);
                s1 = fmaf(x.z, w1.z, s1); s1 = fmaf(x.w, w1.w, s1);
            }
        }
        float* red = xin + TM * 4;  // [2][PARTS][TM]
        red[part * TM + rl] = s0;
        red[(PARTS + part) * TM + rl] = s1;
    }
    __syncthreads();
    const int rloc = tid % TM;
    const int j = tid / TM;
    const int64_t r = row0 + rloc;
    if (r >= M || j >= d_out) return;
    float y = 0.f;
    {
        constexpr int PARTS = kBlock / TM;
        const float* red = xin + TM * 4 + j * PARTS * TM + rloc;
#pragma unroll
        for (int p = 0; p < PARTS; ++p) y += red[p * TM];
        y += net.params[net.b_off[nh] + j];
    }
    if (OUT_MODE == OUT_F32) {
        a.out[blockIdx.y][r * a.ld_out + a.out_col + j] = y;
    } else if (OUT_MODE == OUT_TARGET) {
        // robot.py:338-339 target policy smoothing
        float e;
        if (a.eps) {
            e = a.eps[r * 2 + j];
        } else {
            const double2 z = gauss_pair(philox((uint32_t)r, 0u, NAV_TAG_TNOISE, a.counter,
                                                a.seed_lo, a.seed_hi));
            e = (float)(j == 0 ? z.x : z.y);
        }
        float nz = e * a.policy_noise;
        nz = fminf(fmaxf(nz, -a.noise_clip), a.noise_clip);
        float v = y + nz;
        v = fminf(fmaxf(v, -a.max_action), a.max_action);
        a.out[blockIdx.y][r * a.ld_out + a.out_col + j] = v;
    } else {
        // robot.py:556-567 (training) / 586-593 (testing)
        const double s = a.state[r * 2 + j], g = a.goal[r * 2 + j];
        double c = (s - g) + (double)y;
        if (a.act_mode == 0) {
            double z;
            if (a.noise_z) {
                z = a.noise_z[r * 2 + j];
            } else {
                const double2 zz = gauss_pair(philox(0u, (uint32_t)r, NAV_TAG_NOISE, a.step,
                                                     a.seed_lo, a.seed_hi));
                z = j == 0 ? zz.x : zz.y;
            }
            c = c + (a.noise_scale[r] * a.max_action_d) * z;
        }
        a.action_out[r * 2 + j] = clipd(c, -a.max_action_d, a.max_action_d);
        if (a.out[0]) a.out[0][r * 2 + j] = y;
    }
}

// ---------------- row-local backward ----------------
struct BwdArgs {
    MlpDev net;
    int64_t M;
    const float* dy;
    const uint16_t* masks;
    float* dz;
    float* dx;
};

template <int NT, int RT>
NAV_DEV void mask_and_store(f32x16 (&acc)[RT][2], const uint16_t* mask, float* act, int S_,
                            int64_t rt0) {
    const int lane = threadIdx.x & 63, wv = wave_id(), h = lane >> 5, l32 = lane & 31;
    const WaveCols<NT> wc(wv);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        if (!(j == 0 ? wc.has0 : wc.has1)) continue;
        const int t = j == 0 ? wc.t0 : wc.t1;
        float* col = act + t * 32 + l32 + 4 * h * S_;
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
            const uint32_t bits = mask[mask_idx(rt0 + rt, NT, t, lane)];
#pragma unroll
            for (int i = 0; i < 16; ++i)
                col[(rt * 32 + (i & 3) + 8 * (i >> 2)) * S_] =
                    (bits >> i) & 1u ? acc[rt][j][i] : 0.f;
        }
    }
}

template <int NT, int RT>
__global__ __launch_bounds__(kBlock, 1) void k_mlp_bwd(BwdArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    constexpr int hp = NT * 32, SS = hp + 4, TM = RT * 32;
    const int tid = threadIdx.x, lane = tid & 63, wv = wave_id(), h = lane >> 5, l32 = lane & 31;
    const MlpDev& net = a.net;
    const int64_t M = a.M;
    const int64_t row0 = (int64_t)blockIdx.x * TM;
    const int64_t rt0 = (int64_t)blockIdx.x * RT;
    const int64_t n_rt = mask_rowtiles(M);
    float* act = smem;
    float* dys = smem + TM * SS;
    const int d_in = net.d_in, d_out = net.d_out, nh = net.n_hidden;
    const int64_t MH = M * hp;
    const WaveCols<NT> wc(wv);
    const size_t mstride = (size_t)n_rt * NT * 64;

    if (tid < TM) {
        const int64_t r = row0 + tid;
        float x[2] = {0.f, 0.f};
        if (r < M)
            for (int j = 0; j < d_out; ++j) x[j] = a.dy[r * d_out + j];
        *reinterpret_cast<float4*>(dys + tid * 4) = make_float4(x[0], x[1], 0.f, 0.f);
    }
    __syncthreads();

    // top hidden layer: dz = (dy . Wo) * relu'(.), in the C layout
    {
        const float* Wo = net.params + net.w_off[nh];
        const uint16_t* mk = a.masks + (size_t)(nh - 1) * mstride;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            if (!(j == 0 ? wc.has0 : wc.has1)) continue;
            const int t = j == 0 ? wc.t0 : wc.t1;
            const int c = t * 32 + l32;
            const float w0 = Wo[c];
            const float w1 = d_out > 1 ? Wo[hp + c] : 0.f;
            float* col = act + c + 4 * h * SS;
            const float* gr = dys + 4 * h * 4;
#pragma unroll 1
            for (int rt = 0; rt < RT; ++rt) {
                const uint32_t bits = mk[mask_idx(rt0 + rt, NT, t, lane)];
                float4 gs[16];
#pragma unroll
                for (int i = 0; i < 16; ++i)
                    gs[i] = *reinterpret_cast<const float4*>(gr + (rt * 32 + (i & 3) + 8 * (i >> 2)) * 4);
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const int ro = rt * 32 + (i & 3) + 8 * (i >> 2);
                    const float4 g = gs[i];
                    const float v = fmaf(g.y, w1, g.x * w0);
                    col[ro * SS] = (bits >> i) & 1u ? v : 0.f;
                }
            }
        }
    }
    __syncthreads();
    copy_rows<NT, RT>(act, SS, a.dz + (int64_t)(nh - 1) * MH, row0, M);

    // hidden layers, top-down: dz_{L-1} = (dz_L . W_L) * relu'(act_{L-1}), B = packed Wb_L
    for (int L = nh - 1; L >= 1; --L) {
        f32x16 acc[RT][2];
        gemm_cols<NT, RT>(act, SS,
                          net.packed + (int64_t)(L - 1) * 2 * hp * hp + (int64_t)hp * hp, acc);
        __syncthreads();
        mask_and_store<NT, RT>(acc, a.masks + (size_t)(L - 1) * mstride, act, SS, rt0);
        __syncthreads();
        copy_rows<NT, RT>(act, SS, a.dz + (int64_t)(L - 1) * MH, row0, M);
    }

    // dx = dz_0 . W0 : thread = (row, input pair)
    if (a.dx) {
        const float* W0 = net.params + net.w_off[0];
        const int rloc = tid % TM;
        const int64_t r = row0 + rloc;
        const float* zr = act + rloc * SS;
        for (int jj = tid / TM; jj < d_in; jj += kBlock / TM) {
            float acc = 0.f;
            for (int c = 0; c < hp; ++c) acc = fmaf(zr[c], W0[c * d_in + jj], acc);
            if (r < M) a.dx[r * d_in + jj] = acc;
        }
    }
}

// ---------------- weight gradients (split-M partial slabs) ----------------
struct WgradArgs {
    MlpDev net;
    int64_t M;
    const float* in;
    int ld_in, in_col;
    const float* acts;
    const float* dz;
    const float* dy;
    float* slabs;
    int splits;
    int T;        // 64-wide column panels across hp (edge kinds)
    int TA;       // 128-wide tiles across hp (hidden kind)
    int n_hid;    // hidden-kind jobs = (nh - 1) * TA * TA
};

constexpr int WG_MC = 32;    // rows per staged chunk
constexpr int WG_LD = 68;    // LDS row stride of the staged 64-column panels (edge kinds)
constexpr int WA_W = 128;    // hidden-kind tile width
constexpr int WA_LD = 132;   // LDS row stride of its 128-column panels

inline size_t wgrad_lds_bytes() {
    const size_t hid = (2 * 2 * WG_MC * WA_LD + 2 * WA_W) * 4;
    const size_t edge = (2 * 2 * WG_MC * WG_LD + 2 * WG_MC * 4 + 4 * 64 * 6) * 4;
    return hid > edge ? hid : edge;
}

// v if c else 0, per component (a float4-wide select would be lowered through the stack)
NAV_DEV float4 sel4(bool c, float4 v) {
    return make_float4(c ? v.x : 0.f, c ? v.y : 0.f, c ? v.z : 0.f, c ? v.w : 0.f);
}

// Hidden x hidden layer L, one 128x128 tile (tn, tk) of dW_L = dz_L^T act_{L-1} over the rows of
// one split: the 4 waves own 64x64 quadrants (2x2 v_mfma_f32_32x32x2_f32 tiles each; the MFMA K
// dimension is the row index). 32-row chunks of the two 128-column panels are double-buffered in
// LDS with the next chunk's global loads in flight during the current chunk's MFMAs. Tiles with
// tk == 0 also produce db_L = column sums of dz_L.
template <bool FULL>
NAV_DEV void wgrad_hidden(const WgradArgs& a, int job, int split, float* smem) {
    const MlpDev& net = a.net;
    const int hp = net.hp, TA = a.TA;
    const int L = job / (TA * TA) + 1;
    const int tn = (job % (TA * TA)) / TA, tk = job % TA;
    const int n0 = tn * WA_W, k0 = tk * WA_W;
    const int64_t MH = a.M * hp;
    const float* P = a.dz + (int64_t)L * MH;
    const float* Q = a.acts + (int64_t)(L - 1) * MH;
    float* Ps = smem;                          // [2][32][WA_LD]
    float* Qs = smem + 2 * WG_MC * WA_LD;      // [2][32][WA_LD]
    float* red = smem + 4 * WG_MC * WA_LD;     // [2][128]
    const int tid = threadIdx.x, lane = tid & 63, wv = wave_id(), h = lane >> 5, l32 = lane & 31;
    const int wn = 64 * (wv >> 1), wk = 64 * (wv & 1);
    // 32x32 sub-tiles inside hp (wave-uniform)
    const bool n0k = n0 + wn < hp, n1k = n0 + wn + 32 < hp;
    const bool k0k = k0 + wk < hp, k1k = k0 + wk + 32 < hp;
    const int64_t per = (a.M + a.splits - 1) / a.splits;
    const int64_t m_lo = (int64_t)split * per;
    const int64_t m_hi = m_lo + per < a.M ? m_lo + per : a.M;
    const bool colsum = tk == 0;
    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
    float cs = 0.f;  // column sum: thread = (column tid & 127, row parity tid >> 7)
    // staging: thread loads float4 (row rr, columns 4*c4..) for rr = (tid >> 5) + 8 f
    const int c4 = tid & 31, rr0 = tid >> 5;
    // loads are unconditional from clamped (valid) addresses; out-of-range values are zeroed
    // in registers, so no load sits behind a branch or a pointer select
    const bool pc_ok = n0 + 4 * c4 < hp, qc_ok = k0 + 4 * c4 < hp;
    const float* Pc = P + (pc_ok ? n0 + 4 * c4 : 0);
    const float* Qc = Q + (qc_ok ? k0 + 4 * c4 : 0);
    // (zeroing happens at store time, so nothing consumes the loads before the chunk's MFMAs)
    auto load = [&](int64_t m0, float4 (&rp)[4], float4 (&rq)[4]) {
#pragma unroll
        for (int f = 0; f < 4; ++f) {
            const int64_t m = m0 + rr0 + 8 * f;
            const int64_t mc = m < m_hi ? m : m_lo;
            rp[f] = *reinterpret_cast<const float4*>(Pc + mc * hp);
            rq[f] = *reinterpret_cast<const float4*>(Qc + mc * hp);
        }
    };
    auto store = [&](int buf, int64_t m0, const float4 (&rp)[4], const float4 (&rq)[4]) {
#pragma unroll
        for (int f = 0; f < 4; ++f) {
            const int r = rr0 + 8 * f;
            const bool ok = m0 + r < m_hi;
            *reinterpret_cast<float4*>(Ps + (buf * WG_MC + r) * WA_LD + 4 * c4) =
                sel4(ok && pc_ok, rp[f]);
            *reinterpret_cast<float4*>(Qs + (buf * WG_MC + r) * WA_LD + 4 * c4) =
                sel4(ok && qc_ok, rq[f]);
        }
    };
    float4 rp[4], rq[4];
    const int nch = (int)((m_hi - m_lo + WG_MC - 1) / WG_MC);
    if (nch > 0) {
        load(m_lo, rp, rq);
        store(0, m_lo, rp, rq);
    }
    __syncthreads();
    for (int c = 0; c < nch; ++c) {
        if (c + 1 < nch) load(m_lo + (int64_t)(c + 1) * WG_MC, rp, rq);
        const int buf = c & 1;
        const float* pb = Ps + buf * WG_MC * WA_LD;
        const float* qb = Qs + buf * WG_MC * WA_LD;
        __builtin_amdgcn_sched_barrier(0);
        if (FULL) {
            // branch-free: step s+1's operands are read before step s's 4 MFMAs (fenced so
            // the scheduler cannot sink the reads onto their uses)
            const float* pw = pb + h * WA_LD + wn + l32;
            const float* qw = qb + h * WA_LD + wk + l32;
            float a0 = pw[0], a1 = pw[32], b0 = qw[0], b1 = qw[32];
#pragma unroll
            for (int s = 0; s < WG_MC / 2; ++s) {
                float a0n = 0.f, a1n = 0.f, b0n = 0.f, b1n = 0.f;
                if (s + 1 < WG_MC / 2) {
                    const int o = 2 * (s + 1) * WA_LD;
                    a0n = pw[o];
                    a1n = pw[o + 32];
                    b0n = qw[o];
                    b1n = qw[o + 32];
                }
                __builtin_amdgcn_sched_barrier(0);
                acc[0][0] = mfma(a0, b0, acc[0][0]);
                acc[0][1] = mfma(a0, b1, acc[0][1]);
                acc[1][0] = mfma(a1, b0, acc[1][0]);
                acc[1][1] = mfma(a1, b1, acc[1][1]);
                __builtin_amdgcn_sched_barrier(0);
                a0 = a0n; a1 = a1n; b0 = b0n; b1 = b1n;
            }
        } else {
#pragma unroll
            for (int s = 0; s < WG_MC / 2; ++s) {
                const int row = 2 * s + h;
                const float a0 = pb[row * WA_LD + wn + l32], a1 = pb[row * WA_LD + wn + 32 + l32];
                const float b0 = qb[row * WA_LD + wk + l32], b1 = qb[row * WA_LD + wk + 32 + l32];
                if (n0k && k0k) acc[0][0] = mfma(a0, b0, acc[0][0]);
                if (n0k && k1k) acc[0][1] = mfma(a0, b1, acc[0][1]);
                if (n1k && k0k) acc[1][0] = mfma(a1, b0, acc[1][0]);
                if (n1k && k1k) acc[1][1] = mfma(a1, b1, acc[1][1]);
            }
        }
        if (colsum) {
#pragma unroll
            for (int r = 0; r < WG_MC / 2; ++r) cs += pb[(2 * r + (tid >> 7)) * WA_LD + (tid & 127)];
        }
        __builtin_amdgcn_sched_barrier(0);
        if (c + 1 < nch) store(buf ^ 1, m_lo + (int64_t)(c + 1) * WG_MC, rp, rq);
        __syncthreads();
    }
    float* out = a.slabs + (int64_t)split * net.count;
    float* o = out + net.w_off[L];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            if (!((i ? n1k : n0k) && (j ? k1k : k0k))) continue;
            const int nb = n0 + wn + 32 * i, kb = k0 + wk + 32 * j;
#pragma unroll
            for (int e = 0; e < 16; ++e) o[(int64_t)(nb + acc_row(e, h)) * hp + kb + l32] = acc[i][j][e];
        }
    if (!colsum) return;
    red[tid] = cs;
    __syncthreads();
    if (tid < WA_W && n0 + tid < hp) out[net.b_off[L] + n0 + tid] = red[tid] + red[WA_W + tid];
}

// Edge layers, one 64-column panel per job (VALU, K = d_in or d_out):
//  kind B (layer 0): dW_0 = dz_0^T x and db_0 = column sums of dz_0;
//  kind C (output layer): dW_o = dy^T act_top and db_o = sums of dy.
NAV_DEV void wgrad_edge(const WgradArgs& a, int job, int split, float* smem) {
    typedef float Panel[WG_MC][WG_LD];
    Panel* pa = reinterpret_cast<Panel*>(smem);                       // [2]
    float (*sm)[WG_MC][4] = reinterpret_cast<float (*)[WG_MC][4]>(smem + 2 * WG_MC * WG_LD);
    float (*red)[64][6] = reinterpret_cast<float (*)[64][6]>(smem + 2 * WG_MC * WG_LD +
                                                              2 * WG_MC * 4);
    const MlpDev& net = a.net;
    const int hp = net.hp, T = a.T, nh = net.n_hidden;
    const int kind = job < T ? 1 : 2;
    const int tcol = kind == 1 ? job : job - T;
    const int c0 = tcol * 64;
    const int64_t MH = a.M * hp;
    const float* src = kind == 1 ? a.dz : a.acts + (int64_t)(nh - 1) * MH;
    const int tid = threadIdx.x;
    const int64_t per = (a.M + a.splits - 1) / a.splits;
    const int64_t m_lo = (int64_t)split * per;
    const int64_t m_hi = m_lo + per < a.M ? m_lo + per : a.M;
    const int d_in = net.d_in, d_out = net.d_out;
    // thread = (column c = tid & 63, row group g = tid >> 6: rows g, g+4, ..)
    const int vc = tid & 63, vg = tid >> 6;
    float va[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    auto load = [&](int64_t m0, float4 (&ra)[2], float4& rs) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int i = tid + kBlock * j;
            const int rr = i >> 4, cc = (i & 15) * 4;
            const int64_t m = m0 + rr;
            ra[j] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (m < m_hi && c0 + cc < hp)
                ra[j] = *reinterpret_cast<const float4*>(src + m * hp + c0 + cc);
        }
        rs = make_float4(0.f, 0.f, 0.f, 0.f);
        if (tid < WG_MC && m0 + tid < m_hi) {
            const int64_t m = m0 + tid;
            if (kind == 1) {
                const float* x = a.in + m * a.ld_in + a.in_col;
                rs.x = x[0];
                if (d_in > 1) rs.y = x[1];
                if (d_in > 2) rs.z = x[2];
                if (d_in > 3) rs.w = x[3];
            } else {
                rs.x = a.dy[m * d_out];
                if (d_out > 1) rs.y = a.dy[m * d_out + 1];
            }
        }
    };
    auto store = [&](int buf, float4 (&ra)[2], float4 rs) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int i = tid + kBlock * j;
            const int rr = i >> 4, cc = (i & 15) * 4;
            *reinterpret_cast<float4*>(&pa[buf][rr][cc]) = ra[j];
        }
        if (tid < WG_MC) *reinterpret_cast<float4*>(&sm[buf][tid][0]) = rs;
    };
    float4 ra[2], rs;
    const int nch = (int)((m_hi - m_lo + WG_MC - 1) / WG_MC);
    if (nch > 0) {
        load(m_lo, ra, rs);
        store(0, ra, rs);
    }
    __syncthreads();
    for (int c = 0; c < nch; ++c) {
        if (c + 1 < nch) load(m_lo + (int64_t)(c + 1) * WG_MC, ra, rs);
        const int buf = c & 1;
        if (kind == 1) {
#pragma unroll
            for (int rr = vg; rr < WG_MC; rr += 4) {
                const float g = pa[buf][rr][vc];
                const float4 x = *reinterpret_cast<const float4*>(&sm[buf][rr][0]);
                va[0] = fmaf(g, x.x, va[0]);
                va[1] = fmaf(g, x.y, va[1]);
                va[2] = fmaf(g, x.z, va[2]);
                va[3] = fmaf(g, x.w, va[3]);
                va[4] += g;
            }
        } else {
#pragma unroll
            for (int rr = vg; rr < WG_MC; rr += 4) {
                const float x = pa[buf][rr][vc];
                const float4 g = *reinterpret_cast<const float4*>(&sm[buf][rr][0]);
                va[0] = fmaf(g.x, x, va[0]);
                va[1] = fmaf(g.y, x, va[1]);
                va[2] += g.x;
                va[3] += g.y;
            }
        }
        if (c + 1 < nch) store(buf ^ 1, ra, rs);
        __syncthreads();
    }
    float* out = a.slabs + (int64_t)split * net.count;
    // reduce the 4 row groups of the VALU accumulators
#pragma unroll
    for (int q = 0; q < 6; ++q) red[vg][vc][q] = va[q];
    __syncthreads();
    if (tid >= 64) return;
    float s[6];
#pragma unroll
    for (int q = 0; q < 6; ++q) s[q] = red[0][tid][q] + red[1][tid][q] + red[2][tid][q] + red[3][tid][q];
    const int n = c0 + tid;
    if (kind == 1) {
        if (n < hp) {
            for (int k = 0; k < d_in; ++k) out[net.w_off[0] + n * d_in + k] = s[k];
            out[net.b_off[0] + n] = s[4];
        }
    } else {
        if (n < hp) {
            out[net.w_off[nh] + n] = s[0];
            if (d_out > 1) out[net.w_off[nh] + hp + n] = s[1];
        }
        if (tcol == 0 && tid == 0) {
            out[net.b_off[nh]] = s[2];
            if (d_out > 1) out[net.b_off[nh] + 1] = s[3];
        }
    }
}

// One launch computes every parameter gradient of a network. The 1-D grid lists the hidden-layer
// 128x128 MFMA tiles of every row split first, then the edge panels (T layer-0 + T output) of
// every split: the dispatcher hands out the MFMA-bound blocks one per CU before the VALU/memory
// bound edge blocks fill the second slots, so the two kinds share CUs instead of stacking up.
__global__ __launch_bounds__(kBlock) void k_wgrad(WgradArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int b = blockIdx.x;
    const int n_hid_blocks = a.n_hid * a.splits;
    if (b < n_hid_blocks) {
        const int job = b % a.n_hid, split = b / a.n_hid;
        // tiles entirely inside hp take the branch-free MFMA body
        const int TA = a.TA, t = job % (TA * TA);
        const bool full = (t / TA + 1) * WA_W <= a.net.hp && (t % TA + 1) * WA_W <= a.net.hp;
        if (full)
            wgrad_hidden<true>(a, job, split, smem);
        else
            wgrad_hidden<false>(a, job, split, smem);
    } else {
        const int e = b - n_hid_blocks, ne = 2 * a.T;
        wgrad_edge(a, e % ne, e / ne, smem);
    }
}

// grad = sum of the split slabs, in a fixed order: block = 64 float4 columns x 4 split groups
// (group g sums splits g, g+4, ..), the 4 group sums added in order through LDS.
__global__ __launch_bounds__(kBlock) void k_grad_reduce(const float4* __restrict__ slabs,
                                                        int splits, int64_t n4,
                                                        float4* __restrict__ grad) {
    __shared__ float4 part[4][64];
    const int c = threadIdx.x & 63, g = threadIdx.x >> 6;
    const int64_t i = (int64_t)blockIdx.x * 64 + c;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    if (i < n4) {
#pragma unroll 4
        for (int k = g; k < splits; k += 4) {
            const float4 v = slabs[(int64_t)k * n4 + i];
            s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
        }
    }
    part[g][c] = s;
    __syncthreads();
    if (g != 0 || i >= n4) return;
    float4 r = part[0][c];
#pragma unroll
    for (int q = 1; q < 4; ++q) {
        r.x += part[q][c].x; r.y += part[q][c].y; r.z += part[q][c].z; r.w += part[q][c].w;
    }
    grad[i] = r;
}

// ---------------- optimizer / target update, refreshing the packed images ----------------
struct PackInfo {
    int hp, n_hidden;
    int64_t w_off[kMaxLayers];
    float* packed;
};

NAV_DEV void repack(const PackInfo& pk, int64_t i, float4 v) {
    // i = flat float index of v.x (multiple of 4)
    for (int L = 1; L < pk.n_hidden; ++L) {
        const int64_t off = pk.w_off[L], sz = (int64_t)pk.hp * pk.hp;
        if (i >= off && i < off + sz) {
            const int64_t e = i - off;
            const int n = (int)(e / pk.hp), k = (int)(e % pk.hp);
            float* Wf = pk.packed + (int64_t)(L - 1) * 2 * sz;
            float* Wb = Wf + sz;
            *reinterpret_cast<float4*>(Wf + ((int64_t)(k >> 2) * pk.hp + n) * 4) = v;
            float* d = Wb + ((int64_t)(n >> 2) * pk.hp + k) * 4 + (n & 3);
            d[0] = v.x; d[4] = v.y; d[8] = v.z; d[12] = v.w;
            return;
        }
    }
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

__global__ __launch_bounds__(kBlock) void k_adam(float4* __restrict__ p,
                                                 const float4* __restrict__ g, float4* m,
                                                 float4* v, int64_t n4, float b1w, float b2,
                                                 float omb2, float eps, float ss, float bc2s,
                                                 PackInfo pk) {
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n4;
         i += (int64_t)gridDim.x * kBlock) {
        float4 pp = p[i], gg = g[i], mm = m[i], vv = v[i];
        adam1(pp.x, gg.x, mm.x, vv.x, b1w, b2, omb2, eps, ss, bc2s);
        adam1(pp.y, gg.y, mm.y, vv.y, b1w, b2, omb2, eps, ss, bc2s);
        adam1(pp.z, gg.z, mm.z, vv.z, b1w, b2, omb2, eps, ss, bc2s);
        adam1(pp.w, gg.w, mm.w, vv.w, b1w, b2, omb2, eps, ss, bc2s);
        p[i] = pp; m[i] = mm; v[i] = vv;
        if (pk.packed) repack(pk, i * 4, pp);
    }
}

__global__ __launch_bounds__(kBlock) void k_polyak(float4* __restrict__ t,
                                                   const float4* __restrict__ s, int64_t n4,
                                                   float omt, float tau, PackInfo pk) {
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
        if (pk.packed) repack(pk, i * 4, a);
    }
}

__global__ __launch_bounds__(kBlock) void k_pack(const float4* __restrict__ p, int64_t n4,
                                                 PackInfo pk) {
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n4;
         i += (int64_t)gridDim.x * kBlock)
        repack(pk, i * 4, p[i]);
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

__global__ __launch_bounds__(kBlock) void k_critic_loss(int64_t B, const float* __restrict__ bt,
                                                        const float* q1t, const float* q2t,
                                                        const float* q1, const float* q2,
                                                        float gamma, float norm, float* dq1,
                                                        float* dq2, float* y_out,
                                                        float* loss_part) {
    const int64_t b = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    float l1 = 0.f, l2 = 0.f;
    if (b < B) {
        // robot.py:331-345: y = r + gamma * min(q1', q2') * (1 - done)
        const float r = bt[b * NAV_ROW + 4], d = bt[b * NAV_ROW + 7];
        const float nd = 1.0f - d;
        const float mn = fminf(q1t[b], q2t[b]);
        const float y = r + (gamma * mn) * nd;
        // torch mse_loss backward: (q - y) * (2/B)
        const float e1 = q1[b] - y, e2 = q2[b] - y;
        dq1[b] = e1 * norm;
        dq2[b] = e2 * norm;
        if (y_out) y_out[b] = y;
        l1 = e1 * e1;
        l2 = e2 * e2;
    }
    if (loss_part) {
        __shared__ float part[kBlock / 64][2];
        const float s1 = wave_sum(l1), s2 = wave_sum(l2);
        const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
        if (lane == 0) { part[wv][0] = s1; part[wv][1] = s2; }
        __syncthreads();
        if (threadIdx.x < 2) {
            float acc = 0.f;
            for (int w = 0; w < kBlock / 64; ++w) acc += part[w][threadIdx.x];
            loss_part[(int64_t)blockIdx.x * 2 + threadIdx.x] = acc;
        }
    }
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
    for (int l = 0; l < kMaxLayers; ++l) pk.w_off[l] = l <= d.n_hidden ? d.w_off[l] : 0;
    pk.packed = d.n_hidden > 1 ? packed : nullptr;
    return pk;
}

// ---- launch helpers (template dispatch on NT = hp / 32 and RT = rows / 32) ----
// Workgroup height: RT = 4 (128 rows, one workgroup per CU) or RT = 2 (64 rows, two per CU so one
// workgroup's epilogue overlaps the other's MFMA loop). NAV_MLP_RT overrides (tuning only).
int row_tiles() {
    static const int rt = [] {
        const char* e = getenv("NAV_MLP_RT");
        const int v = e ? atoi(e) : 2;
        return (v == 4) ? 4 : 2;
    }();
    return rt;
}

template <int NT, int RT, int IN_MODE, int OUT_MODE>
void launch_fwd_k(const FwdArgs& a, int n_nets, hipStream_t st) {
    const size_t lds = lds_bytes(NT * 32, RT * 32);
    auto k = k_mlp_fwd<NT, RT, IN_MODE, OUT_MODE>;
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
    const dim3 grid((unsigned)((a.M + RT * 32 - 1) / (RT * 32)), (unsigned)n_nets);
    hipLaunchKernelGGL(k, grid, dim3(kBlock), lds, st, a);
}

template <int IN_MODE, int OUT_MODE>
int launch_fwd(const FwdArgs& a, int n_nets, hipStream_t st) {
    const int rt = row_tiles();
#define NAV_FWD_CASE(NT_)                                                                    \
    case NT_:                                                                                \
        if (rt == 4) launch_fwd_k<NT_, 4, IN_MODE, OUT_MODE>(a, n_nets, st);                 \
        else launch_fwd_k<NT_, 2, IN_MODE, OUT_MODE>(a, n_nets, st);                         \
        break;
    switch (a.net[0].hp / 32) {
        NAV_FWD_CASE(1) NAV_FWD_CASE(2) NAV_FWD_CASE(3) NAV_FWD_CASE(4)
        NAV_FWD_CASE(5) NAV_FWD_CASE(6) NAV_FWD_CASE(7) NAV_FWD_CASE(8)
        default: return NAV_EINVAL;
    }
#undef NAV_FWD_CASE
    NAV_CHECK_LAUNCH();
    return 0;
}

template <int NT, int RT>
void launch_bwd_k(const BwdArgs& a, hipStream_t st) {
    const size_t lds = lds_bytes(NT * 32, RT * 32);
    auto k = k_mlp_bwd<NT, RT>;
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
    const dim3 grid((unsigned)((a.M + RT * 32 - 1) / (RT * 32)));
    hipLaunchKernelGGL(k, grid, dim3(kBlock), lds, st, a);
}

int launch_bwd(const BwdArgs& a, hipStream_t st) {
    const int rt = row_tiles();
#define NAV_BWD_CASE(NT_)                                                                    \
    case NT_:                                                                                \
        if (rt == 4) launch_bwd_k<NT_, 4>(a, st);                                            \
        else launch_bwd_k<NT_, 2>(a, st);                                                    \
        break;
    switch (a.net.hp / 32) {
        NAV_BWD_CASE(1) NAV_BWD_CASE(2) NAV_BWD_CASE(3) NAV_BWD_CASE(4)
        NAV_BWD_CASE(5) NAV_BWD_CASE(6) NAV_BWD_CASE(7) NAV_BWD_CASE(8)
        default: return NAV_EINVAL;
    }
#undef NAV_BWD_CASE
    NAV_CHECK_LAUNCH();
    return 0;
}

}  // namespace

extern "C" {

int64_t nav_mlp_param_count(int32_t d_in, int32_t d_out, int32_t hp, int32_t n_hidden) {
    nav_mlp n{d_in, d_out, hp, hp, n_hidden, reinterpret_cast<float*>(16),
              reinterpret_cast<float*>(16)};
    MlpDev d;
    if (!make_dev(&n, &d)) return NAV_EINVAL;
    return d.count;
}

int64_t nav_mlp_packed_count(int32_t hp, int32_t n_hidden) {
    if (hp < 32 || hp > 256 || (hp & 31) || n_hidden < 1) return NAV_EINVAL;
    return (int64_t)(n_hidden - 1) * 2 * hp * hp;
}

int nav_mlp_layer_offsets(const nav_mlp* net, int32_t layer, int64_t* w_off, int64_t* b_off) {
    MlpDev d;
    if (!make_dev(net, &d) || layer < 0 || layer > net->n_hidden) return NAV_EINVAL;
    if (w_off) *w_off = d.w_off[layer];
    if (b_off) *b_off = d.b_off[layer];
    return 0;
}

int nav_act(const nav_params* p, const nav_mlp* actor, int64_t n, const double* state,
            const double* goal, const double* noise_scale, const double* noise_z, uint32_t step,
            int32_t mode, double* action_out, float* residual_out, void* stream) {
    FwdArgs a{};
    if (!p || !make_dev(actor, &a.net[0]) || actor->d_in != 2 || actor->d_out != 2 || n < 0 ||
        (mode != 0 && mode != 1))
        return NAV_EINVAL;
    if (n == 0) return 0;
    if (!state || !goal || !action_out || (mode == 0 && !noise_scale)) return NAV_EINVAL;
    a.M = n;
    a.state = state;
    a.goal = goal;
    a.noise_scale = noise_scale;
    a.noise_z = noise_z;
    a.step = step;
    a.act_mode = mode;
    a.max_action_d = p->max_action;
    a.action_out = action_out;
    a.out[0] = residual_out;
    a.seed_lo = p->seed_lo;
    a.seed_hi = p->seed_hi;
    return launch_fwd<IN_BASELINE, OUT_ACT>(a, 1, S(stream));
}

int nav_mlp_forward(const nav_mlp* nets, int32_t n_nets, int64_t M, const float* in,
                    int32_t ld_in, int32_t in_col, float* const* out, int32_t ld_out,
                    int32_t out_col, int32_t out_mode, const float* eps, float policy_noise,
                    float noise_clip, float max_action, uint32_t seed_lo, uint32_t seed_hi,
                    uint32_t counter, float* const* acts, uint16_t* const* masks, void* stream) {
    FwdArgs a{};
    if (!nets || n_nets < 1 || n_nets > 2 || M < 0 || !out) return NAV_EINVAL;
    for (int i = 0; i < n_nets; ++i) {
        if (!make_dev(&nets[i], &a.net[i]) || !out[i]) return NAV_EINVAL;
        if (a.net[i].hp != a.net[0].hp || a.net[i].d_in != a.net[0].d_in) return NAV_EINVAL;
        a.out[i] = out[i];
        a.acts[i] = acts ? acts[i] : nullptr;
        a.masks[i] = masks ? masks[i] : nullptr;
    }
    if (M == 0) return 0;
    if (!in || in_col < 0 || in_col + a.net[0].d_in > ld_in || out_col < 0 ||
        out_col + a.net[0].d_out > ld_out)
        return NAV_EINVAL;
    a.M = M;
    a.in = in;
    a.ld_in = ld_in;
    a.in_col = in_col;
    a.ld_out = ld_out;
    a.out_col = out_col;
    a.eps = eps;
    a.policy_noise = policy_noise;
    a.noise_clip = noise_clip;
    a.max_action = max_action;
    a.seed_lo = seed_lo;
    a.seed_hi = seed_hi;
    a.counter = counter;
    if (out_mode == 0) return launch_fwd<IN_F32, OUT_F32>(a, n_nets, S(stream));
    if (out_mode == 1) {
        if (a.net[0].d_out != 2) return NAV_EINVAL;
        return launch_fwd<IN_F32, OUT_TARGET>(a, n_nets, S(stream));
    }
    return NAV_EINVAL;
}

int64_t nav_mlp_mask_count(int32_t hidden_pad, int32_t n_hidden, int64_t M) {
    if (hidden_pad < 32 || hidden_pad > 256 || (hidden_pad & 31) || n_hidden < 1 || M < 0)
        return NAV_EINVAL;
    return (int64_t)n_hidden * mask_rowtiles(M) * (hidden_pad / 32) * 64;
}

int nav_mlp_backward(const nav_mlp* net, int64_t M, const float* dy, const uint16_t* masks,
                     float* dz, float* dx, void* stream) {
    BwdArgs a{};
    if (!make_dev(net, &a.net) || M < 0) return NAV_EINVAL;
    if (M == 0) return 0;
    if (!dy || !masks || !dz) return NAV_EINVAL;
    a.M = M;
    a.dy = dy;
    a.masks = masks;
    a.dz = dz;
    a.dx = dx;
    return launch_bwd(a, S(stream));
}

int nav_mlp_wgrad(const nav_mlp* net, int64_t M, const float* in, int32_t ld_in, int32_t in_col,
                  const float* acts, const float* dz, const float* dy, float* slabs,
                  int32_t splits, void* stream) {
    WgradArgs a{};
    if (!make_dev(net, &a.net) || M < 1 || splits < 1 || !in || !acts || !dz || !dy || !slabs ||
        in_col < 0 || in_col + net->d_in > ld_in)
        return NAV_EINVAL;
    a.M = M;
    a.in = in;
    a.ld_in = ld_in;
    a.in_col = in_col;
    a.acts = acts;
    a.dz = dz;
    a.dy = dy;
    a.slabs = slabs;
    a.splits = splits;
    a.T = (a.net.hp + 63) / 64;
    a.TA = (a.net.hp + WA_W - 1) / WA_W;
    a.n_hid = (a.net.n_hidden - 1) * a.TA * a.TA;
    const size_t lds = wgrad_lds_bytes();
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_wgrad),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(k_wgrad, dim3((unsigned)((a.n_hid + 2 * a.T) * splits)), dim3(kBlock), lds,
                       S(stream), a);
    NAV_CHECK_LAUNCH();
    return 0;
}

int nav_grad_reduce(const float* slabs, int32_t splits, int64_t count, float* grad,
                    void* stream) {
    if (!slabs || !grad || splits < 1 || count < 0 || (count & 3)) return NAV_EINVAL;
    if (count == 0) return 0;
    const int64_t n4 = count / 4;
    hipLaunchKernelGGL(k_grad_reduce, dim3((unsigned)((n4 + 63) / 64)), dim3(kBlock), 0, S(stream),
                       reinterpret_cast<const float4*>(slabs), splits, n4,
                       reinterpret_cast<float4*>(grad));
    NAV_CHECK_LAUNCH();
    return 0;
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
                       step_size, bc2_sqrt, pack_info(d, net->packed));
    NAV_CHECK_LAUNCH();
    return 0;
}

int nav_polyak(const nav_mlp* target, const nav_mlp* source, float tau, void* stream) {
    MlpDev dt, ds;
    if (!make_dev(target, &dt) || !make_dev(source, &ds) || dt.count != ds.count ||
        dt.hp != ds.hp || dt.n_hidden != ds.n_hidden)
        return NAV_EINVAL;
    const int64_t n4 = dt.count / 4;
    hipLaunchKernelGGL(k_polyak, dim3(grid_stride_blocks(n4)), dim3(kBlock), 0, S(stream),
                       reinterpret_cast<float4*>(target->params),
                       reinterpret_cast<const float4*>(source->params), n4, 1.0f - tau, tau,
                       pack_info(dt, target->packed));
    NAV_CHECK_LAUNCH();
    return 0;
}

int nav_mlp_pack(const nav_mlp* net, void* stream) {
    MlpDev d;
    if (!make_dev(net, &d)) return NAV_EINVAL;
    if (d.n_hidden < 2) return 0;
    const int64_t n4 = d.count / 4;
    hipLaunchKernelGGL(k_pack, dim3(grid_stride_blocks(n4)), dim3(kBlock), 0, S(stream),
                       reinterpret_cast<const float4*>(net->params), n4,
                       pack_info(d, net->packed));
    NAV_CHECK_LAUNCH();
    return 0;
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

int nav_td3_critic_loss(int64_t B, const float* batch, const float* q1t, const float* q2t,
                        const float* q1, const float* q2, float gamma, float* dq1, float* dq2,
                        float* y_out, float* loss_part, void* stream) {
    if (B < 1 || !batch || !q1t || !q2t || !q1 || !q2 || !dq1 || !dq2) return NAV_EINVAL;
    const float norm = (float)(2.0 / (double)B);
    hipLaunchKernelGGL(k_critic_loss, dim3(blocks_for(B)), dim3(kBlock), 0, S(stream), B, batch,
                       q1t, q2t, q1, q2, gamma, norm, dq1, dq2, y_out, loss_part);
    NAV_CHECK_LAUNCH();
    return 0;
}

int nav_batch_sa(int64_t B, const float* batch, float* sa, void* stream) {
    return nav_strided_copy(batch, NAV_ROW, 0, sa, 4, 0, B, 4, stream);
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
