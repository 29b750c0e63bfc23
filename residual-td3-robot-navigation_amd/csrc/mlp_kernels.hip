// mlp_kernels.hip — the residual-TD3 actor/critic MLPs (robot.py:128-206) and their learner
// (robot.py:209-398) on gfx950.
//
// Forward / row-backward: one 256-thread workgroup = 4 waves = a block of 64 rows (32 for small
// batches) kept in LDS as fp32 (row stride hp+4) across all layers. Hidden x hidden layers run on
// the fp16 matrix cores (v_mfma_f32_32x32x16_f16) at f32-class accuracy: each fp32 operand is
// scaled by a power of two (A per 32-row tile, B per column) and split into two fp16 planes
// (hi + lo carries 22 significant bits), and the three products lo.hi + hi.lo + hi.hi accumulate
// in fp32 (mlp_common.h; tests/test_gpu_mlp.py pins the result against an fp64 reference at 2e-6
// of scale). Every wave owns 1-2 32-column tiles of all the block's rows; the A operand is split
// once per k step into an LDS stage shared by the 4 waves, the B operand streams from the
// L2-resident split weight image (refreshed after Adam / Polyak). The thin input layer (K = d_in
// <= 4) and the bias run on f32 MFMA (layer0_unit's fma chain bit for bit), the output layer (N =
// 1 or 2) on the VALU with a lane-transpose reduce; ReLU derivatives travel from forward to
// backward as C-layout bit masks. The cross-row weight
// gradients and the reduce + Adam are learner_kernels.hip.
#include "mlp_common.h"
#include "nav_tick.h"


namespace {

// 32-row blocks double-buffer the split stage and pass one barrier per k step (r03zt)
constexpr bool kStageDb1 = true;
// 32-row blocks split the whole layer's A once, then run the product without barriers
// (gemm_cols_whole); NAV_WHOLE1=0 restores the per-step stage (A/B)
#ifndef NAV_WHOLE1
#define NAV_WHOLE1 1
#endif
constexpr bool kWholeStage1 = NAV_WHOLE1;
// L2 warmer workgroups beside small row-kernel grids (warm_l2); NAV_WARM=0 for A/B
#ifndef NAV_WARM
#define NAV_WARM 1
#endif
[[maybe_unused]] constexpr bool kWarmL2 = NAV_WARM;
// B-fragment prefetch distance (k steps) of the 64-row GEMMs in the critic row kernel and the
// forward / tick kernels (the actor row kernel keeps 1: profiles/r05aq)
#ifndef NAV_PF_WIDE
#define NAV_PF_WIDE 2
#endif
constexpr int kPfWide = NAV_PF_WIDE;

template <int NT>
struct WaveCols {
    int t0, t1;
    bool has0, has1;
    NAV_DEV WaveCols(int wv) : t0(wv), t1(wv + 4), has0(NT >= 4 || wv < NT), has1(NT >= 8 || wv + 4 < NT) {}
};

// Per-(32-row tile, wave) max |value| slots of the block (float[RT][kWaves], just past gemm_cols'
// split stage): the epilogue that writes a GEMM's A rows into LDS publishes its values' max per
// row tile here, and gemm_cols reads them (after the epilogue's barrier) for the A operand's
// power-of-two scale of each 32-row tile. Per row tile, not per workgroup: 32- and 64-row blocks
// then scale every row identically, so the forward stays bit-identical across block heights.
template <int TM>
NAV_DEV float* amax_slots(_Float16* stage);
NAV_DEV _Float16* whole_stage(_Float16* stage);

template <int RT>
NAV_DEV void publish_amax(float* slots, const float (&m)[RT]) {
    if (!slots) return;
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
        const float v = wave_max_abs(m[rt]);
        if ((threadIdx.x & 63) == 0) slots[rt * kWaves + (threadIdx.x >> 6)] = v;
    }
}

// acc[rt][j] = A[TM rows][hp] (LDS f32, row stride S_) x B[hp][tile t_j] on the fp16 matrix
// cores at f32 accuracy (mlp_common.h: power-of-two scales, two-plane fp16 split, three
// products). Per 16-deep k step the workgroup scales and splits the step's TM x 16 A values ONCE,
// four per thread, into an LDS stage of two fp16 planes (split_stage), and every wave reads its
// 16-B fragments from there (before: each of the 4 waves split every A value it read — the split
// was ~15 % of the GEMM; probe r03v: -10 %). Two barriers per step: stage written, stage read. B is
// the layer's image (split_entry layout, per-column exponents after the planes) in global
// memory, L2-resident, its two planes loaded PF steps ahead. Lane (h, l32) holds A[row
// l32][16q + 8h + j] and B[16q + 8h + j][col l32], j = 0..7 (the 32x32x16 operand maps). Every wave
// runs the split and the barriers; waves without a column tile (NT < 4) skip only the MFMAs. The
// result is unscaled before it is returned: the callers see acc = A . B in f32.
#ifndef NAV_PF1
#define NAV_PF1 2
#endif
constexpr int kPF1 = NAV_PF1;  // B prefetch distance of 32-row blocks

// gemm_cols for 32-row blocks (small batches, latency-bound): the workgroup scales and splits
// the whole layer's 32 x hp A values into the whole-layer stage at once (two k steps per pass of
// the block, the same per-step layout and swizzle as the stage below), passes ONE barrier, and
// every wave then runs all k steps from LDS with no barrier in the product; the per-step stage
// cost a barrier + fragment-read round trip per k step (~640 cycles per step at hp = 224 vs the
// step's 6 MFMAs, profiles/r06x). Same products, same order: bit-identical to the per-step form.
template <int NT>
NAV_DEV void gemm_cols_whole(const float* __restrict__ A, int S_, const float* __restrict__ img,
                             _Float16* stage, f32x16 (&acc)[1][2]) {
    constexpr int hp = NT * 32;
    constexpr int nq = hp / 16;
    constexpr size_t PL = (size_t)nq * 2 * hp;
    constexpr size_t STEP = 2 * (size_t)hp;
    constexpr int PP = 32 * 16;  // fp16 per plane per step
    const int tid = threadIdx.x, lane = tid & 63, wv = wave_id(), h = lane >> 5, l32 = lane & 31;
    const WaveCols<NT> wc(wv);
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[0][j][i] = 0.f;
    const int t0 = wc.has0 ? wc.t0 : 0, t1 = wc.has1 ? wc.t1 : t0;
    const float* sl = amax_slots<32>(stage);
    const int ea = pow2_exp(fmaxf(fmaxf(sl[0], sl[1]), fmaxf(sl[2], sl[3])));
    const int* ex = image_exps(img, hp);
    const int eb0 = ex[t0 * 32 + l32], eb1 = ex[t1 * 32 + l32];
    const char* Bb = reinterpret_cast<const char*>(img);
    const uint32_t o0 = (uint32_t)(h * hp + t0 * 32 + l32) * 16u;
    const uint32_t o1 = (uint32_t)(h * hp + t1 * 32 + l32) * 16u;
    auto ldB = [&](uint32_t o, int p, int q) {
        return *reinterpret_cast<const f16x8*>(Bb + (o + (uint32_t)((p * PL + q * STEP) * 16)));
    };
    constexpr int PF = kPF1 < nq ? kPF1 : nq;
    f16x8 bq0[PF + 1][2], bq1[PF + 1][2];
#pragma unroll
    for (int d = 0; d < PF; ++d)
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            bq0[d][p] = ldB(o0, p, d);
            bq1[d][p] = ldB(o1, p, d);
        }
    // the split: thread (step parity qo, row sr, k offset sk) takes 4 values of steps qo, qo + 2, ..
    _Float16* const whole = whole_stage(stage);
    const int qo = tid >> 7, sr = (tid >> 2) & 31, sk = (tid & 3) * 4;
    const float* src = A + sr * S_ + sk + 16 * qo;
    _Float16* dst = whole + qo * 2 * PP + sr * 16 + ((((sk >> 3) ^ (sr >> 3)) & 1) << 3) + (sk & 7);
    const float sa = ldexpf(1.f, ea);
    float4 xs[nq / 2];
#pragma unroll
    for (int p = 0; p < nq / 2; ++p) xs[p] = *reinterpret_cast<const float4*>(src + 32 * p);
#pragma unroll
    for (int p = 0; p < nq / 2; ++p) {
        const float v[4] = {xs[p].x * sa, xs[p].y * sa, xs[p].z * sa, xs[p].w * sa};
        f16x4 ph, pl;
#pragma unroll
        for (int j = 0; j < 4; ++j) ph[j] = (_Float16)v[j];
        pin_value(ph);  // lo from the stored hi's bits (mlp_common.h)
#pragma unroll
        for (int j = 0; j < 4; ++j) pl[j] = (_Float16)(v[j] - (float)ph[j]);
        *reinterpret_cast<f16x4*>(dst + p * 4 * PP) = ph;
        *reinterpret_cast<f16x4*>(dst + p * 4 * PP + PP) = pl;
    }
    __syncthreads();
    const _Float16* frag = whole + l32 * 16 + (((h ^ (l32 >> 3)) & 1) << 3);
    auto ldA = [&](int q) {
        Split2 a;
        a.h = *reinterpret_cast<const f16x8*>(frag + q * 2 * PP);
        a.l = *reinterpret_cast<const f16x8*>(frag + q * 2 * PP + PP);
        return a;
    };
    Split2 af = ldA(0);
#pragma unroll
    for (int q = 0; q < nq; ++q) {
        if (q + PF < nq) {
#pragma unroll
            for (int p = 0; p < 2; ++p) {
                bq0[(q + PF) % (PF + 1)][p] = ldB(o0, p, q + PF);
                bq1[(q + PF) % (PF + 1)][p] = ldB(o1, p, q + PF);
            }
        }
        Split2 an;
        if (q + 1 < nq) an = ldA(q + 1);
        if (wc.has0) {  // wave-uniform
            acc[0][0] = mfma_x3(af, bq0[q % (PF + 1)], acc[0][0]);
            if (NT >= 8 || wc.has1) acc[0][1] = mfma_x3(af, bq1[q % (PF + 1)], acc[0][1]);
        }
        if (q + 1 < nq) af = an;
        // a scheduling fence per k step (as in gemm_bits): without a barrier in the loop the
        // scheduler sinks the prefetched loads down to their uses
        __builtin_amdgcn_sched_barrier(0);
    }
    const int u0 = -(ea + eb0), u1 = -(ea + eb1);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        acc[0][0][i] = ldexpf(acc[0][0][i], u0);
        acc[0][1][i] = ldexpf(acc[0][1][i], u1);
    }
}

template <int NT, int RT, int PFB = 1>
NAV_DEV void gemm_cols(const float* __restrict__ A, int S_, const float* __restrict__ img,
                       _Float16* stage, f32x16 (&acc)[RT][2]) {
    if constexpr (RT == 1 && kWholeStage1) {
        gemm_cols_whole<NT>(A, S_, img, stage, acc);
        return;
    }
    constexpr int hp = NT * 32;
    constexpr int nq = hp / 16;
    constexpr int TM = RT * 32;
    constexpr size_t PL = (size_t)nq * 2 * hp;  // 16-B entries per plane
    constexpr size_t STEP = 2 * (size_t)hp;     // entries per k step
    constexpr int PP = TM * 16;                 // fp16 per stage plane
    const int tid = threadIdx.x, lane = tid & 63, wv = wave_id(), h = lane >> 5, l32 = lane & 31;
    const WaveCols<NT> wc(wv);
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[rt][j][i] = 0.f;
    // A wave without a second tile re-reads its first tile's B (same cache lines) so every load
    // is unconditional; its second-tile MFMAs are skipped by a scalar branch (a wave without any
    // tile reads tile 0's and issues none).
    const int t0 = wc.has0 ? wc.t0 : 0, t1 = wc.has1 ? wc.t1 : t0;
    // the scales: A's per 32-row tile from the producing epilogue's published maxima, B's per
    // column (in flight under the whole product)
    const float* slots = amax_slots<TM>(stage);
    int ea[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
        const float* sl = slots + rt * kWaves;
        ea[rt] = pow2_exp(fmaxf(fmaxf(sl[0], sl[1]), fmaxf(sl[2], sl[3])));
    }
    const int* ex = image_exps(img, hp);
    const int eb0 = ex[t0 * 32 + l32], eb1 = ex[t1 * 32 + l32];
    // B entries as the uniform image base + a 32-bit per-lane byte offset (SGPR base + VGPR
    // offset addressing: one 32-bit add per load instead of a 64-bit address pair)
    const char* Bb = reinterpret_cast<const char*>(img);
    const uint32_t o0 = (uint32_t)(h * hp + t0 * 32 + l32) * 16u;
    const uint32_t o1 = (uint32_t)(h * hp + t1 * 32 + l32) * 16u;
    auto ldB = [&](uint32_t o, int p, int q) {
        return *reinterpret_cast<const f16x8*>(Bb + (o + (uint32_t)((p * PL + q * STEP) * 16)));
    };
    // B planes PF steps ahead: one step for 64-row blocks (the register budget of the big row
    // kernels), two for 32-row blocks, whose step (6 MFMAs per wave) is shorter than an L2 hit
    // B prefetch distance in k steps: 64-row blocks take the caller's PFB (2 in the critic row
    // kernel and the forward / tick launches, 1 in the 256-register actor row kernel, where a
    // second step of B fragments costs more than it hides: profiles/r05ap)
    constexpr int PF = RT == 1 ? kPF1 : PFB;
    f16x8 bq0[PF + 1][2], bq1[PF + 1][2];
#pragma unroll
    for (int d = 0; d < PF; ++d)
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            const int qd = d < nq ? d : nq - 1;
            bq0[d][p] = ldB(o0, p, qd);
            bq1[d][p] = ldB(o1, p, qd);
        }
    // this thread's share of a step: 4 values of row sr at k offset sk; the stage's two 16-B
    // halves of row r are swapped when (r >> 3) & 1, which makes both the 8-B stores and the
    // waves' 16-B fragment reads bank-conflict-free (ds_read_b128 lane groups). With 64 rows
    // every thread has a share (no branch: the split sits in the MFMAs' basic block)
    const bool sp = TM * 4 >= kBlock || tid < TM * 4;
    const int sr = tid >> 2, sk = (tid & 3) * 4;
    const float* src = A + sr * S_ + sk;
    _Float16* dst = stage + sr * 16 + ((((sk >> 3) ^ (sr >> 3)) & 1) << 3) + (sk & 7);
    const _Float16* frag = stage + l32 * 16 + (((h ^ (l32 >> 3)) & 1) << 3);
    float4 x = sp ? *reinterpret_cast<const float4*>(src) : make_float4(0.f, 0.f, 0.f, 0.f);
    const float sa = ldexpf(1.f, RT == 1 ? ea[0] : ea[(sr >> 5) < RT ? (sr >> 5) : RT - 1]);
    // scale + split of step q's share (x) into the stage, the next x from the LDS rows, B planes
    // ahead. 32-row blocks (small batches: latency-bound, one wave per SIMD) double-buffer the
    // stage and pass one barrier per step: step q + 1's stores go to the buffer step q - 1 was
    // read from, which every wave finished reading (and consumed in its MFMAs) before step q's
    // barrier
    constexpr bool DB = RT == 1 && kStageDb1;
    constexpr int SB = 2 * PP;  // fp16 per stage buffer
    auto produce = [&](int q) {
        if (sp) {
            _Float16* const dq = dst + (DB ? (q & 1) * SB : 0);
            const float v[4] = {x.x * sa, x.y * sa, x.z * sa, x.w * sa};
            f16x4 ph, pl;
#pragma unroll
            for (int j = 0; j < 4; ++j) ph[j] = (_Float16)v[j];
            pin_value(ph);  // lo from the stored hi's bits (mlp_common.h)
#pragma unroll
            for (int j = 0; j < 4; ++j) pl[j] = (_Float16)(v[j] - (float)ph[j]);
            *reinterpret_cast<f16x4*>(dq) = ph;
            *reinterpret_cast<f16x4*>(dq + PP) = pl;
            if (q + 1 < nq) x = *reinterpret_cast<const float4*>(src + 16 * (q + 1));
        }
        // production of step q runs during step q - 1's MFMAs: the B planes loaded here are
        // step q - 1 + PF's (steps 0 .. PF - 1 come from the prologue)
        const int qb = q - 1 + PF;
        if (q >= 1 && qb < nq) {
#pragma unroll
            for (int p = 0; p < 2; ++p) {
                bq0[qb % (PF + 1)][p] = ldB(o0, p, qb);
                bq1[qb % (PF + 1)][p] = ldB(o1, p, qb);
            }
        }
    };
    Split2 sa2[RT];
    // two barriers per step (one buffer): the stage is written, then read (the next step may
    // overwrite it); one barrier with the double buffer
    auto consume = [&](int q) {
        __syncthreads();
        const _Float16* fq = frag + (DB ? (q & 1) * SB : 0);
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
            const _Float16* f = fq + rt * 32 * 16;
            sa2[rt].h = *reinterpret_cast<const f16x8*>(f);
            sa2[rt].l = *reinterpret_cast<const f16x8*>(f + PP);
        }
        if (!DB) __syncthreads();
    };
    produce(0);
    consume(0);
    // Two workgroups share a CU at the bench shapes (blocks b and b + kCUs, dispatched together),
    // and at equal priority the SIMD arbiter issues the older wave first: the second workgroup's
    // GEMMs lag and it ends its last ~50 k cycles alone at the lone-workgroup MFMA rate (critic_rows:
    // 247 k vs 297 k cycles). The younger partner of each pair (odd multiples of kCUs) raises its
    // wave priority inside its GEMMs, which balances the pair (270 k / 267 k; critic_rows 161.6 ->
    // 153.5 us, profiles/r04y, r04z). At a 512-block grid this is the grid's upper half.
    const bool favored = (blockIdx.x / kCUs) & 1;
    if (favored) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int q = 0; q < nq; ++q) {
        // step q + 1's production comes first in program order, so the scheduler can place it
        // between step q's MFMAs (its stage stores follow step q's second barrier)
        if (q + 1 < nq) produce(q + 1);
        Split2 cur[RT];
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) cur[rt] = sa2[rt];
        if (wc.has0) {  // wave-uniform
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) {
                acc[rt][0] = mfma_x3(cur[rt], bq0[q % (PF + 1)], acc[rt][0]);
                if (NT >= 8 || wc.has1)
                    acc[rt][1] = mfma_x3(cur[rt], bq1[q % (PF + 1)], acc[rt][1]);
            }
        }
        if (q + 1 < nq) consume(q + 1);
    }
    if (favored) __builtin_amdgcn_s_setprio(0);
    // unscale: acc 2^-(ea[rt] + e_n), exact (v_ldexp_f32)
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
        const int u0 = -(ea[rt] + eb0), u1 = -(ea[rt] + eb1);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            acc[rt][0][i] = ldexpf(acc[rt][0][i], u0);
            acc[rt][1][i] = ldexpf(acc[rt][1][i], u1);
        }
    }
}

// ---- the top hidden layer's row backward of a d_out = 1 network on its ReLU bits ----
// dz_{L-1}[r][c] = e_{L-1}[r][c] * sum_n dz_L[r][n] W_L[n][c] with dz_L[r][n] = e_L[r][n] g[r]
// Wo[n] (g = dL/dq, e = the forward's ReLU bits) is g[r] * sum_n e_L[r][n] Wt[n][c], Wt[n][c] =
// Wo[n] W_L[n][c]: the A operand is the bit matrix itself, exact in fp16 (0 / 1.0), so only B (the
// Wt image, k_pack_img) is split and each k step takes 2 products instead of 3; no A rows, no
// split stage, no barrier in the product. The bits come row-major from LDS: word w of row r holds
// e_L[r][32 w .. 32 w + 31] (bits_stage), one byte per lane and k step picks a 16-B fragment of
// the 256-entry table of 8 fp16 zeros / ones.
constexpr int kBitTab = 256 * 4;  // floats of the fragment table (256 x 16 B)
// LDS words per row of the bit image: NT + 1 (odd: the 32 lanes of a half read 32 rows without a
// bank conflict)
template <int NT>
constexpr int bit_ws() { return NT + 1; }

// The fragment table (entry b: fp16 bit j of b at element j) and the bit image of the lanes'
// C-layout mask words (mb[rt][j]: bit i = row c_row(rt, i, h), column t_j * 32 + l32) into the
// scratch at `scr` (tab [256][4] u32, then bits [TM][bit_ws] u32, then g [TM]). One ballot per
// (row tile, column tile, C element) yields a row's word for the wave's column tile (lanes h = 0:
// row +0, h = 1: row +4); writelane parks it at the row's lane, lanes 0-31 carry the first tile
// and 32-63 the second, and one store per row tile writes both.
// lane ^ M_ across the wave: DPP moves inside 16-lane rows for M_ <= 8 (out_partials, bits_stage)
template <int M_>
NAV_DEV float lane_xor(float v) {
    const int x = __float_as_int(v);
    if constexpr (M_ == 1) {
        return __int_as_float(__builtin_amdgcn_mov_dpp(x, 0xB1, 0xF, 0xF, false));  // [1,0,3,2]
    } else if constexpr (M_ == 2) {
        return __int_as_float(__builtin_amdgcn_mov_dpp(x, 0x4E, 0xF, 0xF, false));  // [2,3,0,1]
    } else if constexpr (M_ == 4) {
        const int m7 = __builtin_amdgcn_mov_dpp(x, 0x141, 0xF, 0xF, false);  // l ^ 7
        return __int_as_float(__builtin_amdgcn_mov_dpp(m7, 0x1B, 0xF, 0xF, false));  // ^ 3
    } else if constexpr (M_ == 8) {
        return __int_as_float(__builtin_amdgcn_mov_dpp(x, 0x128, 0xF, 0xF, false));  // ror 8
    } else {
        return __shfl_xor(v, M_, 64);
    }
}

// one stage of the 32 x 32 bit transpose: lanes l and l ^ S swap the off-diagonal S x S blocks
// (lane_xor: DPP row moves for S <= 8, one ds_bpermute for 16)
template <int S>
NAV_DEV uint32_t bfly_stage(uint32_t x, int lane, uint32_t m) {
    const uint32_t y = __float_as_uint(lane_xor<S>(__uint_as_float(x)));
    return (lane & S) ? (((y >> S) & m) | (x & ~m)) : ((x & m) | ((y & m) << S));
}

template <int NT, int RT>
NAV_DEV void bits_stage(float* scr, const uint32_t (&mb)[RT][2], const float* dys) {
    constexpr int TM = RT * 32, WS = bit_ws<NT>();
    const int tid = threadIdx.x, lane = tid & 63;
    const WaveCols<NT> wc(wave_id());
    static_assert((kBitTab + TM * WS + TM) * 4 <= TM * (NT * 32 + 4) * 4,
                  "the bit scratch fits in the block's LDS rows");
    uint32_t* tab = reinterpret_cast<uint32_t*>(scr);
    uint32_t* bw = tab + kBitTab;
    float* gq = reinterpret_cast<float*>(bw + TM * WS);
    {
        const uint32_t b = (uint32_t)tid;  // kBlock = 256 entries
        uint4 e;
        e.x = ((b & 1u) ? 0x3C00u : 0u) | ((b & 2u) ? 0x3C000000u : 0u);
        e.y = ((b & 4u) ? 0x3C00u : 0u) | ((b & 8u) ? 0x3C000000u : 0u);
        e.z = ((b & 16u) ? 0x3C00u : 0u) | ((b & 32u) ? 0x3C000000u : 0u);
        e.w = ((b & 64u) ? 0x3C00u : 0u) | ((b & 128u) ? 0x3C000000u : 0u);
        reinterpret_cast<uint4*>(tab)[tid] = e;
    }
    if (tid < TM) gq[tid] = dys[tid * 4];
    // per row tile: lanes 0-31 build the column words of the wave's first tile, lanes 32-63 of
    // its second (one exchange across the halves: lane (h, l32) holds rows +4h of both), then a
    // 32 x 32 bit transpose inside each half (5 butterfly exchanges) leaves row l32's word of its
    // half's tile in lane l32. VGPR shuffles only: a ballot form (v_cmp to an SGPR pair, selects
    // on it) gave timing-dependent words in the older workgroup of a co-resident pair
    // (tools/dbg_bits.py, profiles/r06g).
    const int h = lane >> 5;
    auto spread = [](uint32_t w) {  // nibble k of a 16-bit word -> bits 8k .. 8k + 3
        return (w & 0xFu) | ((w & 0xF0u) << 4) | ((w & 0xF00u) << 8) | ((w & 0xF000u) << 12);
    };
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
        const uint32_t send = h ? mb[rt][0] : mb[rt][1];
        const uint32_t recv = (uint32_t)__shfl_xor((int)send, 32, 64);
        const uint32_t w0 = h ? recv : mb[rt][0], w1 = h ? mb[rt][1] : recv;
        // bit r of x = E[rt * 32 + r][column (tile h) * 32 + l32]
        uint32_t x = spread(w0) | (spread(w1) << 4);
        x = bfly_stage<16>(x, lane, 0x0000FFFFu);
        x = bfly_stage<8>(x, lane, 0x00FF00FFu);
        x = bfly_stage<4>(x, lane, 0x0F0F0F0Fu);
        x = bfly_stage<2>(x, lane, 0x33333333u);
        x = bfly_stage<1>(x, lane, 0x55555555u);
        if (h == 0 ? wc.has0 : wc.has1)
            bw[(rt * 32 + (lane & 31)) * WS + (h == 0 ? wc.t0 : wc.t1)] = x;
    }
}

// acc[rt][j] = g[row] * (E[TM rows][hp] (bit image) x Wt[hp][tile t_j]) from bits_stage's
// scratch and the Wt image (B planes PF steps ahead as in gemm_cols; the A fragments one step
// ahead). Unscaled and multiplied by g[row] before it returns.
template <int NT, int RT, int PFB = 1>
NAV_DEV void gemm_bits(const float* scr, const float* __restrict__ img, f32x16 (&acc)[RT][2]) {
    constexpr int hp = NT * 32;
    constexpr int nq = hp / 16;
    constexpr int TM = RT * 32, WS = bit_ws<NT>();
    constexpr size_t PL = (size_t)nq * 2 * hp;
    constexpr size_t STEP = 2 * (size_t)hp;
    const int lane = threadIdx.x & 63, wv = wave_id(), h = lane >> 5, l32 = lane & 31;
    const WaveCols<NT> wc(wv);
    const uint4* tab = reinterpret_cast<const uint4*>(scr);
    const uint32_t* bw = reinterpret_cast<const uint32_t*>(scr) + kBitTab;
    const float* gq = reinterpret_cast<const float*>(bw + TM * WS);
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[rt][j][i] = 0.f;
    // the zero accumulators as registers: folded into an inline-constant C operand, the first
    // product's untied destination was allocated over its own B fragment, and the results came
    // out timing-dependent (a few rows per launch; tools/dbg_bits.py, profiles/r06d)
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int j = 0; j < 2; ++j) pin_value(acc[rt][j]);
    const int t0 = wc.has0 ? wc.t0 : 0, t1 = wc.has1 ? wc.t1 : t0;
    const int* ex = image_exps(img, hp);
    const int eb0 = ex[t0 * 32 + l32], eb1 = ex[t1 * 32 + l32];
    const char* Bb = reinterpret_cast<const char*>(img);
    const uint32_t o0 = (uint32_t)(h * hp + t0 * 32 + l32) * 16u;
    const uint32_t o1 = (uint32_t)(h * hp + t1 * 32 + l32) * 16u;
    auto ldB = [&](uint32_t o, int p, int q) {
        return *reinterpret_cast<const f16x8*>(Bb + (o + (uint32_t)((p * PL + q * STEP) * 16)));
    };
    // B prefetch distance in k steps as gemm_cols
    constexpr int PF = RT == 1 ? kPF1 : PFB;
    f16x8 bq0[PF + 1][2], bq1[PF + 1][2];
#pragma unroll
    for (int d = 0; d < PF; ++d)
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            const int qd = d < nq ? d : nq - 1;
            bq0[d][p] = ldB(o0, p, qd);
            bq1[d][p] = ldB(o1, p, qd);
        }
    // the lane's row words (row rt * 32 + l32; word q / 2 covers k steps q, q + 1) and the A
    // fragment of step q: byte 2 (q & 1) + h of word q / 2
    const uint32_t* wrow = bw + l32 * WS;
    uint32_t w[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) w[rt] = wrow[rt * 32 * WS];
    auto frag = [&](int q, int rt) {
        const uint32_t byte = (w[rt] >> (16 * (q & 1) + 8 * h)) & 0xFFu;
        // (fragments built by VALU from the byte instead: neutral, r06r)
        return __builtin_bit_cast(f16x8, tab[byte]);
    };
    f16x8 af[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) af[rt] = frag(0, rt);
    const bool favored = (blockIdx.x / kCUs) & 1;  // gemm_cols' co-resident balance
    if (favored) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int q = 0; q < nq; ++q) {
        // step q + 1's operands first in program order (in flight under step q's MFMAs)
        const int qb = q + PF;
        if (qb < nq) {
#pragma unroll
            for (int p = 0; p < 2; ++p) {
                bq0[qb % (PF + 1)][p] = ldB(o0, p, qb);
                bq1[qb % (PF + 1)][p] = ldB(o1, p, qb);
            }
        }
        f16x8 an[RT];
        if (q + 1 < nq) {
            if ((q & 1) == 1) {
#pragma unroll
                for (int rt = 0; rt < RT; ++rt) w[rt] = wrow[rt * 32 * WS + ((q + 1) >> 1)];
            }
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) an[rt] = frag(q + 1, rt);
        }
        if (wc.has0) {  // wave-uniform
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) {
                const f16x8(&b0)[2] = bq0[q % (PF + 1)];
                acc[rt][0] = mfma_h(af[rt], b0[1], acc[rt][0]);
                acc[rt][0] = mfma_h(af[rt], b0[0], acc[rt][0]);
                if (NT >= 8 || wc.has1) {
                    const f16x8(&b1)[2] = bq1[q % (PF + 1)];
                    acc[rt][1] = mfma_h(af[rt], b1[1], acc[rt][1]);
                    acc[rt][1] = mfma_h(af[rt], b1[0], acc[rt][1]);
                }
            }
        }
        if (q + 1 < nq) {
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) af[rt] = an[rt];
        }
        // a scheduling fence per k step: without a barrier in the loop the scheduler would sink
        // the prefetched loads down to their uses (a full L2 / LDS round trip exposed per step)
        __builtin_amdgcn_sched_barrier(0);
    }
    if (favored) __builtin_amdgcn_s_setprio(0);
    // unscale 2^-e_n (exact), then dL/dq of the element's row, in place one group of 4 rows at
    // a time (fenced: hoisting every g load and keeping the unscaled copies beside the
    // accumulators pushed the row kernels past 256 registers, one workgroup per CU)
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const float4 g = *reinterpret_cast<const float4*>(gq + rt * 32 + 8 * m + 4 * h);
            const float gv[4] = {g.x, g.y, g.z, g.w};
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int i = 4 * m + u;
                acc[rt][0][i] = ldexpf(acc[rt][0][i], -eb0) * gv[u];
                acc[rt][1][i] = ldexpf(acc[rt][1][i], -eb1) * gv[u];
            }
            __builtin_amdgcn_sched_barrier(0);
        }
}

// the fp16 B images of hidden layer L (1 .. n_hidden-1): forward (B[k][n] = W_L[n][k]) and
// backward (B[k][n] = W_L[k][n]; for d_out = 1 the top layer's is Wo[k] W_L[k][n], gemm_bits)
NAV_DEV const float* img_fwd(const MlpDev& net, int L) {
    return net.packed + (int64_t)(L - 1) * 2 * split_image_floats(net.hp);
}
NAV_DEV const float* img_bwd(const MlpDev& net, int L) {
    return net.packed + (int64_t)(L - 1) * 2 * split_image_floats(net.hp) + split_image_floats(net.hp);
}

enum { IN_F32 = 0, IN_BASELINE = 1 };
enum { OUT_F32 = 0, OUT_TARGET = 1, OUT_ACT = 2, OUT_LOSS = 3, OUT_TICK = 4 };


struct FwdArgs {
    MlpDev net[2];
    int64_t M;
    const float* in;
    int ld_in, in_col;
    float* out[2];
    int ld_out, out_col;
    float* acts[2];
    uint32_t save_mask;  // bit L: hidden layer L's output rows are copied to acts + L*M*hp
    uint16_t* masks[2];
    // OUT_LOSS: train_critic's online twin forward with the TD error and the output layer's
    // gradient partials (robot.py:341-361)
    const float* batch;  // [M][8] replay rows (r at 4, done at 7)
    const float* qt[2];  // target twin values q1', q2' [M]
    float gamma, norm;   // discount, 2/B (mse_loss backward)
    float* dq[2];        // [M] dL/dq
    float* loss_part[2]; // [blocks] sum of (q - y)^2 over the block's rows
    float* eslab[2];     // [blocks][edge_count]: Wo / bo partials (nullable)
    int64_t ecount;
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
    // OUT_TICK: the training tick of every row's env with the action just formed (one launch:
    // nav_act + nav_agent_step(_indexed); nav_act_tick)
    nav_params p;
    nav_env_soa env;
    const float2* field;
    float4* rows;
    int64_t cap, base;
    nav_step_out sout;
    DemoIdx demo;
    double* reward_out;
};

// Output-layer partial sums: [d_out <= 2][4 waves][TM rows] (red_floats per block).
__host__ __device__ constexpr int red_floats(int tm) { return 2 * kWaves * tm; }

// bytes of gemm_cols' split stage for TM rows: [2 planes][TM][16] fp16 (two buffers for 32-row
// blocks), then the kWaves amax slots
__host__ __device__ constexpr size_t stage_halves(int tm) {
    return (size_t)(tm == 32 && kStageDb1 ? 2 : 1) * 2 * tm * 16;
}
// 32-row blocks also take the whole-layer stage past the slots (gemm_cols_whole): [hp / 16 k
// steps][2 planes][32][16] fp16, hp * 128 bytes
__host__ __device__ constexpr size_t stage_bytes(int tm, int hp) {
    return stage_halves(tm) * 2 + 4 * kWaves * (tm / 32) +
           (tm == 32 && kWholeStage1 ? (size_t)hp * 128 : 0);
}
template <int TM>
NAV_DEV float* amax_slots(_Float16* stage) {
    return reinterpret_cast<float*>(stage + stage_halves(TM));
}
NAV_DEV _Float16* whole_stage(_Float16* stage) {
    return stage + stage_halves(32) + 2 * kWaves;  // past the 32-row block's 4 slots (16 B)
}

// rows [tm][hp+4] + input/dy staging [tm][4] + output-layer partial sums, then the split stage
__host__ __device__ constexpr size_t lds_floats(int hp, int tm) {
    return (size_t)tm * (hp + 4) + tm * 4 + red_floats(tm);
}
inline size_t lds_bytes(int hp, int tm) { return lds_floats(hp, tm) * 4 + stage_bytes(tm, hp); }


// Store a layer's C-layout result into the LDS rows (the next layer's A operand) and its ReLU
// mask bits; with slots, publish the rows' max |value| for the next GEMM's A scale. Global copies
// of the rows are written afterwards by copy_rows (coalesced).
template <int NT, int RT>
NAV_DEV void store_layer(f32x16 (&acc)[RT][2], float* act, int S_, uint16_t* mask, int64_t rt0,
                         float* slots = nullptr) {
    const int lane = threadIdx.x & 63, wv = wave_id(), h = lane >> 5, l32 = lane & 31;
    const WaveCols<NT> wc(wv);
    float m[RT] = {};
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
                bits |= pos_bit(v) << i;
                m[rt] = max_nn(m[rt], v);  // post-ReLU: v >= 0
            }
            if (mask) mask[mask_idx(rt0 + rt, NT, t, lane)] = (uint16_t)bits;
        }
    }
    publish_amax(slots, m);
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

// Edge partials over the block's TM LDS rows, one thread per column n < hp, rows summed in order.
template <int TM>
NAV_DEV void edge_col_sums(const float* act, int S_, int hp, float* out) {
    const int n = threadIdx.x;
    if (n >= hp) return;
    float s = 0.f;
#pragma unroll 8
    for (int r = 0; r < TM; ++r) s += act[r * S_ + n];
    out[n] = s;
}

// dW0 partial: out[n*d_in + k] = sum_r dz0[r][n] * x[r][k]
template <int TM>
NAV_DEV void edge_w0(const float* act, int S_, int hp, const float* xin, int d_in, float* out) {
    const int n = threadIdx.x;
    if (n >= hp) return;
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
#pragma unroll 8
    for (int r = 0; r < TM; ++r) {
        const float g = act[r * S_ + n];
        const float4 x = *reinterpret_cast<const float4*>(xin + 4 * r);
        s0 = fmaf(g, x.x, s0);
        s1 = fmaf(g, x.y, s1);
        s2 = fmaf(g, x.z, s2);
        s3 = fmaf(g, x.w, s3);
    }
    out[n * d_in] = s0;
    if (d_in > 1) out[n * d_in + 1] = s1;
    if (d_in > 2) out[n * d_in + 2] = s2;
    if (d_in > 3) out[n * d_in + 3] = s3;
}

// output j of block row rloc from fwd_net's per-wave partial sums, added in wave order
template <int RT>
NAV_DEV float out_y(const MlpDev& net, const float* red, int rloc, int j) {
    constexpr int TM = RT * 32;
    float y = 0.f;
#pragma unroll
    for (int p = 0; p < kWaves; ++p) y += red[(j * kWaves + p) * TM + rloc];
    return y + net.params[net.b_off[net.n_hidden] + j];
}

// Block row of C-layout element i of row tile rt in lane half h.
NAV_DEV int c_row(int rt, int i, int h) { return rt * 32 + (i & 3) + 8 * (i >> 2) + 4 * h; }

// ReLU mask words of a layer from its C-layout registers (store_layer's bits without the rows).
template <int NT, int RT>
NAV_DEV void store_mask(const f32x16 (&acc)[RT][2], uint16_t* mask, int64_t rt0) {
    const int lane = threadIdx.x & 63;
    const WaveCols<NT> wc(wave_id());
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        if (!(j == 0 ? wc.has0 : wc.has1)) continue;
        const int t = j == 0 ? wc.t0 : wc.t1;
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
            uint32_t bits = 0;
#pragma unroll
            for (int i = 0; i < 16; ++i) bits |= pos_bit(acc[rt][j][i]) << i;  // post-ReLU
            mask[mask_idx(rt0 + rt, NT, t, lane)] = (uint16_t)bits;
        }
    }
}

// Output layer (N = d_out <= 2) straight from the top hidden layer's C-layout registers: every
// lane forms, per block row it holds, the dot product of its (up to) 2 columns with Wo; a
// transpose-reduce across the 32 lanes of each lane half (5 xor exchanges that each halve the
// list a lane carries: 31 exchanges for RT = 2) sums the columns of the wave; the 4 waves'
// partials meet in LDS (red [d_out][4][TM]) and out_y adds them in wave order. No LDS copy of the
// top layer, no barrier between the last GEMM and the output layer. The exchanges run in lane-
// mask order 1, 2, 4, 8, 16, so the big early stages are DPP moves inside a 16-lane row (xor 1 /
// 2: quad_perm, xor 4: half-row mirror then quad_perm, xor 8: row rotate by 8) and only the last,
// single-element one crosses rows (ds_bpermute).

// one halving stage of the transpose-reduce: lanes with bit M_ set keep the upper half of the
// list (n entries) and send the lower half to lane ^ M_
template <int M_, int N_>
NAV_DEV void halve(float* v, int l32) {
    const uint32_t um = (l32 & M_) ? 0xffffffffu : 0u;
    // bitwise selects: a ?: over the list would be turned into a dynamic array index
#pragma unroll
    for (int k = 0; k < N_ / 2; ++k) {
        const uint32_t lo = __float_as_uint(v[k]), hi = __float_as_uint(v[k + N_ / 2]);
        const float send = __uint_as_float((lo & um) | (hi & ~um));
        const float keep = __uint_as_float((hi & um) | (lo & ~um));
        v[k] = keep + lane_xor<M_>(send);
    }
}
// Wo entries of the lane's columns (0 for absent tiles): wo[output][tile]
struct WoCols {
    float w[2][2];
};
template <int NT>
NAV_DEV WoCols load_wo(const MlpDev& net) {
    constexpr int hp = NT * 32;
    const int l32 = threadIdx.x & 31;
    const WaveCols<NT> wc(wave_id());
    const float* Wo = net.params + net.w_off[net.n_hidden];
    const int c0 = wc.t0 * 32 + l32, c1 = (wc.has1 ? wc.t1 : wc.t0) * 32 + l32;
    WoCols r;
#pragma unroll
    for (int jo = 0; jo < 2; ++jo) {
        const bool on = jo < net.d_out;
        r.w[jo][0] = on && wc.has0 ? Wo[jo * hp + c0] : 0.f;
        r.w[jo][1] = on && wc.has1 ? Wo[jo * hp + c1] : 0.f;
    }
    return r;
}

template <int NT, int RT>
NAV_DEV void out_partials(const MlpDev& net, const f32x16 (&top)[RT][2], const WoCols& wo,
                          float* red) {
    // RT = 2 (V = 32): after the 5 halvings lane l32 holds list element bitrev5(l32). RT = 1
    // (V = 16): four halvings leave lanes l32 and l32 ^ 16 with the two halves of element
    // bitrev4(l32 & 15); the fifth exchange adds them and the lane with bit 4 clear writes
    static_assert(RT == 1 || RT == 2, "row tiles per workgroup");
    constexpr int TM = RT * 32, V = RT * 16;
    const int lane = threadIdx.x & 63, wv = wave_id(), h = lane >> 5, l32 = lane & 31;
#pragma unroll
    for (int jo = 0; jo < 2; ++jo) {
        if (jo >= net.d_out) break;
        const float w0 = wo.w[jo][0], w1 = wo.w[jo][1];
        float v[V];
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
            for (int i = 0; i < 16; ++i) v[rt * 16 + i] = fmaf(top[rt][1][i], w1, top[rt][0][i] * w0);
        // lane bit b (mask 16 .. 1) picks which half of the list the lane keeps: the survivor k
        // of lane l32 is list element (l32 * KEEP + k)
        halve<1, V>(v, l32);
        halve<2, V / 2>(v, l32);
        halve<4, V / 4>(v, l32);
        halve<8, V / 8>(v, l32);
        if constexpr (V >= 32) {
            halve<16, V / 16>(v, l32);
            const int e = (int)(__builtin_bitreverse32((uint32_t)l32) >> 27);
            red[(jo * kWaves + wv) * TM + c_row(e >> 4, e & 15, h)] = v[0];
        } else {
            v[0] += lane_xor<16>(v[0]);
            if ((l32 & 16) == 0) {
                const int e = (int)(__builtin_bitreverse32((uint32_t)l32) >> 28);
                red[(jo * kWaves + wv) * TM + c_row(0, e, h)] = v[0];
            }
        }
    }
}

// Output-layer weight-gradient partials dWo[jo][c] = sum_rows g[row][jo] * h_top[row][c] of the
// block, straight from the top layer's C-layout registers (g = dL/dy rows in LDS, row stride
// gstride): each lane sums its 16 * RT rows of its columns in (row tile, element) order, then
// the two lane halves (rows +0 / +4) meet by one exchange. bwd_net's h_top path (rows from
// global memory) adds in the same order, so both give the same bits.
template <int NT, int RT>
NAV_DEV void wo_grad_regs(const MlpDev& net, const f32x16 (&top)[RT][2], const float* g,
                          int gstride, float* es) {
    const int lane = threadIdx.x & 63, h = lane >> 5, l32 = lane & 31;
    const WaveCols<NT> wc(wave_id());
#pragma unroll
    for (int jo = 0; jo < 2; ++jo) {
        if (jo >= net.d_out) break;
        float s0 = 0.f, s1 = 0.f;
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const float gv = g[c_row(rt, i, h) * gstride + jo];
                s0 = fmaf(gv, top[rt][0][i], s0);
                s1 = fmaf(gv, top[rt][1][i], s1);
            }
        s0 += __shfl_xor(s0, 32, 64);
        s1 += __shfl_xor(s1, 32, 64);
        if (h == 0) {
            float* o = es + e_wo(net) + jo * net.hp;
            if (wc.has0) o[wc.t0 * 32 + l32] = s0;
            if (wc.has1) o[wc.t1 * 32 + l32] = s1;
        }
    }
}

// OUT_LOSS (d_out = 1): q from the output-layer partials against the TD target yt of the thread's
// row (robot.py:341-345, from the caller), mse_loss's gradient dq = (q - yt) * 2/B, the block's
// sum of (q - y)^2, and the output layer's gradient partials dWo = dq^T h_top, dbo = sum dq while
// h_top is still in LDS. `red` = the [2][PARTS][TM] partial-sum scratch (second half reused).
template <int NT, int RT>
NAV_DEV void loss_epilogue(const MlpDev& net, const f32x16 (&top)[RT][2], float* red,
                           int64_t row0, int64_t M, float yt, float norm, float* dq,
                           float* loss_slot, float* es) {
    constexpr int TM = RT * 32;
    const int tid = threadIdx.x;
    const int64_t r = row0 + tid;
    float dqv = 0.f, e2 = 0.f;
    if (tid < TM && r < M) {
        const float y = out_y<RT>(net, red, tid, 0);
        const float e = y - yt;
        dqv = e * norm;
        e2 = e * e;
        dq[r] = dqv;
    }
    float* dqs = red + kWaves * TM;  // [TM] dq (past output 0's partials), then the wave sums
    float* ws = dqs + TM;
    if (tid < TM) dqs[tid] = dqv;
    const float w = wave_sum(e2);
    if ((tid & 63) == 0) ws[tid >> 6] = w;
    __syncthreads();
    if (tid == 0) {
        float sum = 0.f;
#pragma unroll
        for (int k = 0; k < kBlock / 64; ++k) sum += ws[k];
        *loss_slot = sum;
    }
    if (!es) return;
    wo_grad_regs<NT, RT>(net, top, dqs, 1, es);
    // bo = sum of dq over the block's rows (all in wave 0: TM <= 64), and its 3 padding floats
    if (tid < 64) {
        const float sb = wave_sum(dqv);
        if (tid < 4) es[e_bo(net) + tid] = tid == 0 ? sb : 0.f;
    }
}

// Layer 0's per-lane constants (W0 columns h and 2 + h, the bias) of the wave's column tiles:
// loaded one network pass ahead by the fused row programs, so their latency hides under the
// previous pass instead of opening this pass's layer 0
struct L0Pre {
    float wa[2], wb[2], bias[2];
};
template <int NT>
NAV_DEV L0Pre load_l0(const MlpDev& net) {
    const int lane = threadIdx.x & 63, h = lane >> 5, l32 = lane & 31;
    const WaveCols<NT> wc(wave_id());
    const float* W0 = net.params + net.w_off[0];
    const float* b0 = net.params + net.b_off[0];
    const int d_in = net.d_in;
    L0Pre p;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const bool has = j == 0 ? wc.has0 : wc.has1;
        const int c = (j == 0 ? wc.t0 : wc.t1) * 32 + l32;
        p.wa[j] = has && h < d_in ? W0[c * d_in + h] : 0.f;
        p.wb[j] = has && 2 + h < d_in ? W0[c * d_in + 2 + h] : 0.f;
        p.bias[j] = has ? b0[c] : 0.f;  // the column's bias in both lane halves (the C operand)
    }
    return p;
}

// One network's forward over the block's TM rows (input rows xin [TM][4] in LDS). The top hidden
// layer stays in registers (`top`, C layout) — its LDS rows are written only when save_mask asks
// for its global copy — and the output layer's per-wave partials land in `red` (ready for out_y
// after the trailing barrier).
// DIN: the network's d_in when the caller knows it (2 actor, 4 critic; 0: read net.d_in), so the
// layer-0 product has no branch on the input count
template <int NT, int RT, int PFB = 1, int DIN = 0>
NAV_DEV void fwd_net(const MlpDev& net, float* act, _Float16* stage, const float* xin, float* red,
                     uint16_t* masks, int64_t n_rt, float* act_save, uint32_t save_mask,
                     int64_t row0, int64_t M, int64_t rt0, f32x16 (&top)[RT][2], int mk = -64,
                     const L0Pre* pre = nullptr, uint32_t* top_bits = nullptr,
                     WoCols* wo_out = nullptr) {
    constexpr int hp = NT * 32, SS = hp + 4;
    NAV_MARK(mk);
    const int tid = threadIdx.x, lane = tid & 63, wv = wave_id(), h = lane >> 5, l32 = lane & 31;
    const int nh = net.n_hidden;
    const WaveCols<NT> wc(wv);
    (void)tid;
    // the output layer's Wo columns: issued now, in flight under layer 0 and the GEMMs
    const WoCols wo = load_wo<NT>(net);
    if (wo_out) *wo_out = wo;
    // ---- layer 0 (K = d_in <= 4) on MFMA, straight into the C layout of the wave's column
    // tiles: the C tile starts at the bias (set by VALU), then x[:, 0:2] and (d_in > 2) x[:, 2:4]
    // against W0's columns: each element is fma(x3, w3, fma(x2, w2, fma(x1, w1, fma(x0, w0, b))))
    // — layer0_unit's chain, bit for bit (absent inputs and weights are 0)
    {
        const L0Pre l0 = pre ? *pre : load_l0<NT>(net);
        float m0[RT] = {};
        const bool x23 = DIN == 0 ? net.d_in > 2 : DIN > 2;
        // A operands: row l32 of each row tile, inputs h and 2 + h
        float xa[RT], xb[RT];
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
            const float4 xr = *reinterpret_cast<const float4*>(xin + (rt * 32 + l32) * 4);
            xa[rt] = h ? xr.y : xr.x;
            xb[rt] = h ? xr.w : xr.z;
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            if (!(j == 0 ? wc.has0 : wc.has1)) continue;
            const int t = j == 0 ? wc.t0 : wc.t1;
            const int c = t * 32 + l32;
            const float wa = l0.wa[j], wb = l0.wb[j];
            // the C tile starts at the column's bias, set by VALU (exactly what the K = 2 MFMA of
            // (1, 0) x (b, 0) gave); inputs 2, 3 only for d_in > 2
            f32x16 bias;
#pragma unroll
            for (int i = 0; i < 16; ++i) bias[i] = l0.bias[j];
            float* col = act + c + 4 * h * SS;
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) {
                f32x16 v = mfma(xa[rt], wa, bias);
                if (x23) v = mfma(xb[rt], wb, v);
                uint32_t bits = 0;
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const float r = relu(v[i]);
                    col[(rt * 32 + (i & 3) + 8 * (i >> 2)) * SS] = r;
                    bits |= pos_bit(r) << i;
                    m0[rt] = max_nn(m0[rt], r);
                }
                if (masks) masks[mask_idx(rt0 + rt, NT, t, lane)] = (uint16_t)bits;
            }
        }
        if (nh >= 2) publish_amax(amax_slots<RT * 32>(stage), m0);  // layer 1's A scale
    }
    NAV_MARK(mk + 1);
    __syncthreads();
    NAV_MARK(mk + 2);
    if (act_save && (save_mask & 1u)) copy_rows<NT, RT>(act, SS, act_save, row0, M);
    // one hidden x hidden layer on MFMA: acc = relu(rows . W_L + b_L), C layout
    auto hidden_layer = [&](int L, f32x16 (&acc)[RT][2]) {
        // the bias is loaded before the product so its latency hides under the MFMAs
        const float* bL = net.params + net.b_off[L];
        const float bb0 = wc.has0 ? bL[wc.t0 * 32 + l32] : 0.f;
        const float bb1 = wc.has1 ? bL[wc.t1 * 32 + l32] : 0.f;
        gemm_cols<NT, RT, PFB>(act, SS, img_fwd(net, L), stage, acc);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            if (!(j == 0 ? wc.has0 : wc.has1)) continue;
            const float b = j == 0 ? bb0 : bb1;
#pragma unroll
            for (int rt = 0; rt < RT; ++rt)
#pragma unroll
                for (int i = 0; i < 16; ++i) acc[rt][j][i] = relu(acc[rt][j][i] + b);
        }
    };
    auto mask_of = [&](int L) { return masks ? masks + (size_t)L * n_rt * NT * 64 : nullptr; };
    // ---- layers 1 .. nh-2: rows back into LDS for the next layer
    for (int L = 1; L + 1 < nh; ++L) {
        f32x16 acc[RT][2];
        hidden_layer(L, acc);
        NAV_TRACE_MARK(50);
        __syncthreads();  // every wave has finished reading the layer's input rows
        store_layer<NT, RT>(acc, act, SS, mask_of(L), rt0, amax_slots<RT * 32>(stage));
        __syncthreads();
        NAV_TRACE_MARK(51);
        if (act_save && ((save_mask >> L) & 1u))
            copy_rows<NT, RT>(act, SS, act_save + (int64_t)L * M * hp, row0, M);
    }
    // ---- the top hidden layer: registers (defined here only, so they are not live above)
    if (nh >= 2) {
        const int L = nh - 1;
        hidden_layer(L, top);
        NAV_MARK(mk + 3);
        if (act_save && ((save_mask >> L) & 1u)) {
            __syncthreads();
            store_layer<NT, RT>(top, act, SS, mask_of(L), rt0);
            __syncthreads();
            copy_rows<NT, RT>(act, SS, act_save + (int64_t)L * M * hp, row0, M);
        } else if (masks && !top_bits) {
            store_mask<NT, RT>(top, mask_of(L), rt0);
        }
        if (top_bits) {  // the top layer's ReLU bits stay in registers for the row backward
            uint16_t* mk = masks && !(act_save && ((save_mask >> L) & 1u)) ? mask_of(L) : nullptr;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const bool has = j == 0 ? wc.has0 : wc.has1;
#pragma unroll
                for (int rt = 0; rt < RT; ++rt) {
                    uint32_t bits = 0;
#pragma unroll
                    for (int i = 0; i < 16; ++i) bits |= pos_bit(top[rt][j][i]) << i;  // post-ReLU
                    top_bits[rt * 2 + j] = has ? bits : 0u;
                    if (mk && has)
                        mk[mask_idx(rt0 + rt, NT, j == 0 ? wc.t0 : wc.t1, lane)] = (uint16_t)bits;
                }
            }
        }
    } else {
        // the top layer is layer 0: its C-layout registers from the LDS rows just written
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const bool has = j == 0 ? wc.has0 : wc.has1;
            const float* col = act + (j == 0 ? wc.t0 : wc.t1) * 32 + l32;
#pragma unroll
            for (int rt = 0; rt < RT; ++rt)
#pragma unroll
                for (int i = 0; i < 16; ++i) top[rt][j][i] = has ? col[c_row(rt, i, h) * SS] : 0.f;
        }
    }

    // ---- output layer (N = d_out <= 2) from the registers; a barrier publishes the partials
    out_partials<NT, RT>(net, top, wo, red);
    NAV_MARK(mk + 4);
    __syncthreads();
    NAV_MARK(mk + 5);
}

template <int NT, int RT, int IN_MODE, int OUT_MODE>
__global__ __launch_bounds__(kBlock, 1) void k_mlp_fwd(FwdArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    constexpr int hp = NT * 32, SS = hp + 4, TM = RT * 32;
    const int tid = threadIdx.x;
    const MlpDev& net = a.net[blockIdx.y];
    float* act_save = a.acts[blockIdx.y];
    uint16_t* masks = a.masks[blockIdx.y];
    const int64_t M = a.M;
    const int64_t row0 = (int64_t)blockIdx.x * TM;
    const int64_t rt0 = (int64_t)blockIdx.x * RT;
    const int64_t n_rt = mask_rowtiles(M);
    float* act = smem;
    float* xin = smem + TM * SS;  // [TM][4]
    _Float16* stage = reinterpret_cast<_Float16*>(smem + lds_floats(hp, TM));
    const int d_in = net.d_in, d_out = net.d_out;
    // layer 0's per-lane weights and bias: issued first, in flight under the input rows' loads
    const L0Pre l0 = load_l0<NT>(net);
    if constexpr (OUT_MODE == OUT_TICK) NAV_CLOCK(2, 0);

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
    // OUT_TICK: the row's tick inputs that do not depend on its action (state, goal, meta, the
    // plan counters, the stuck ring, the field value), its noise scale and exploration noise are
    // loaded / drawn now, so their latency hides under the network pass
    TickIn tin{};
    double nsc = 0.0;
    double2 zz = make_double2(0.0, 0.0);
    if constexpr (OUT_MODE == OUT_TICK) {
        const int64_t r = row0 + tid;
        if (tid < TM && r < M) {
            tin = tick_load(a.env, a.field, r);
            if (a.act_mode == 0) {
                nsc = a.noise_scale[r];
                if (a.noise_z)
                    zz = make_double2(a.noise_z[r * 2], a.noise_z[r * 2 + 1]);
                else
                    zz = gauss_pair(philox(0u, (uint32_t)r, NAV_TAG_NOISE, a.step, a.p.seed_lo,
                                           a.p.seed_hi));
            }
        }
    }
    __syncthreads();

    float* red = xin + TM * 4;  // [2][PARTS][TM]
    f32x16 top[RT][2];
    fwd_net<NT, RT, kPfWide, IN_MODE == IN_BASELINE ? 2 : 0>(net, act, stage, xin, red, masks, n_rt, act_save, a.save_mask, row0, M, rt0, top,
                    OUT_MODE == OUT_TICK ? NAV_TICK_MK : -64, &l0);
    const int rloc = tid % TM;
    const int j = tid / TM;
    const int64_t r = row0 + rloc;
    if (OUT_MODE == OUT_LOSS) {
        // robot.py:341-345 TD target y = r + gamma * min(q1', q2') * (1 - done)
        float yt = 0.f;
        if (tid < TM && r < M) {
            const float rw = a.batch[r * NAV_ROW + 4], dn = a.batch[r * NAV_ROW + 7];
            const float mn = fminf(a.qt[0][r], a.qt[1][r]);
            yt = rw + (a.gamma * mn) * (1.0f - dn);
        }
        const int q = blockIdx.y;
        loss_epilogue<NT, RT>(net, top, red, row0, M, yt, a.norm, a.dq[q],
                              a.loss_part[q] + blockIdx.x,
                              a.eslab[q] ? a.eslab[q] + (int64_t)blockIdx.x * a.ecount : nullptr);
        return;
    }
    if constexpr (OUT_MODE == OUT_TICK) {
        // robot.py:556-567 as OUT_ACT, the action parked in LDS (the input rows are done with),
        // then the tick of env row0 + t by thread t < TM: nav_agent_step's device code
        // the row's thread forms both action components (the same expressions per component as
        // OUT_ACT) and runs its env's tick; no LDS round trip, no barrier in between
        DemoPend pend{false, false, 0.0, make_double2(0.0, 0.0)};
        TickStats st{0.f, 0.f, 0.f, 0.f, 0.f};
        NAV_TRACE_MARK(NAV_TICK_MK + 6);
        if (tid < TM && r < M) {
            double v[2];
#pragma unroll
            for (int jj = 0; jj < 2; ++jj) {
                const float y = out_y<RT>(net, red, tid, jj);
                const double sj = jj == 0 ? tin.s.x : tin.s.y, gj = jj == 0 ? tin.g.x : tin.g.y;
                double c = (sj - gj) + (double)y;
                if (a.act_mode == 0) c = c + (nsc * a.max_action_d) * (jj == 0 ? zz.x : zz.y);
                v[jj] = clipd(c, -a.max_action_d, a.max_action_d);
                if (a.action_out) a.action_out[r * 2 + jj] = v[jj];
            }
            const double2 av = make_double2(v[0], v[1]);
            st = a.demo.cand ? agent_tick_in<true>(a.p, a.env, r, tin, av, a.rows, a.cap, a.base,
                                                   a.sout, true, pend)
                             : agent_tick_in<false>(a.p, a.env, r, tin, av, a.rows, a.cap,
                                                    a.base, a.sout, false, pend);
        }
        NAV_TRACE_MARK(NAV_TICK_MK + 7);
        if (a.demo.cand) {  // block-uniform: the demo pass of the block's envs, all threads
            // the LDS rows are done with (the actions live in xin)
            auto* scratch = reinterpret_cast<DemoScratch<TM, kBlock>*>(act);
            const double rd = demo_pass<TM, kBlock>(a.p, a.demo, *scratch, pend, r,
                                                    reinterpret_cast<float*>(a.rows), a.cap,
                                                    a.base, a.reward_out);
            if (pend.need) st.r = (float)rd;  // the final reward of a flagged env
        }
        NAV_TRACE_MARK(NAV_TICK_MK + 8);
        if (tid < TM && a.sout.block_stats && row0 + (tid & ~63) < M)
            wave_stats(st, a.sout.block_stats, r);
        NAV_TRACE_MARK(NAV_TICK_MK + 9);
        NAV_CLOCK(2, 1);
        return;
    }
    if (r >= M || j >= d_out) return;
    const float y = out_y<RT>(net, red, rloc, j);
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
    MlpDev net[2];           // 1 or 2 networks (blockIdx.y), same shapes, same input rows
    int64_t M;
    const float* dy[2];
    int ld_dy;               // dy row stride (0: one row broadcast to every row)
    const uint16_t* masks[2];
    const float* in;         // the forward's input rows (dW0 partials), with eslab
    int ld_in, in_col;
    const float* h_top[2];   // nullable: [M][hp] top activations -> Wo / bo partials here
    float* dz[2];            // [n_hidden][M][hp], layers with a save_mask bit written
    uint32_t save_mask;
    float* dx[2];
    float* eslab[2];         // nullable: [blocks][edge_count] W0 / bias (/ Wo / bo) partials
    int64_t ecount;
};

// The lane's ReLU mask words of one layer (issued ahead of the product that needs them).
template <int NT, int RT>
NAV_DEV void load_mask_bits(const uint16_t* mask, int64_t rt0, uint32_t (&bits)[RT][2]) {
    const int lane = threadIdx.x & 63;
    const WaveCols<NT> wc(wave_id());
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const bool has = j == 0 ? wc.has0 : wc.has1;
        const int t = j == 0 ? wc.t0 : wc.t1;
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) bits[rt][j] = has ? mask[mask_idx(rt0 + rt, NT, t, lane)] : 0u;
    }
}

// Edge partials of one hidden layer's dz from the C-layout registers: db[c] = column sum over the
// block's rows (each lane sums its 16 * RT rows in (row tile, element) order, then the two lane
// halves meet: rows +0 / +4), and for layer 0 also dW0[c][k] = sum_rows dz[row][c] x[row][k]
// (x rows from xin [TM][4], one broadcast read per row shared by both column tiles).
template <int NT, int RT>
NAV_DEV void edge_regs(const MlpDev& net, const f32x16 (&z)[RT][2], const float* xin, int L,
                       float* es) {
    const int lane = threadIdx.x & 63, h = lane >> 5, l32 = lane & 31;
    const WaveCols<NT> wc(wave_id());
    const int d_in = net.d_in;
    float sb[2] = {0.f, 0.f}, sw[2][4] = {};
    if (L == 0) {
        // dW0's four input columns as two packed pairs (v_pk_fma_f32: the same fused op per
        // element as fmaf, two elements per instruction)
        typedef float f32x2 __attribute__((ext_vector_type(2)));
        f32x2 w01[2] = {{0.f, 0.f}, {0.f, 0.f}}, w23[2] = {{0.f, 0.f}, {0.f, 0.f}};
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const float4 x = *reinterpret_cast<const float4*>(xin + c_row(rt, i, h) * 4);
                const f32x2 x01 = {x.x, x.y}, x23 = {x.z, x.w};
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const float v = z[rt][j][i];
                    const f32x2 vv = {v, v};
                    sb[j] += v;
                    w01[j] = __builtin_elementwise_fma(vv, x01, w01[j]);
                    w23[j] = __builtin_elementwise_fma(vv, x23, w23[j]);
                }
            }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            sw[j][0] = w01[j].x; sw[j][1] = w01[j].y; sw[j][2] = w23[j].x; sw[j][3] = w23[j].y;
        }
    } else {
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
            for (int i = 0; i < 16; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) sb[j] += z[rt][j][i];
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        sb[j] += __shfl_xor(sb[j], 32, 64);
        if (L == 0)
#pragma unroll
            for (int k = 0; k < 4; ++k) sw[j][k] += __shfl_xor(sw[j][k], 32, 64);
    }
    if (h != 0) return;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        if (!(j == 0 ? wc.has0 : wc.has1)) continue;
        const int c = (j == 0 ? wc.t0 : wc.t1) * 32 + l32;
        es[e_b(net, L) + c] = sb[j];
        if (L == 0)
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (k < d_in) es[net.w_off[0] + c * d_in + k] = sw[j][k];
    }
}

// Masks the layer's dz registers in place (ReLU derivative bits), without the LDS rows.
template <int NT, int RT>
NAV_DEV void mask_regs(f32x16 (&acc)[RT][2], const uint32_t (&mbits)[RT][2]) {
    const WaveCols<NT> wc(wave_id());
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const bool has = j == 0 ? wc.has0 : wc.has1;
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
            for (int i = 0; i < 16; ++i)
                acc[rt][j][i] = has && ((mbits[rt][j] >> i) & 1u) ? acc[rt][j][i] : 0.f;
    }
}

// Masks the layer's dz registers in place (ReLU derivative bits) and stores them to the LDS rows;
// with slots, publishes their max |value| for the next GEMM's A scale.
template <int NT, int RT>
NAV_DEV void mask_and_store(f32x16 (&acc)[RT][2], const uint32_t (&mbits)[RT][2], float* act,
                            int S_, float* slots = nullptr) {
    const int lane = threadIdx.x & 63, wv = wave_id(), h = lane >> 5, l32 = lane & 31;
    const WaveCols<NT> wc(wv);
    float m[RT] = {};
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        if (!(j == 0 ? wc.has0 : wc.has1)) {
#pragma unroll
            for (int rt = 0; rt < RT; ++rt)
#pragma unroll
                for (int i = 0; i < 16; ++i) acc[rt][j][i] = 0.f;
            continue;
        }
        const int t = j == 0 ? wc.t0 : wc.t1;
        float* col = act + t * 32 + l32 + 4 * h * S_;
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
            const uint32_t bits = mbits[rt][j];
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                acc[rt][j][i] = (bits >> i) & 1u ? acc[rt][j][i] : 0.f;
                col[(rt * 32 + (i & 3) + 8 * (i >> 2)) * S_] = acc[rt][j][i];
                m[rt] = fmaxf(m[rt], fabsf(acc[rt][j][i]));
            }
        }
    }
    publish_amax(slots, m);
}

// One network's row backward over the block's TM rows: dy rows in dys [TM][4] (LDS, ready), the
// forward's ReLU bits in masks; leaves dz_0 in the LDS rows `act`. With es: the per-block edge
// partials (every bias, dW0 from the input rows xin [TM][4], and dWo / dbo when h_top [M][hp] is
// given); dz_L rows to dz for save_mask bits.
// BM: the top layer's product form. 0: every layer on gemm_cols (any d_out); 1: d_out = 1, the
// top layer on gemm_bits, the layers below on gemm_cols (n_hidden >= 3); 2: d_out = 1 and
// n_hidden = 2, gemm_bits only. Compile-time, so a kernel carries only the forms it runs (both
// forms in one function took the row kernels past 256 registers: one workgroup per CU).
template <int NT, int RT, int PFB = 1, int BM = 0>
NAV_DEV void bwd_net(const MlpDev& net, float* act, _Float16* stage, const float* dys, const float* xin,
                     const uint16_t* masks, int64_t n_rt, float* es, const float* h_top,
                     float* dz, uint32_t save_mask, int64_t row0, int64_t M, int64_t rt0,
                     int mk = -64, const uint32_t* top_bits = nullptr,
                     const WoCols* wo_in = nullptr, bool dz0_rows = true) {
    constexpr int hp = NT * 32, SS = hp + 4, TM = RT * 32;
    NAV_MARK(mk);
    const int tid = threadIdx.x, lane = tid & 63, wv = wave_id(), h = lane >> 5, l32 = lane & 31;
    const int d_in = net.d_in, d_out = net.d_out, nh = net.n_hidden;
    const int64_t MH = M * hp;
    const WaveCols<NT> wc(wv);
    const size_t mstride = (size_t)n_rt * NT * 64;
    if (es) {
        // output layer (robot.py:361 / 392 backward): dWo = dy^T h_top, dbo = sum dy, when the
        // forward did not produce them (it does for the critic's TD loss)
        if (h_top) {
            // rows in wo_grad_regs' order: per lane half, (row tile, C element); halves added last
            const int n = tid;
            if (n < hp) {
                float s0[2] = {0.f, 0.f}, s1[2] = {0.f, 0.f};
#pragma unroll
                for (int hh = 0; hh < 2; ++hh)
#pragma unroll
                    for (int rt = 0; rt < RT; ++rt)
#pragma unroll 4
                        for (int i = 0; i < 16; ++i) {
                            const int rr = c_row(rt, i, hh);
                            if (row0 + rr >= M) continue;
                            const float hv = h_top[(row0 + rr) * hp + n];
                            s0[hh] = fmaf(dys[rr * 4], hv, s0[hh]);
                            s1[hh] = fmaf(dys[rr * 4 + 1], hv, s1[hh]);
                        }
                es[e_wo(net) + n] = s0[0] + s0[1];
                if (d_out > 1) es[e_wo(net) + hp + n] = s1[0] + s1[1];
            }
            if (tid < 4) {
                float s = 0.f;
                if (tid < d_out)
                    for (int rr = 0; rr < TM; ++rr) s += dys[rr * 4 + tid];
                es[e_bo(net) + tid] = s;
            }
        }
    }

    // d_out = 1: the top layer's backward product runs on the forward's ReLU bits (gemm_bits; the
    // Wt image is the only backward image of that layer); its dz rows are still formed (and
    // copied out) where save_mask asks for them
    constexpr bool bits_path = BM > 0;
    const bool save_top = (save_mask >> (nh - 1)) & 1u;
    // top hidden layer: dz = (dy . Wo) * relu'(.), in the C layout: one K = 2 MFMA per tile of
    // dy rows (lane l32 = row, h = output) against Wo's columns, fma(dy1, w1, dy0 w0) — the
    // chain the weight-gradient kernel recomputes — then the forward's ReLU bits. On the bits
    // path these registers only feed the layer's bias partials (and are skipped without es).
    uint32_t mb[RT][2];
    {
        const float* Wo = net.params + net.w_off[nh];
        const uint16_t* mk = masks + (size_t)(nh - 1) * mstride;
        const f32x16 zero = {};
        float ga[RT];
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
            const float4 g = *reinterpret_cast<const float4*>(dys + (rt * 32 + l32) * 4);
            ga[rt] = h < d_out ? (h ? g.y : g.x) : 0.f;
        }
        if (top_bits) {  // the forward's bits of this top layer, still in registers
#pragma unroll
            for (int rt = 0; rt < RT; ++rt)
#pragma unroll
                for (int j = 0; j < 2; ++j) mb[rt][j] = top_bits[rt * 2 + j];
        } else {
            load_mask_bits<NT, RT>(mk, rt0, mb);
        }
        if (!bits_path || (es && nh > 1) || save_top) {
            f32x16 z[RT][2];
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const bool has = j == 0 ? wc.has0 : wc.has1;
                const int c = (j == 0 ? wc.t0 : has ? wc.t1 : wc.t0) * 32 + l32;
                // the forward's Wo registers: wo.w[output][tile] holds Wo[output][c] (0 when absent)
                const float wb = wo_in ? (h ? wo_in->w[1][j] : wo_in->w[0][j])
                                       : has && h < d_out ? Wo[h * hp + c] : 0.f;
#pragma unroll
                for (int rt = 0; rt < RT; ++rt) z[rt][j] = mfma(ga[rt], wb, zero);
            }
            if (bits_path && !save_top)
                mask_regs<NT, RT>(z, mb);
            else
                mask_and_store<NT, RT>(z, mb, act, SS,
                                       !bits_path && nh > 1 ? amax_slots<TM>(stage) : nullptr);
            if (es && nh > 1) edge_regs<NT, RT>(net, z, xin, nh - 1, es);
        }
        if (bits_path) {
            if (save_top) {  // the top layer's dz rows themselves, before the scratch reuses act
                __syncthreads();
                copy_rows<NT, RT>(act, SS, dz + (int64_t)(nh - 1) * MH, row0, M);
                __syncthreads();
            }
            bits_stage<NT, RT>(act, mb, dys);
        }
    }
    NAV_MARK(mk + 1);
    __syncthreads();
    // per layer: the rows themselves only where the weight-gradient kernel cannot recompute them
    // (save_mask); the edge partials come from the registers (edge_regs), except for a one-layer
    // network's layer 0 written by the top unit above (LDS column sums)
    auto finish_layer = [&](int L) {
        if (es && nh == 1) {
            edge_col_sums<TM>(act, SS, hp, es + e_b(net, L));
            edge_w0<TM>(act, SS, hp, xin, d_in, es + net.w_off[0]);
        }
        if ((save_mask >> L) & 1u) copy_rows<NT, RT>(act, SS, dz + (int64_t)L * MH, row0, M);
    };
    if (!bits_path) finish_layer(nh - 1);
    NAV_MARK(mk + 2);

    // after layer L's product (acc = dz_L . W_L): mask with layer L - 1's bits, its rows to LDS
    // where a reader follows, its edge partials
    auto after_product = [&](int L, f32x16 (&acc)[RT][2], const uint32_t (&mbits)[RT][2]) {
        __syncthreads();
        // layer 0's rows only when a reader follows (the caller's dx, the save copy); its edge
        // partials come from the registers
        if (L > 1 || dz0_rows || (save_mask & 1u))
            mask_and_store<NT, RT>(acc, mbits, act, SS, L > 1 ? amax_slots<TM>(stage) : nullptr);
        else
            mask_regs<NT, RT>(acc, mbits);
        if (es) edge_regs<NT, RT>(net, acc, xin, L - 1, es);
        __syncthreads();
        NAV_MARK(mk + 4);
        finish_layer(L - 1);
    };
    int Ltop = nh - 1;
    if (bits_path) {
        f32x16 acc[RT][2];
        uint32_t mbits[RT][2];
        load_mask_bits<NT, RT>(masks + (size_t)(nh - 2) * mstride, rt0, mbits);
        gemm_bits<NT, RT, PFB>(act, img_bwd(net, nh - 1), acc);
        NAV_MARK(mk + 3);
        after_product(nh - 1, acc, mbits);
        Ltop = nh - 2;
    }
    // hidden layers, top-down: dz_{L-1} = (dz_L . W_L) * relu'(act_{L-1}), B = packed Wb_L
    if constexpr (BM != 2) {
        for (int L = Ltop; L >= 1; --L) {
            f32x16 acc[RT][2];
            uint32_t mbits[RT][2];
            load_mask_bits<NT, RT>(masks + (size_t)(L - 1) * mstride, rt0, mbits);
            gemm_cols<NT, RT, PFB>(act, SS, img_bwd(net, L), stage, acc);
            NAV_MARK(mk + 3);
            after_product(L, acc, mbits);
        }
    }
    NAV_MARK(mk + 5);

}

// dL/dx[row][jj] = dz_0[row] . W0[:, jj] from the LDS rows (after bwd_net)
template <int NT>
NAV_DEV float dx_unit(const MlpDev& net, const float* act, int rloc, int jj) {
    constexpr int hp = NT * 32, SS = hp + 4;
    const float* W0 = net.params + net.w_off[0];
    const float* zr = act + rloc * SS;
    float acc = 0.f;
    for (int c = 0; c < hp; ++c) acc = fmaf(zr[c], W0[c * net.d_in + jj], acc);
    return acc;
}

template <int NT, int RT, int BM>
__global__ __launch_bounds__(kBlock, 1) void k_mlp_bwd(BwdArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    constexpr int hp = NT * 32, SS = hp + 4, TM = RT * 32;
    const int tid = threadIdx.x;
    const int y = blockIdx.y;
    const MlpDev& net = a.net[y];
    const int64_t M = a.M;
    const int64_t row0 = (int64_t)blockIdx.x * TM;
    const int64_t rt0 = (int64_t)blockIdx.x * RT;
    const int64_t n_rt = mask_rowtiles(M);
    float* act = smem;
    _Float16* stage = reinterpret_cast<_Float16*>(smem + lds_floats(hp, TM));
    float* dys = smem + TM * SS;  // [TM][4] dy rows
    float* xin = dys + TM * 4;    // [TM][4] forward input rows (dW0), inside the red scratch
    const int d_in = net.d_in, d_out = net.d_out;
    static_assert(hp <= kBlock, "one thread per hidden column");
    float* es = a.eslab[y] ? a.eslab[y] + (int64_t)blockIdx.x * a.ecount : nullptr;

    if (tid < TM) {
        const int64_t r = row0 + tid;
        float x[2] = {0.f, 0.f};
        float xi[4] = {0.f, 0.f, 0.f, 0.f};
        if (r < M) {
            for (int j = 0; j < d_out; ++j) x[j] = a.dy[y][r * a.ld_dy + j];
            if (es)
                for (int k = 0; k < d_in; ++k) xi[k] = a.in[r * a.ld_in + a.in_col + k];
        }
        *reinterpret_cast<float4*>(dys + tid * 4) = make_float4(x[0], x[1], 0.f, 0.f);
        *reinterpret_cast<float4*>(xin + tid * 4) = make_float4(xi[0], xi[1], xi[2], xi[3]);
    }
    __syncthreads();
    bwd_net<NT, RT, 1, BM>(net, act, stage, dys, xin, a.masks[y], n_rt, es, a.h_top[y], a.dz[y],
                           a.save_mask, row0, M, rt0);

    // dx = dz_0 . W0 : thread = (row, input)
    if (a.dx[y]) {
        const int rloc = tid % TM;
        const int64_t r = row0 + rloc;
        for (int jj = tid / TM; jj < d_in; jj += kBlock / TM) {
            const float v = dx_unit<NT>(net, act, rloc, jj);
            if (r < M) a.dx[y][r * d_in + jj] = v;
        }
    }
}

// ---------------- fused TD3 row programs ----------------
// Everything in train_critic / train_actor that is local to a batch row runs as one launch per
// row block, the rows staying in LDS between the network passes (the launches that remain are
// the cross-row reductions: weight gradients and their reduce + Adam).

// ReplayBuffer.sample (robot.py:98-115) of row b: injected index or Philox with replacement
NAV_DEV void sample_row(const float* rows, int64_t size, const int64_t* idx, uint32_t s0,
                        uint32_t s1, uint32_t ctr, int64_t b, float4& lo, float4& hi) {
    int64_t k;
    if (idx) {
        k = idx[b];
    } else {
        const uint4 w = philox((uint32_t)b, 0u, NAV_TAG_SAMPLE, ctr, s0, s1);
        k = (int64_t)(((uint64_t)w.x * (uint64_t)size) >> 32);
    }
    const float4* src = reinterpret_cast<const float4*>(rows) + 2 * k;
    lo = src[0];
    hi = src[1];
}

// ---- L2 warmers for small grids ----
// A 32-row workgroup streams every weight image it multiplies by (hp^2 + hp floats per layer)
// and, alone on its XCD at small batches, each k step's B fragments arrive from beyond its L2 at
// one CU's fetch rate (~75 GB/s: ~500 cycles per step of 6 MFMAs at hp = 224, flat in the
// prefetch depth; profiles/r06za). The row kernels therefore launch, when the compute grid leaves
// most CUs idle, extra workgroup rows (blockIdx.y >= y0) that only touch one 4-B word per 128-B
// line of the launch's images, in the order the compute workgroups consume them, so the lines
// are in each XCD's L2 before the compute workgroups ask. Blocks are dealt round-robin over the
// 8 XCDs (MI355X_MICROARCH: b and b + 8 share one; speed only, never correctness): the warmers
// with equal (index mod 8) split the image list between them.
constexpr int kWarmMax = 16;         // image ranges per launch
constexpr int kWarmPerXcd = 16;      // warmer workgroups per XCD
constexpr int64_t kWarmGrid = 128;   // compute workgroups up to which warmers are launched
struct WarmList {
    int y0;                          // grid rows of compute workgroups (warmers: rows >= y0)
    int n;                           // ranges (0: no warmers)
    const char* p[kWarmMax];
    uint32_t bytes[kWarmMax];
};

NAV_DEV void warm_l2(const WarmList& w) {
    const uint32_t j = blockIdx.x + gridDim.x * (blockIdx.y - (uint32_t)w.y0);
    const uint32_t nw = gridDim.x * (gridDim.y - (uint32_t)w.y0);
    const uint32_t cnt = (nw - (j & 7u) + 7u) >> 3, rank = j >> 3;  // warmers of this XCD
    uint32_t x = 0;
    for (int i = 0; i < w.n; ++i) {
        const uint32_t lines = (w.bytes[i] + 127u) >> 7;
        const uint32_t per = (lines + cnt - 1u) / cnt;
        const uint32_t l1 = min(lines, (rank + 1u) * per);
        const char* p = w.p[i];
#pragma unroll 4
        for (uint32_t l = rank * per + threadIdx.x; l < l1; l += kBlock)
            x ^= *reinterpret_cast<const uint32_t*>(p + ((size_t)l << 7));
    }
    asm volatile("" ::"v"(x));  // keeps the loads
}

// host: append [p, p + bytes) to the list; false when full
inline bool warm_add(WarmList& w, const float* p, int64_t floats) {
    if (w.n >= kWarmMax) return false;
    w.p[w.n] = reinterpret_cast<const char*>(p);
    w.bytes[w.n++] = (uint32_t)(floats * 4);
    return true;
}
// host: a network's forward images (layers 1 .. nh-1), or its whole packed buffer (all images)
inline bool warm_net(WarmList& w, const MlpDev& net, bool fwd_only) {
    if (net.n_hidden < 2) return true;
    const int64_t im = split_image_floats(net.hp);
    if (!fwd_only) return warm_add(w, net.packed, (int64_t)(net.n_hidden - 1) * 2 * im);
    for (int L = 1; L < net.n_hidden; ++L)
        if (!warm_add(w, net.packed + (int64_t)(L - 1) * 2 * im, im)) return false;
    return true;
}
// host: grid rows of warmers for a compute grid of gx x gy (0: none)
inline unsigned warm_rows(const WarmList& w, unsigned gx, unsigned gy) {
    if (w.n == 0 || (int64_t)gx * gy > kWarmGrid) return 0;
    return (8u * kWarmPerXcd + gx - 1) / gx;
}

struct CriticRowsArgs {
    MlpDev actor_t, critic_t[2], critic[2];
    int64_t B;
    const float* rows;
    int64_t rsize;
    const int64_t* idx;
    uint32_t seed_lo, seed_hi, sample_ctr, noise_ctr;
    const float* eps;
    float policy_noise, noise_clip, max_action, gamma, norm;
    float* batch;
    float* dq[2];
    float* loss_part[2];
    float* eslab[2];
    int64_t ecount;
    float* acts[2];
    uint32_t save_mask;
    uint16_t* masks[2];
    int row_backward;     // also each online critic's row backward (robot.py:361 .backward())
    int split_twins;      // grid.y = 2: workgroup y runs online critic y only (small batches)
    float* dz[2];         // [nh][B][hp] dz rows of dz_save_mask layers (row_backward)
    uint32_t dz_save_mask;
    WarmList warm;        // set by the launcher
};
static_assert(sizeof(CriticRowsArgs) <= 4096, "kernel argument size");

// train_critic (robot.py:329-361) for one block of TM batch rows: sample, target policy
// smoothing through the target actor, twin target critics, TD target, then the twin online
// critics with mse_loss's gradient, the loss and the output layers' gradient partials, and
// (row_backward) each online critic's row backward with its W0 / bias partials right after its
// forward, while its rows and ReLU bits are fresh.
// CBM: the critics' row-backward form (bwd_net's BM: 0 for one hidden layer, else 1), chosen by
// the launcher from n_hidden
template <int NT, int RT, int CBM>
__global__ __launch_bounds__(kBlock, 1) void k_td3_critic_rows(CriticRowsArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    if (a.warm.n && (int)blockIdx.y >= a.warm.y0) {  // an L2 warmer row (small grids)
        warm_l2(a.warm);
        return;
    }
    constexpr int hp = NT * 32, SS = hp + 4, TM = RT * 32;
    const int tid = threadIdx.x;
    const int64_t B = a.B, row0 = (int64_t)blockIdx.x * TM, rt0 = (int64_t)blockIdx.x * RT;
    const int64_t n_rt = mask_rowtiles(B);
    float* act = smem;
    float* xin = act + TM * SS;    // [TM][4] network input rows
    float* red = xin + TM * 4;     // [2][PARTS][TM] output partial sums
    float* brow = red + red_floats(TM);  // [TM][8] the sampled replay rows
    float* qv = brow + TM * 8;     // [TM] q1'
    float* dys = qv + TM;          // [TM][4] dL/dq rows of the row backward
    _Float16* stage = reinterpret_cast<_Float16*>(dys + TM * 4);  // gemm_cols' split stage
    NAV_MARK(0);
    NAV_CLOCK(0, 0);
    const L0Pre l0_at = load_l0<NT>(a.actor_t);  // in flight under the sampling
    // the sampled replay row of thread tid < TM: its gather is issued first, so it is in flight
    // while the smoothing noise below is formed
    float4 lo = make_float4(0.f, 0.f, 0.f, 0.f), hi = lo;
    if (tid < TM && row0 + tid < B)
        sample_row(a.rows, a.rsize, a.idx, a.seed_lo, a.seed_hi, a.sample_ctr, row0 + tid, lo, hi);
    // target policy smoothing noise of (row, output) (tid - TM) % TM, (tid - TM) / TM: clamp(
    // policy_noise * eps, +-noise_clip) — threads past the sampling ones, so its f64 Box-Muller
    // runs on other waves (other SIMDs) than the sampling's Philox draw and gather
    static_assert(3 * TM <= kBlock, "sampling threads, then the noise's");
    float tnz = 0.f;
    const int tn = tid - TM;
    if (tn >= 0 && tn < 2 * TM && row0 + tn % TM < B) {
        const int64_t r = row0 + tn % TM;
        const int j = tn / TM;
        float e;
        if (a.eps) {
            e = a.eps[r * 2 + j];
        } else {
            const double2 z = gauss_pair(philox((uint32_t)r, 0u, NAV_TAG_TNOISE, a.noise_ctr,
                                                a.seed_lo, a.seed_hi));
            e = (float)(j == 0 ? z.x : z.y);
        }
        tnz = fminf(fmaxf(e * a.policy_noise, -a.noise_clip), a.noise_clip);
    }
    if (tid < TM) {
        const int64_t b = row0 + tid;
        if (b < B && blockIdx.y == 0) {  // split twins: one writer per batch row
            float4* dst = reinterpret_cast<float4*>(a.batch) + 2 * b;
            dst[0] = lo;
            dst[1] = hi;
        }
        *reinterpret_cast<float4*>(brow + tid * 8) = lo;
        *reinterpret_cast<float4*>(brow + tid * 8 + 4) = hi;
        *reinterpret_cast<float4*>(xin + tid * 4) = make_float4(hi.y, hi.z, 0.f, 0.f);  // s'
    }
    __syncthreads();
    NAV_MARK(1);
    // target actor; a' = clamp(pi'(s') + clamp(policy_noise * eps, +-noise_clip), +-max_action).
    // Each pass's layer-0 constants are loaded one pass ahead (L0Pre).
    f32x16 top[RT][2];
    const L0Pre l0_ct1 = load_l0<NT>(a.critic_t[0]);
    fwd_net<NT, RT, kPfWide, 2>(a.actor_t, act, stage, xin, red, nullptr, n_rt, nullptr, 0u, row0, B, rt0, top, 2,
                    &l0_at);
    if (tn >= 0 && tn < 2 * TM) {  // the noise's threads
        const int rloc = tn % TM, j = tn / TM;
        const int64_t r = row0 + rloc;
        float v = 0.f;
        if (r < B) {
            const float y = out_y<RT>(a.actor_t, red, rloc, j);
            v = y + tnz;
            v = fminf(fmaxf(v, -a.max_action), a.max_action);
        }
        xin[rloc * 4 + 2 + j] = v;
    }
    __syncthreads();
    NAV_MARK(8);
    // twin target critics on (s', a'), then y = r + gamma * min(q1', q2') * (1 - done), kept in
    // the row's thread
    const L0Pre l0_ct2 = load_l0<NT>(a.critic_t[1]);
    fwd_net<NT, RT, kPfWide, 4>(a.critic_t[0], act, stage, xin, red, nullptr, n_rt, nullptr, 0u, row0, B, rt0, top,
                    9, &l0_ct1);
    if (tid < TM) qv[tid] = out_y<RT>(a.critic_t[0], red, tid, 0);
    const int q0 = a.split_twins ? (int)blockIdx.y : 0;  // the first online critic of the block
    L0Pre l0_on = load_l0<NT>(a.critic[q0]);
    fwd_net<NT, RT, kPfWide, 4>(a.critic_t[1], act, stage, xin, red, nullptr, n_rt, nullptr, 0u, row0, B, rt0, top,
                    15, &l0_ct2);
    float yt = 0.f;
    if (tid < TM) {
        const float q2 = out_y<RT>(a.critic_t[1], red, tid, 0);
        const float rw = brow[tid * 8 + 4], dn = brow[tid * 8 + 7];
        yt = rw + (a.gamma * fminf(qv[tid], q2)) * (1.0f - dn);
        *reinterpret_cast<float4*>(xin + tid * 4) = *reinterpret_cast<const float4*>(brow + tid * 8);
    }
    __syncthreads();
    NAV_MARK(21);
    // online critics on (s, a): both, or (split_twins) the one of this workgroup's grid row
#pragma unroll 1
    for (int q = 0; q < 2; ++q) {
        if (a.split_twins && q != (int)blockIdx.y) continue;  // workgroup-uniform
        uint32_t top_bits[RT * 2];
        WoCols wo;
        fwd_net<NT, RT, kPfWide, 4>(a.critic[q], act, stage, xin, red, a.masks[q], n_rt, a.acts[q], a.save_mask, row0,
                        B, rt0, top, 22 + 14 * q, &l0_on, top_bits, &wo);
        if (q == 0 && !a.split_twins) l0_on = load_l0<NT>(a.critic[1]);
        float* es = a.eslab[q] ? a.eslab[q] + (int64_t)blockIdx.x * a.ecount : nullptr;
        loss_epilogue<NT, RT>(a.critic[q], top, red, row0, B, yt, a.norm, a.dq[q],
                              a.loss_part[q] + blockIdx.x, es);
        __syncthreads();
        NAV_MARK(28 + 14 * q);
        if (a.row_backward) {
            if (tid < TM)
                *reinterpret_cast<float4*>(dys + tid * 4) =
                    make_float4(red[kWaves * TM + tid], 0.f, 0.f, 0.f);  // loss_epilogue's dq
            __syncthreads();
            bwd_net<NT, RT, kPfWide, CBM>(a.critic[q], act, stage, dys, xin, a.masks[q], n_rt, es, nullptr, a.dz[q],
                            a.dz_save_mask, row0, B, rt0, 29 + 14 * q, top_bits, &wo, false);
            __syncthreads();  // the next forward's layer 0 overwrites the rows
        }
        NAV_MARK(35 + 14 * q);
    }
    NAV_CLOCK(0, 1);
}

struct ActorRowsArgs {
    MlpDev actor, critic;
    int64_t B;
    const float* rows;
    int64_t rsize;
    const int64_t* idx;
    uint32_t seed_lo, seed_hi, sample_ctr;
    float dq;            // d(-mean Q)/dQ = -1/B
    float* batch;        // [B][8] sampled rows
    float* q;            // [B] Q1(s, pi(s)), nullable
    float* da;           // [B][2] dL/da
    float* acts;         // actor [nh][B][hp], save_mask layers (the top one feeds dWo)
    uint32_t save_mask;
    float* dz;           // actor [nh][B][hp], dz_save_mask layers
    uint32_t dz_save_mask;
    uint16_t* masks_a;
    uint16_t* masks_c;
    float* eslab;        // actor edge partials
    int64_t ecount;
    WarmList warm;       // set by the launcher
};

// train_actor (robot.py:382-390) for one block of TM batch rows: sample, actor forward,
// critic-1 forward on (s, pi(s)), backward of -mean(Q) through critic 1 to its action input
// (critic grads discarded, as zero_grad does), and the actor's row backward with its edge
// partials.
template <int NT, int RT, int CBM>
__global__ __launch_bounds__(kBlock, 1) void k_td3_actor_rows(ActorRowsArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    if (a.warm.n && (int)blockIdx.y >= a.warm.y0) {  // an L2 warmer row (small grids)
        warm_l2(a.warm);
        return;
    }
    constexpr int hp = NT * 32, SS = hp + 4, TM = RT * 32;
    const int tid = threadIdx.x;
    const int64_t B = a.B, row0 = (int64_t)blockIdx.x * TM, rt0 = (int64_t)blockIdx.x * RT;
    const int64_t n_rt = mask_rowtiles(B);
    float* act = smem;
    float* xin = act + TM * SS;      // [TM][4] (s, pi(s))
    float* red = xin + TM * 4;       // [2][PARTS][TM]
    float* dys = red + red_floats(TM);  // [TM][4] critic dy
    float* dys2 = dys + TM * 4;      // [TM][4] actor dy = dL/da
    _Float16* stage = reinterpret_cast<_Float16*>(dys2 + TM * 4);  // gemm_cols' split stage
    const L0Pre l0_a = load_l0<NT>(a.actor);  // in flight under the sampling
    NAV_CLOCK(1, 0);
    if (tid < TM) {
        const int64_t b = row0 + tid;
        float4 lo = make_float4(0.f, 0.f, 0.f, 0.f), hi = lo;
        if (b < B) {
            sample_row(a.rows, a.rsize, a.idx, a.seed_lo, a.seed_hi, a.sample_ctr, b, lo, hi);
            float4* dst = reinterpret_cast<float4*>(a.batch) + 2 * b;
            dst[0] = lo;
            dst[1] = hi;
        }
        *reinterpret_cast<float4*>(xin + tid * 4) = make_float4(lo.x, lo.y, 0.f, 0.f);  // s
        *reinterpret_cast<float4*>(dys + tid * 4) =
            make_float4(b < B ? a.dq : 0.f, 0.f, 0.f, 0.f);
    }
    __syncthreads();
    // the actor's top hidden layer stays in registers until dL/da is known (its dWo partials)
    f32x16 topa[RT][2];
    fwd_net<NT, RT, 1, 2>(a.actor, act, stage, xin, red, a.masks_a, n_rt, a.acts, a.save_mask, row0, B, rt0,
                    topa, -64, &l0_a);
    const L0Pre l0_c = load_l0<NT>(a.critic);  // in flight under the action epilogue
    if (tid < 2 * TM) {
        const int rloc = tid % TM, j = tid / TM;
        xin[rloc * 4 + 2 + j] = row0 + rloc < B ? out_y<RT>(a.actor, red, rloc, j) : 0.f;
    }
    __syncthreads();
    // the critic's top-layer ReLU bits and Wo columns go from its forward to its row backward in
    // registers (as in critic_rows)
    f32x16 top[RT][2];
    uint32_t top_bits[RT * 2];
    WoCols wo;
    fwd_net<NT, RT, 1, 4>(a.critic, act, stage, xin, red, a.masks_c, n_rt, nullptr, 0u, row0, B, rt0, top,
                    -64, &l0_c, top_bits, &wo);
    if (tid < TM && a.q && row0 + tid < B) a.q[row0 + tid] = out_y<RT>(a.critic, red, tid, 0);
    bwd_net<NT, RT, 1, CBM>(a.critic, act, stage, dys, xin, a.masks_c, n_rt, nullptr, nullptr,
                                    nullptr, 0u, row0, B, rt0, -64, top_bits, &wo);
    if (tid < 2 * TM) {
        const int rloc = tid % TM, j = tid / TM;
        const int64_t r = row0 + rloc;
        const float v = r < B ? dx_unit<NT>(a.critic, act, rloc, 2 + j) : 0.f;
        dys2[rloc * 4 + j] = v;
        if (r < B) a.da[r * 2 + j] = v;
    }
    if (tid < TM) {
        dys2[tid * 4 + 2] = 0.f;
        dys2[tid * 4 + 3] = 0.f;
    }
    __syncthreads();
    // the actor's output layer gradient partials: dWo from its top-layer registers, dbo = column
    // sums of dL/da (bwd_net's order)
    float* es = a.eslab + (int64_t)blockIdx.x * a.ecount;
    wo_grad_regs<NT, RT>(a.actor, topa, dys2, 4, es);
    if (tid < 4) {
        float sb = 0.f;
        if (tid < a.actor.d_out)
            for (int rr = 0; rr < TM; ++rr) sb += dys2[rr * 4 + tid];
        es[e_bo(a.actor) + tid] = sb;
    }
    bwd_net<NT, RT>(a.actor, act, stage, dys2, xin, a.masks_a, n_rt, es, nullptr, a.dz, a.dz_save_mask,
                    row0, B, rt0, -64, nullptr, nullptr, false);
    NAV_CLOCK(1, 1);
}


// ---- launch helpers (template dispatch on NT = hp / 32 and RT = rows / 32) ----
// Workgroup height: RT = 2 (64 rows, two workgroups per CU so one workgroup's epilogue overlaps
// the other's MFMA loop; RT = 4, 128 rows and one workgroup per CU, measured slower in round 1:
// profiles/r01c_micro_rt4.json, no longer built).
// Small batches take RT = 1 (32-row workgroups): at M <= kSmallRows the 64-row grid leaves CUs
// idle (config 1's 100 rows: 2 workgroups), and a 32-row block halves each wave's MFMA chain per
// layer, so the latency-bound small-batch learner runs twice the workgroups at half the chain.
// Not for the fused tick (its demo pass works on whole waves of envs).
constexpr int64_t kSmallRows = 16384;
int row_tiles_for(int64_t M, bool tick) { return (!tick && M <= kSmallRows) ? 1 : 2; }

// The row kernels (forward, row backward, critic_rows, actor_rows) are instantiated per NT in
// their own objects (this file built with NAV_MLP_PART = NT, see the Makefile) so the heavy
// template instantiations compile in parallel; the main object (NAV_MLP_PART = 0) dispatches to
// them through nav_mlp_rows_<NT>(). Argument structs travel as const void* (same definitions).
enum { FAM_FWD = 0, FAM_BWD = 1, FAM_CRITIC = 2, FAM_ACTOR = 3 };

}  // namespace

#define NAV_ROWS_DECL(NT_)                                                                   \
    int nav_mlp_rows_##NT_(int fam, int rt, int in_mode, int out_mode, const void* args,      \
                           int n_nets, hipStream_t st);
NAV_ROWS_DECL(1) NAV_ROWS_DECL(2) NAV_ROWS_DECL(3) NAV_ROWS_DECL(4)
NAV_ROWS_DECL(5) NAV_ROWS_DECL(6) NAV_ROWS_DECL(7) NAV_ROWS_DECL(8)
#undef NAV_ROWS_DECL

#if NAV_MLP_PART > 0
namespace {
template <int NT, int RT, int IN_MODE, int OUT_MODE>
void launch_fwd_k(const FwdArgs& a, int n_nets, hipStream_t st) {
    const size_t lds = lds_bytes(NT * 32, RT * 32);
    auto k = k_mlp_fwd<NT, RT, IN_MODE, OUT_MODE>;
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
    const dim3 grid((unsigned)((a.M + RT * 32 - 1) / (RT * 32)), (unsigned)n_nets);
    hipLaunchKernelGGL(k, grid, dim3(kBlock), lds, st, a);
}

template <int NT, int RT>
void launch_bwd_k(const BwdArgs& a, int n_nets, hipStream_t st) {
    const size_t lds = lds_bytes(NT * 32, RT * 32);
    // d_out = 1 networks' top backward image is the Wt image: their top product is gemm_bits
    const int nh = a.net[0].n_hidden;
    auto k = a.net[0].d_out != 1 || nh < 2 ? k_mlp_bwd<NT, RT, 0>
             : nh == 2                      ? k_mlp_bwd<NT, RT, 2>
                                            : k_mlp_bwd<NT, RT, 1>;
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
    const dim3 grid((unsigned)((a.M + RT * 32 - 1) / (RT * 32)), (unsigned)n_nets);
    hipLaunchKernelGGL(k, grid, dim3(kBlock), lds, st, a);
}

template <int NT, int RT>
void launch_critic_rows_k(const CriticRowsArgs& a, hipStream_t st) {
    constexpr int TM = RT * 32;
    const size_t lds =
        ((size_t)TM * (NT * 32 + 4) + TM * 4 + red_floats(TM) + TM * 8 + TM + TM * 4) * 4 +
        stage_bytes(TM, NT * 32);
    // form 1 also for 2 hidden layers (its gemm_cols loop then runs no layer): the form-2
    // instantiation came out at 286 registers (one workgroup per CU), form 1 at 236
    auto k = a.critic[0].n_hidden == 1 ? k_td3_critic_rows<NT, RT, 0> : k_td3_critic_rows<NT, RT, 1>;
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
    const unsigned gx = (unsigned)((a.B + TM - 1) / TM), gy = a.split_twins ? 2u : 1u;
    // the images in the order the compute workgroups consume them (targets: forward only)
    CriticRowsArgs w = a;
    w.warm = WarmList{};
    bool ok = kWarmL2 && warm_net(w.warm, a.actor_t, true) && warm_net(w.warm, a.critic_t[0], true) &&
              warm_net(w.warm, a.critic_t[1], true) && warm_net(w.warm, a.critic[0], false) &&
              warm_net(w.warm, a.critic[1], false);
    if (!ok) w.warm.n = 0;
    w.warm.y0 = (int)gy;
    const unsigned wy = warm_rows(w.warm, gx, gy);
    if (wy == 0) w.warm.n = 0;
    hipLaunchKernelGGL(k, dim3(gx, gy + wy), dim3(kBlock), lds, st, w);
}

template <int NT, int RT>
void launch_actor_rows_k(const ActorRowsArgs& a, hipStream_t st) {
    constexpr int TM = RT * 32;
    const size_t lds = ((size_t)TM * (NT * 32 + 4) + TM * 4 + red_floats(TM) + TM * 8) * 4 +
                       stage_bytes(TM, NT * 32);
    auto k = a.critic.n_hidden == 1 ? k_td3_actor_rows<NT, RT, 0> : k_td3_actor_rows<NT, RT, 1>;
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
    const unsigned gx = (unsigned)((a.B + TM - 1) / TM);
    ActorRowsArgs w = a;
    w.warm = WarmList{};
    const bool ok = kWarmL2 && warm_net(w.warm, a.actor, false) && warm_net(w.warm, a.critic, false);
    if (!ok) w.warm.n = 0;
    w.warm.y0 = 1;
    const unsigned wy = warm_rows(w.warm, gx, 1u);
    if (wy == 0) w.warm.n = 0;
    hipLaunchKernelGGL(k, dim3(gx, 1u + wy), dim3(kBlock), lds, st, w);
}

template <int RT>
int rows_rt(int fam, int in_mode, int out_mode, const void* args, int n_nets, hipStream_t st) {
    constexpr int NT = NAV_MLP_PART;
    switch (fam) {
        case FAM_FWD: {
            const FwdArgs& a = *static_cast<const FwdArgs*>(args);
            if (in_mode == IN_BASELINE && out_mode == OUT_ACT)
                launch_fwd_k<NT, RT, IN_BASELINE, OUT_ACT>(a, n_nets, st);
            else if (in_mode == IN_BASELINE && out_mode == OUT_TICK) {
                if constexpr (RT >= 2)
                    launch_fwd_k<NT, RT, IN_BASELINE, OUT_TICK>(a, n_nets, st);
                else
                    return NAV_EINVAL;
            } else if (in_mode == IN_F32 && out_mode == OUT_F32)
                launch_fwd_k<NT, RT, IN_F32, OUT_F32>(a, n_nets, st);
            else if (in_mode == IN_F32 && out_mode == OUT_TARGET)
                launch_fwd_k<NT, RT, IN_F32, OUT_TARGET>(a, n_nets, st);
            else if (in_mode == IN_F32 && out_mode == OUT_LOSS)
                launch_fwd_k<NT, RT, IN_F32, OUT_LOSS>(a, n_nets, st);
            else
                return NAV_EINVAL;
            return 0;
        }
        case FAM_BWD: launch_bwd_k<NT, RT>(*static_cast<const BwdArgs*>(args), n_nets, st); return 0;
        case FAM_CRITIC:
            launch_critic_rows_k<NT, RT>(*static_cast<const CriticRowsArgs*>(args), st);
            return 0;
        case FAM_ACTOR:
            launch_actor_rows_k<NT, RT>(*static_cast<const ActorRowsArgs*>(args), st);
            return 0;
        default: return NAV_EINVAL;
    }
}

}  // namespace

#define NAV_CAT2(a, b) a##b
#define NAV_CAT(a, b) NAV_CAT2(a, b)
int NAV_CAT(nav_mlp_rows_, NAV_MLP_PART)(int fam, int rt, int in_mode, int out_mode,
                                           const void* args, int n_nets, hipStream_t st) {
    return rt == 1 ? rows_rt<1>(fam, in_mode, out_mode, args, n_nets, st)
                   : rows_rt<2>(fam, in_mode, out_mode, args, n_nets, st);
}

// (a trace variant builds one part with NAV_PHASE_TRACE: tools/build_variant.sh)
#if defined(NAV_PHASE_TRACE)
extern "C" int nav_phase_trace_read(unsigned long long* host, int n) {
    const size_t bytes = sizeof(g_phase_trace);
    if (!host || (size_t)n * sizeof(unsigned long long) < bytes) return NAV_EINVAL;
    const hipError_t e = hipMemcpyFromSymbol(host, HIP_SYMBOL(g_phase_trace), bytes);
    return e == hipSuccess ? 0 : -(int)e;
}
#endif

#if defined(NAV_CLOCK_STAMP) && NAV_MLP_PART == 8
extern "C" int nav_clock_stamp_read(unsigned long long* host, int n) {
    const size_t bytes = sizeof(g_clock_stamp);
    if (!host || (size_t)n * sizeof(unsigned long long) < bytes) return NAV_EINVAL;
    const hipError_t e = hipMemcpyFromSymbol(host, HIP_SYMBOL(g_clock_stamp), bytes);
    return e == hipSuccess ? 0 : -(int)e;
}
#endif

#else  // NAV_MLP_PART == 0

namespace {

// hp / 32 -> the per-NT object
int rows_dispatch(int hp, int fam, int in_mode, int out_mode, const void* args, int n_nets,
                  int64_t M, hipStream_t st) {
    const int rt = row_tiles_for(M, fam == FAM_FWD && out_mode == OUT_TICK);
    int r;
    switch (hp / 32) {
        case 1: r = nav_mlp_rows_1(fam, rt, in_mode, out_mode, args, n_nets, st); break;
        case 2: r = nav_mlp_rows_2(fam, rt, in_mode, out_mode, args, n_nets, st); break;
        case 3: r = nav_mlp_rows_3(fam, rt, in_mode, out_mode, args, n_nets, st); break;
        case 4: r = nav_mlp_rows_4(fam, rt, in_mode, out_mode, args, n_nets, st); break;
        case 5: r = nav_mlp_rows_5(fam, rt, in_mode, out_mode, args, n_nets, st); break;
        case 6: r = nav_mlp_rows_6(fam, rt, in_mode, out_mode, args, n_nets, st); break;
        case 7: r = nav_mlp_rows_7(fam, rt, in_mode, out_mode, args, n_nets, st); break;
        case 8: r = nav_mlp_rows_8(fam, rt, in_mode, out_mode, args, n_nets, st); break;
        default: return NAV_EINVAL;
    }
    if (r) return r;
    NAV_CHECK_LAUNCH();
    return 0;
}

template <int IN_MODE, int OUT_MODE>
int launch_fwd(const FwdArgs& a, int n_nets, hipStream_t st) {
    return rows_dispatch(a.net[0].hp, FAM_FWD, IN_MODE, OUT_MODE, &a, n_nets, a.M, st);
}

int launch_bwd(const BwdArgs& a, int n_nets, hipStream_t st) {
    return rows_dispatch(a.net[0].hp, FAM_BWD, 0, 0, &a, n_nets, a.M, st);
}

#define NAV_ROWS_SWITCH(HP, FAM, ARGS, ST)                                                  \
    {                                                                                       \
        const int r_ = rows_dispatch((HP), (FAM), 0, 0, &(ARGS), 1, (ARGS).B, (ST));        \
        if (r_) return r_;                                                                  \
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
    return (int64_t)(n_hidden - 1) * 2 * split_image_floats(hp);
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

int nav_act_tick(const nav_params* p, const nav_mlp* actor, const nav_env_soa* env,
                 const float* field, const double* noise_z, uint32_t step, int32_t mode,
                 const nav_replay* replay, int64_t replay_base, const nav_step_out* out,
                 const double* demo_xy, const int64_t* demo_off, int32_t envs_per_group,
                 const int64_t* cell_start, const int32_t* cand, double* action_out,
                 double* reward_out, void* stream) {
    FwdArgs a{};
    if (!p || !env || !make_dev(actor, &a.net[0]) || actor->d_in != 2 || actor->d_out != 2 ||
        (mode != 0 && mode != 1) || !field || !replay || !replay->rows || !out ||
        env->n < 0 || env->n >= ((int64_t)1 << 31) || replay->capacity < env->n ||
        replay->capacity <= 0 || replay_base < 0 || (demo_off && envs_per_group <= 0))
        return NAV_EINVAL;
    if (env->n == 0) return 0;
    if (!env->state || !env->goal || !env->region || !env->hist || !env->meta ||
        !env->plan_index || !env->path_length || !env->episodes || !env->noise_scale)
        return NAV_EINVAL;
    const bool demo = demo_xy != nullptr;
    if (demo && (!cell_start || !cand)) return NAV_EINVAL;
    a.M = env->n;
    a.state = env->state;
    a.goal = env->goal;
    a.noise_scale = env->noise_scale;
    a.noise_z = noise_z;
    a.step = step;
    a.act_mode = mode;
    a.max_action_d = p->max_action;
    a.action_out = action_out;
    a.p = *p;
    a.env = *env;
    a.field = reinterpret_cast<const float2*>(field);
    a.rows = reinterpret_cast<float4*>(replay->rows);
    a.cap = replay->capacity;
    a.base = replay_base % replay->capacity;
    a.sout = *out;
    if (demo)
        a.demo = DemoIdx{reinterpret_cast<const double2*>(demo_xy), demo_off,
                         envs_per_group > 0 ? envs_per_group : 1, cell_start, cand};
    a.reward_out = reward_out;
    return launch_fwd<IN_BASELINE, OUT_TICK>(a, 1, S(stream));
}

int nav_mlp_forward(const nav_mlp* nets, int32_t n_nets, int64_t M, const float* in,
                    int32_t ld_in, int32_t in_col, float* const* out, int32_t ld_out,
                    int32_t out_col, int32_t out_mode, const float* eps, float policy_noise,
                    float noise_clip, float max_action, uint32_t seed_lo, uint32_t seed_hi,
                    uint32_t counter, float* const* acts, uint32_t save_mask,
                    uint16_t* const* masks, void* stream) {
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
    a.save_mask = save_mask;
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

int64_t nav_mlp_row_blocks(int64_t M) {
    if (M < 0) return NAV_EINVAL;
    const int64_t tm = (int64_t)row_tiles_for(M, false) * 32;
    return (M + tm - 1) / tm;
}

int64_t nav_mlp_edge_count(int32_t d_in, int32_t d_out, int32_t hidden_pad, int32_t n_hidden) {
    nav_mlp n{d_in, d_out, hidden_pad, hidden_pad, n_hidden, reinterpret_cast<float*>(16),
              reinterpret_cast<float*>(16)};
    MlpDev d;
    if (!make_dev(&n, &d)) return NAV_EINVAL;
    return edge_count(d);
}

int64_t nav_mlp_hidden_count(int32_t hidden_pad, int32_t n_hidden) {
    if (hidden_pad < 32 || hidden_pad > 256 || (hidden_pad & 31) || n_hidden < 1)
        return NAV_EINVAL;
    return (int64_t)(n_hidden - 1) * hidden_pad * hidden_pad;
}

int nav_td3_critic_forward(const nav_mlp* nets, int64_t B, const float* in, int32_t ld_in,
                           int32_t in_col, const float* batch, const float* q1t, const float* q2t,
                           float gamma, float* const* dq, float* const* loss_part,
                           float* const* edge_slabs, float* const* acts, uint32_t save_mask,
                           uint16_t* const* masks, void* stream) {
    FwdArgs a{};
    if (!nets || B < 1 || !in || !batch || !q1t || !q2t || !dq || !loss_part || !masks)
        return NAV_EINVAL;
    for (int i = 0; i < 2; ++i) {
        if (!make_dev(&nets[i], &a.net[i]) || nets[i].d_out != 1 || !dq[i] || !loss_part[i] ||
            !masks[i])
            return NAV_EINVAL;
        if (a.net[i].hp != a.net[0].hp || a.net[i].d_in != a.net[0].d_in ||
            a.net[i].n_hidden != a.net[0].n_hidden)
            return NAV_EINVAL;
        a.out[i] = dq[i];  // unused by OUT_LOSS, non-null for uniformity
        a.acts[i] = acts ? acts[i] : nullptr;
        if (save_mask && !a.acts[i]) return NAV_EINVAL;
        a.masks[i] = masks[i];
        a.dq[i] = dq[i];
        a.loss_part[i] = loss_part[i];
        a.eslab[i] = edge_slabs ? edge_slabs[i] : nullptr;
    }
    if (in_col < 0 || in_col + a.net[0].d_in > ld_in) return NAV_EINVAL;
    a.M = B;
    a.in = in;
    a.ld_in = ld_in;
    a.in_col = in_col;
    a.save_mask = save_mask;
    a.batch = batch;
    a.qt[0] = q1t;
    a.qt[1] = q2t;
    a.gamma = gamma;
    a.norm = (float)(2.0 / (double)B);
    a.ecount = edge_count(a.net[0]);
    return launch_fwd<IN_F32, OUT_LOSS>(a, 2, S(stream));
}

int nav_td3_critic_rows(const nav_mlp* target_actor, const nav_mlp* target_critics,
                        const nav_mlp* critics, const nav_replay* replay, int64_t size,
                        int64_t B, const int64_t* idx, uint32_t seed_lo, uint32_t seed_hi,
                        uint32_t counter, const float* eps, float policy_noise,
                        float noise_clip, float max_action, float gamma, float* batch,
                        float* const* dq, float* const* loss_part, float* const* edge_slabs,
                        float* const* acts, uint32_t save_mask, uint16_t* const* masks,
                        int32_t row_backward, float* const* dz, uint32_t dz_save_mask,
                        int32_t split_twins, void* stream) {
    CriticRowsArgs a{};
    if (row_backward && dz_save_mask && !dz) return NAV_EINVAL;
    if (!target_actor || !target_critics || !critics || !replay || !replay->rows || B < 1 ||
        size < 1 || size > replay->capacity || size > ((int64_t)1 << 32) || !batch || !dq ||
        !loss_part || !masks || !make_dev(target_actor, &a.actor_t) || target_actor->d_in != 2 ||
        target_actor->d_out != 2)
        return NAV_EINVAL;
    for (int i = 0; i < 2; ++i) {
        if (!make_dev(&target_critics[i], &a.critic_t[i]) || !make_dev(&critics[i], &a.critic[i]) ||
            critics[i].d_in != 4 || critics[i].d_out != 1 || target_critics[i].d_in != 4 ||
            target_critics[i].d_out != 1 || !dq[i] || !loss_part[i] || !masks[i])
            return NAV_EINVAL;
        if (a.critic_t[i].hp != a.actor_t.hp || a.critic[i].hp != a.actor_t.hp ||
            a.critic[i].n_hidden != a.critic[0].n_hidden)
            return NAV_EINVAL;
        a.dq[i] = dq[i];
        a.loss_part[i] = loss_part[i];
        a.eslab[i] = edge_slabs ? edge_slabs[i] : nullptr;
        a.acts[i] = acts ? acts[i] : nullptr;
        if (save_mask && !a.acts[i]) return NAV_EINVAL;
        a.masks[i] = masks[i];
        a.dz[i] = dz ? dz[i] : nullptr;
        if (row_backward && ((dz_save_mask && !a.dz[i]) ||
                             (dz_save_mask >> critics[i].n_hidden)))
            return NAV_EINVAL;
    }
    a.row_backward = row_backward ? 1 : 0;
    a.dz_save_mask = row_backward ? dz_save_mask : 0u;
    // Small batches leave most CUs idle and each workgroup's chain of network passes sets the
    // time: the twin online critics then run in separate workgroups (grid.y = 2), each repeating
    // the sampling, target actor and twin target critics (identical values) — 5 instead of 7
    // passes per workgroup. split_twins < 0 picks that form for B <= 2048 (profiles/r02aq).
    a.split_twins = split_twins < 0 ? (B <= 2048 ? 1 : 0) : (split_twins ? 1 : 0);
    a.B = B;
    a.rows = replay->rows;
    a.rsize = size;
    a.idx = idx;
    a.seed_lo = seed_lo;
    a.seed_hi = seed_hi;
    a.sample_ctr = 2u * counter;  // the actor's batch of the same epoch uses 2*counter + 1
    a.noise_ctr = counter;
    a.eps = eps;
    a.policy_noise = policy_noise;
    a.noise_clip = noise_clip;
    a.max_action = max_action;
    a.gamma = gamma;
    a.norm = (float)(2.0 / (double)B);
    a.batch = batch;
    a.ecount = edge_count(a.critic[0]);
    a.save_mask = save_mask;
    NAV_ROWS_SWITCH(a.actor_t.hp, FAM_CRITIC, a, S(stream))
    NAV_CHECK_LAUNCH();
    return 0;
}

int nav_td3_actor_rows(const nav_mlp* actor, const nav_mlp* critic, const nav_replay* replay,
                       int64_t size, int64_t B, const int64_t* idx, uint32_t seed_lo,
                       uint32_t seed_hi, uint32_t counter, float* batch, float* q, float* da,
                       float* acts, uint32_t save_mask, float* dz, uint32_t dz_save_mask,
                       uint16_t* masks_actor, uint16_t* masks_critic, float* edge_slabs,
                       void* stream) {
    ActorRowsArgs a{};
    if (!actor || !critic || !replay || !replay->rows || B < 1 || size < 1 ||
        size > replay->capacity || size > ((int64_t)1 << 32) || !batch || !da ||
        (save_mask && !acts) || !masks_actor || !masks_critic || !edge_slabs ||
        !make_dev(actor, &a.actor) || !make_dev(critic, &a.critic) || actor->d_in != 2 ||
        actor->d_out != 2 || critic->d_in != 4 || critic->d_out != 1 ||
        a.actor.hp != a.critic.hp || (save_mask >> actor->n_hidden) ||
        (dz_save_mask && !dz) || (dz_save_mask >> actor->n_hidden))
        return NAV_EINVAL;
    a.B = B;
    a.rows = replay->rows;
    a.rsize = size;
    a.idx = idx;
    a.seed_lo = seed_lo;
    a.seed_hi = seed_hi;
    a.sample_ctr = 2u * counter + 1u;
    a.dq = (float)(-1.0 / (double)B);
    a.batch = batch;
    a.q = q;
    a.da = da;
    a.acts = acts;
    a.save_mask = save_mask;
    a.dz = dz;
    a.dz_save_mask = dz_save_mask;
    a.masks_a = masks_actor;
    a.masks_c = masks_critic;
    a.eslab = edge_slabs;
    a.ecount = edge_count(a.actor);
    NAV_ROWS_SWITCH(a.actor.hp, FAM_ACTOR, a, S(stream))
    NAV_CHECK_LAUNCH();
    return 0;
}

int64_t nav_mlp_mask_count(int32_t hidden_pad, int32_t n_hidden, int64_t M) {
    if (hidden_pad < 32 || hidden_pad > 256 || (hidden_pad & 31) || n_hidden < 1 || M < 0)
        return NAV_EINVAL;
    return (int64_t)n_hidden * mask_rowtiles(M) * (hidden_pad / 32) * 64;
}

int nav_mlp_backward(const nav_mlp* nets, int32_t n_nets, int64_t M, const float* const* dy,
                     int32_t ld_dy, const uint16_t* const* masks, const float* in, int32_t ld_in,
                     int32_t in_col, const float* const* h_top, float* const* dz,
                     uint32_t save_mask, float* const* dx, float* const* edge_slabs,
                     void* stream) {
    BwdArgs a{};
    if (!nets || n_nets < 1 || n_nets > 2 || M < 0 || ld_dy < 0 || !dy || !masks) return NAV_EINVAL;
    bool any_edges = false;
    for (int i = 0; i < n_nets; ++i) {
        if (!make_dev(&nets[i], &a.net[i])) return NAV_EINVAL;
        if (a.net[i].hp != a.net[0].hp || a.net[i].d_in != a.net[0].d_in ||
            a.net[i].n_hidden != a.net[0].n_hidden || a.net[i].d_out != a.net[0].d_out)
            return NAV_EINVAL;
        a.dy[i] = dy[i];
        a.masks[i] = masks[i];
        a.h_top[i] = h_top ? h_top[i] : nullptr;
        a.dz[i] = dz ? dz[i] : nullptr;
        a.dx[i] = dx ? dx[i] : nullptr;
        a.eslab[i] = edge_slabs ? edge_slabs[i] : nullptr;
        if (M > 0 && (!a.dy[i] || !a.masks[i] || (save_mask && !a.dz[i]))) return NAV_EINVAL;
        any_edges = any_edges || a.eslab[i];
    }
    if (M == 0) return 0;
    if ((save_mask >> a.net[0].n_hidden) ||
        (any_edges && (!in || in_col < 0 || in_col + a.net[0].d_in > ld_in)))
        return NAV_EINVAL;
    a.M = M;
    a.ld_dy = ld_dy;
    a.in = in;
    a.ld_in = ld_in;
    a.in_col = in_col;
    a.save_mask = save_mask;
    a.ecount = edge_count(a.net[0]);
    return launch_bwd(a, n_nets, S(stream));
}

}  // extern "C"

#endif  // NAV_MLP_PART
