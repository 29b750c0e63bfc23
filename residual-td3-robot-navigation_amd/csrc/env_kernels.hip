// env_kernels.hip — the vectorised Environment (environment.py) and the Robot's per-step tick
// (robot.py) as gfx950 kernels: one env per lane, structure-of-arrays state in HBM, f64 state
// math (the reference's robot_state is float64), reward/done counts reduced per block through
// wave shuffles and LDS.
#include <stdlib.h>

#include "nav_tick.h"

using namespace nav;

namespace {

NAV_DEV void region_of(int r, double u, double* reg) {
    // environment.py:29-49 (left, right, bottom, top)
    const double W = 100.0, S = 25.0;
    const double v = 0.0 + (W - S - 0.0) * u;
    double l, rr, b, t;
    if (r == 0) { l = 0.0; rr = S; b = v; t = b + S; }
    else if (r == 1) { l = v; rr = l + S; b = W - S; t = W; }
    else if (r == 2) { l = W - S; rr = W; b = v; t = b + S; }
    else { l = v; rr = l + S; b = 0.0; t = S; }
    reg[0] = l; reg[1] = rr; reg[2] = b; reg[3] = t;
}

__global__ __launch_bounds__(kBlock) void k_env_init(nav_params p, nav_env_soa env, int32_t epg,
                                                     int32_t demo_flag, int32_t* draws_out) {
    const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (e >= env.n) return;
    const uint32_t sid = (uint32_t)(e / epg);
    // environment.py:28-56 on the Philox stream (NAV_TAG_INIT, stream id)
    uint4 w = philox(0u, sid, NAV_TAG_INIT, 0u, p.seed_lo, p.seed_hi);
    double reg[4];
    region_of((int)(w.x & 3u), u01(w.z, w.w), reg);
    const double mx = 0.5 * (reg[0] + reg[1]), my = 0.5 * (reg[2] + reg[3]);
    double gx = 0.0, gy = 0.0;
    int32_t used = 0;
    for (int k = 1; k <= p.max_goal_draws; ++k) {
        w = philox((uint32_t)k, sid, NAV_TAG_INIT, 0u, p.seed_lo, p.seed_hi);
        gx = 5.0 + 90.0 * u01(w.x, w.y);
        gy = 5.0 + 90.0 * u01(w.z, w.w);
        if (norm2(gx - mx, gy - my) >= 90.0) { used = k; break; }
    }
    reinterpret_cast<double2*>(env.goal)[e] = make_double2(gx, gy);
    double4* rg = reinterpret_cast<double4*>(env.region);
    rg[e] = make_double4(reg[0], reg[1], reg[2], reg[3]);
    // Robot state at the first training step after 3 demos (robot.py:443-489 trace)
    const int32_t ep0 = 5;
    env.plan_index[e] = 5;
    env.path_length[e] = p.path_length0;
    env.episodes[e] = ep0;
    env.noise_scale[e] = 1.0;  // robot.py:32 INITIAL_NOISE
    env.meta[e] = demo_flag ? M_DEMO : 0u;
    // environment.py:130-137 first reset on the reset stream of this env
    w = philox(0u, (uint32_t)e, NAV_TAG_RESET, (uint32_t)ep0, p.seed_lo, p.seed_hi);
    reinterpret_cast<double2*>(env.state)[e] = region_sample(reg, u01(w.x, w.y), u01(w.z, w.w));
    if (draws_out) draws_out[e] = used;
}

__global__ __launch_bounds__(kBlock) void k_env_reset(nav_params p, nav_env_soa env,
                                                      const uint8_t* mask, const double2* uni) {
    const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (e >= env.n) return;
    if (mask && !mask[e]) return;
    double u0, u1;
    if (uni) {
        const double2 u = uni[e];
        u0 = u.x; u1 = u.y;
    } else {
        const uint4 w = philox(0u, (uint32_t)e, NAV_TAG_RESET, (uint32_t)env.episodes[e],
                               p.seed_lo, p.seed_hi);
        u0 = u01(w.x, w.y); u1 = u01(w.z, w.w);
    }
    const double4 r = reinterpret_cast<const double4*>(env.region)[e];
    const double reg[4] = {r.x, r.y, r.z, r.w};
    reinterpret_cast<double2*>(env.state)[e] = region_sample(reg, u0, u1);
}

template <bool NT>
__global__ __launch_bounds__(kBlock) void k_env_step(int64_t n, double2* __restrict__ state,
                                                     const float2* __restrict__ field,
                                                     const double2* __restrict__ action,
                                                     double2* __restrict__ next_out) {
    // environment.py:122-127: 16 B state in, 16 B action in, 16 B state out per env
    const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (e >= n) return;
    double2 s, a;
    if (NT) {
        s.x = __builtin_nontemporal_load(&state[e].x);
        s.y = __builtin_nontemporal_load(&state[e].y);
        a.x = __builtin_nontemporal_load(&action[e].x);
        a.y = __builtin_nontemporal_load(&action[e].y);
    } else {
        s = state[e];
        a = action[e];
    }
    const double2 nx = dynamics(field, s, a);
    const bool ok = in_world(nx);
    if (NT) {
        if (ok) {
            __builtin_nontemporal_store(nx.x, &state[e].x);
            __builtin_nontemporal_store(nx.y, &state[e].y);
        }
    } else if (ok) {
        state[e] = nx;
    }
    if (next_out) next_out[e] = ok ? nx : s;
}

__global__ __launch_bounds__(kBlock) void k_dynamics(int64_t n, const float2* __restrict__ field,
                                                     const double2* __restrict__ s,
                                                     const double2* __restrict__ a,
                                                     double2* __restrict__ out) {
    const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (e >= n) return;
    out[e] = dynamics(field, s[e], a[e]);
}

// Robot.check_if_stuck alone (robot.py:509-538): history ring update + stuck verdict.
__global__ __launch_bounds__(kBlock) void k_check_if_stuck(nav_params p, nav_env_soa env,
                                                           const double2* __restrict__ st,
                                                           uint8_t* __restrict__ stuck_out) {
    const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (e >= env.n) return;
    double2* hist = reinterpret_cast<double2*>(env.hist);
    const double2 s = st[e];
    const uint32_t meta = env.meta[e];
    int cnt = (int)((meta >> 8) & 7u), head = (int)((meta >> 12) & 7u);
    bool stuck = false;
    if (cnt >= NAV_HIST) {
        bool all = true;
        for (int k = 0; k < NAV_HIST; ++k) {
            const double2 h = hist[(int64_t)k * env.n + e];
            all = all && (norm2(s.x - h.x, s.y - h.y) < p.stuck_threshold);
        }
        if (all) {
            stuck = true;
            cnt = 0;
        } else {
            head = head == NAV_HIST - 1 ? 0 : head + 1;
            cnt -= 1;
        }
    }
    int sl = head + cnt;
    if (sl >= NAV_HIST) sl -= NAV_HIST;
    hist[(int64_t)sl * env.n + e] = s;
    cnt += 1;
    env.meta[e] = (meta & 0xffu) | ((uint32_t)cnt << 8) | ((uint32_t)head << 12);
    stuck_out[e] = stuck ? 1 : 0;
}

// Robot.process_transition alone (the N = 1 drop-in's path): s, a, s' given by the caller.
__global__ __launch_bounds__(kBlock) void k_transition(nav_params p, nav_env_soa env,
                                                       const double2* __restrict__ st,
                                                       const double2* __restrict__ act,
                                                       const double2* __restrict__ nst,
                                                       float4* __restrict__ rows, int64_t cap,
                                                       int64_t base, nav_step_out out,
                                                       int32_t demo_pending) {
    const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (e >= env.n) return;
    const uint32_t meta = env.meta[e];
    const double2 s = st[e], a = act[e], ns = nst[e];
    const TransOut t = transition(p, env, e, s, a, ns, meta, env.plan_index[e],
                                  env.path_length[e], demo_pending != 0);
    push_row(rows, (base + e) % cap, s, a, t.r, ns, t.done);
    env.meta[e] = t.meta;
    if (out.next_state) reinterpret_cast<double2*>(out.next_state)[e] = nst[e];
    if (out.goal_term) out.goal_term[e] = t.gt;
    if (out.flags) out.flags[e] = flag_byte(t, false);
}

// robot.py:753 demo-proximity min distance, f64 exactly as scipy's cdist (dx*dx + dy*dy, no
// fma; sqrt is monotone and correctly rounded, so sqrt(min) == min(sqrt)). One wave = 64 envs of
// one group; every lane tests the same point at the same time, so the points are read with
// wave-uniform (scalar-unit) loads straight into SGPRs — no LDS staging, no bank traffic — and
// four independent min chains keep the f64 pipe busy. A workgroup = kDemoSplit waves over the
// SAME 64 envs, each scanning 1/kDemoSplit of the points (4 waves per SIMD hide the scalar-cache
// latency), combined through LDS.
constexpr int kDemoEnvs = 64;
constexpr int kDemoSplit = 8;
constexpr int kDemoBlock = kDemoEnvs * kDemoSplit;

NAV_DEV double demo_min_uniform(const double* __restrict__ d, int m, double x, double y) {
    double b0 = __builtin_inf(), b1 = b0, b2 = b0, b3 = b0;
    int j = 0;
    for (; j + 4 <= m; j += 4) {
        const double* q = d + 2 * j;
        const double v0 = sqd(x, y, q[0], q[1]), v1 = sqd(x, y, q[2], q[3]);
        const double v2 = sqd(x, y, q[4], q[5]), v3 = sqd(x, y, q[6], q[7]);
        // fmin == (v < b ? v : b) here: no NaN among the distances
        b0 = fmin(v0, b0);
        b1 = fmin(v1, b1);
        b2 = fmin(v2, b2);
        b3 = fmin(v3, b3);
    }
    for (; j < m; ++j) b0 = fmin(sqd(x, y, d[2 * j], d[2 * j + 1]), b0);
    return fmin(fmin(b0, b1), fmin(b2, b3));
}

__global__ __launch_bounds__(kDemoBlock) void k_demo_reward(nav_params p, int64_t n,
                                                            const double2* __restrict__ ns,
                                                            const double* __restrict__ gterm,
                                                            const uint8_t* __restrict__ flags,
                                                            const double* __restrict__ demo,
                                                            const int64_t* __restrict__ off,
                                                            int64_t m_shared, int32_t epg,
                                                            float* __restrict__ rows,
                                                            int64_t cap, int64_t base,
                                                            double* __restrict__ reward_out) {
    __shared__ double part[kDemoSplit][kDemoEnvs];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t e0 = (int64_t)blockIdx.x * kDemoEnvs;
    const int64_t e = e0 + lane;
    const bool live = e < n;
    const uint8_t f = live ? flags[e] : 0;
    const bool want = live && (f & F_DEMO);
    if (!__syncthreads_or(want ? 1 : 0)) return;
    double x = 0.0, y = 0.0;
    if (live) {
        const double2 s = ns[e];
        x = s.x;
        y = s.y;
    }
    const int64_t last = e0 + kDemoEnvs - 1 < n ? e0 + kDemoEnvs - 1 : n - 1;
    const int64_t g0 = off ? e0 / epg : 0, g1 = off ? last / epg : 0;
    double best;
    if (g0 == g1) {  // the 64 envs share one group: wave-uniform scalar loads
        const int64_t lo = off ? off[g0] : 0, hi = off ? off[g0 + 1] : m_shared;
        const int64_t m = hi - lo, per = (m + kDemoSplit - 1) / kDemoSplit;
        const int64_t a = lo + wv * per, b = a + per < hi ? a + per : hi;
        best = a < b ? demo_min_uniform(demo + 2 * a, (int)(b - a), x, y) : __builtin_inf();
    } else if (wv == 0) {
        const int64_t g = live ? e / epg : g0;
        best = demo_min_global(reinterpret_cast<const double2*>(demo) + off[g],
                               off[g + 1] - off[g], x, y);
    } else {
        best = __builtin_inf();
    }
    part[wv][lane] = best;
    __syncthreads();
    if (wv != 0 || !want) return;
#pragma unroll
    for (int k = 1; k < kDemoSplit; ++k) best = fmin(best, part[k][lane]);
    // robot.py:756-760 then the stuck penalty of robot.py:667-669
    const double mn = sqrt(best);
    double r = gterm[e] + p.demo_factor * (-mn);
    if (f & F_STUCK) r -= p.stuck_penalty;
    const int64_t slot = (base + e) % cap;
    rows[slot * NAV_ROW + 4] = (float)r;
    if (reward_out) reward_out[e] = r;
}

// The same for a handful of envs (the N = 1 drop-in's process_transition): one workgroup per env,
// its threads over the demonstration points (a lane per point instead of a lane per env), the
// minimum by wave shuffles and LDS — the same f64 minimum over the same set, so the same reward.
__global__ __launch_bounds__(kDemoBlock) void k_demo_reward_few(nav_params p,
                                                                const double2* __restrict__ ns,
                                                                const double* __restrict__ gterm,
                                                                const uint8_t* __restrict__ flags,
                                                                const double* __restrict__ demo,
                                                                const int64_t* __restrict__ off,
                                                                int64_t m_shared, int32_t epg,
                                                                float* __restrict__ rows,
                                                                int64_t cap, int64_t base,
                                                                double* __restrict__ reward_out) {
    __shared__ double part[kDemoBlock / 64];
    const int64_t e = blockIdx.x;
    const uint8_t f = flags[e];
    if (!(f & F_DEMO)) return;  // workgroup-uniform
    const double2 s = ns[e];
    const int64_t g = off ? e / epg : 0;
    const int64_t lo = off ? off[g] : 0, hi = off ? off[g + 1] : m_shared;
    double best = __builtin_inf();
    for (int64_t j = lo + threadIdx.x; j < hi; j += kDemoBlock)
        best = fmin(sqd(s.x, s.y, demo[2 * j], demo[2 * j + 1]), best);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) best = fmin(best, __shfl_xor(best, o, 64));
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = best;
    __syncthreads();
    if (threadIdx.x != 0) return;
#pragma unroll
    for (int k = 1; k < kDemoBlock / 64; ++k) best = fmin(best, part[k]);
    // robot.py:756-760 then the stuck penalty of robot.py:667-669 (k_demo_reward's order)
    const double mn = sqrt(best);
    double r = gterm[e] + p.demo_factor * (-mn);
    if (f & F_STUCK) r -= p.stuck_penalty;
    const int64_t slot = (base + e) % cap;
    rows[slot * NAV_ROW + 4] = (float)r;
    if (reward_out) reward_out[e] = r;
}

// Batched open-loop rollouts through Environment.dynamics (the CEM demonstrator's inner loop,
// environment.py:151-165): lane = path, T sequential steps, state carried in f64; paths [P][T+1][2]
// f64; reward (nullable) = -||f32(s_T) - goal|| as compute_reward on the float32 planning_paths
// row (environment.py:164, 182-183).
__global__ __launch_bounds__(kBlock) void k_rollout(const float2* __restrict__ field, int64_t P,
                                                    int32_t T, const double2* __restrict__ start,
                                                    const double2* __restrict__ actions,
                                                    double2* __restrict__ paths,
                                                    const double* __restrict__ goal,
                                                    double* __restrict__ reward) {
    const int64_t pth = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (pth >= P) return;
    double2 s = start[pth];
    paths[pth * (T + 1)] = s;
    for (int t = 0; t < T; ++t) {
        s = dynamics(field, s, actions[pth * T + t]);
        paths[pth * (T + 1) + t + 1] = s;
    }
    if (reward) {
        const double fx = (double)(float)s.x, fy = (double)(float)s.y;
        reward[pth] = -norm2(fx - goal[0], fy - goal[1]);
    }
}

// ---------------- batched CEM demonstrator (environment.py:140-179) ----------------
// n_prob independent CEM problems (one per group and demonstration), each P paths x T steps. One
// rollout launch per CEM iteration over every problem's paths (lane = path, state in f64 as the
// reference's planning_state), then one elite launch per iteration (workgroup = problem).
// Iteration 0 takes the +-5 actions drawn by np.random.choice, later ones
// a = mean[t] + std[t] * z in f64 (legacy normal = loc + scale * gauss) with z the standard
// normal draws; both are drawn on the host from each problem's numpy stream, in the reference's
// order, so the plans equal nav.Environment.get_demonstration's on the same stream.
__global__ __launch_bounds__(kBlock) void k_cem_rollout(const float2* __restrict__ field,
                                                        int32_t n_prob, int32_t P, int32_t T,
                                                        int32_t iter,
                                                        const double* __restrict__ region,
                                                        const double2* __restrict__ uni,
                                                        const double2* __restrict__ goal,
                                                        const double2* __restrict__ a0,
                                                        const double2* __restrict__ z,
                                                        const float2* __restrict__ mean,
                                                        const float2* __restrict__ stdv,
                                                        float2* __restrict__ actions,
                                                        float2* __restrict__ paths,
                                                        double* __restrict__ reward) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;  // problem * P + path
    if (i >= (int64_t)n_prob * P) return;
    const int64_t prob = i / P;
    // environment.py:150 get_random_robot_init_state (the same formula as nav_env_reset)
    const double* rg = region + 4 * prob;
    const double reg[4] = {rg[0], rg[1], rg[2], rg[3]};
    const double2 u = uni[prob];
    double2 s = region_sample(reg, u.x, u.y);
    const int64_t base = i * T;
    if (paths) paths[i * (T + 1)] = make_float2((float)s.x, (float)s.y);
    for (int t = 0; t < T; ++t) {
        double2 a;
        if (iter == 0) {
            a = a0[base + t];
        } else {
            const float2 m = mean[prob * T + t], sd = stdv[prob * T + t];
            const double2 zz = z[base + t];
            a = make_double2((double)m.x + (double)sd.x * zz.x, (double)m.y + (double)sd.y * zz.y);
        }
        actions[base + t] = make_float2((float)a.x, (float)a.y);  // planning_actions (float32)
        s = dynamics(field, s, a);
        if (paths) paths[i * (T + 1) + t + 1] = make_float2((float)s.x, (float)s.y);
    }
    // environment.py:164, 182-183 on the float32 planning_paths row
    const double2 g = goal[prob];
    reward[i] = -norm2((double)(float)s.x - g.x, (double)(float)s.y - g.y);
}

// ---------------- dynamics fields (environment.py:59-95 set_dynamics; nav.fields) ----------------
// nav.fields' construction on the device: per cell (i, j) of the x-major 100 x 100 grid the f64
// gradient noise of octave o at (i/100*o, j/100*o) from the unit gradient table g_o [o+1][o+1][2]
// (quintic fade, bilinear blend), speed cells = f32((n5 + .5 n10) + .25 n20), angle cells =
// f32(n5) (the same octave-5 values), each min-max normalised in f32 and the speed stretched by 1/(1 + exp(-10 (x - .5)))
// in f32 (the exp rounded from f64) — numpy's operation order, -ffp-contract=off. One 1024-thread workgroup (10 000 cells,
// block min / max in LDS); field out [100][100][2] (speed, angle) interleaved, the kernels'
// table layout.
constexpr int kFieldThreads = 1024;
NAV_DEV double grad_noise(const double* __restrict__ g, int oct, int i, int j) {
    const double x = ((double)i / 100.0) * oct, y = ((double)j / 100.0) * oct;
    const double xf = floor(x), yf = floor(y);
    const int x0 = (int)xf, y0 = (int)yf;
    const double fx = x - xf, fy = y - yf;
    const int w = oct + 1;
    auto dot = [&](int ix, int iy, double dx, double dy) {
        const double* v = g + ((int64_t)ix * w + iy) * 2;
        return v[0] * dx + v[1] * dy;
    };
    auto fade = [](double t) { return t * t * t * (t * (t * 6.0 - 15.0) + 10.0); };
    const double n00 = dot(x0, y0, fx, fy);
    const double n10 = dot(x0 + 1, y0, fx - 1.0, fy);
    const double n01 = dot(x0, y0 + 1, fx, fy - 1.0);
    const double n11 = dot(x0 + 1, y0 + 1, fx - 1.0, fy - 1.0);
    const double wx = fade(fx), wy = fade(fy);
    return (n00 * (1.0 - wx) + n10 * wx) * (1.0 - wy) + (n01 * (1.0 - wx) + n11 * wx) * wy;
}

NAV_DEV void block_minmax(float& mn, float& mx, float* red) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        mn = fminf(mn, __shfl_xor(mn, o, 64));
        mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    }
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) {
        red[2 * wv] = mn;
        red[2 * wv + 1] = mx;
    }
    __syncthreads();
    mn = red[0];
    mx = red[1];
    for (int w = 1; w < kFieldThreads / 64; ++w) {
        mn = fminf(mn, red[2 * w]);
        mx = fmaxf(mx, red[2 * w + 1]);
    }
}

__global__ __launch_bounds__(kFieldThreads) void k_fields(const double* __restrict__ g5,
                                                          const double* __restrict__ g10,
                                                          const double* __restrict__ g20,
                                                          float2* __restrict__ field) {
    constexpr int N = NAV_WORLD_CELLS * NAV_WORLD_CELLS;
    __shared__ float sp[N];
    __shared__ float an[N];
    __shared__ float red[2 * kFieldThreads / 64];
    float smn = __builtin_inff(), smx = -__builtin_inff(), amn = smn, amx = smx;
    for (int c = threadIdx.x; c < N; c += kFieldThreads) {
        const int i = c / NAV_WORLD_CELLS, j = c % NAV_WORLD_CELLS;
        // the angle's noise IS the speed's first term (environment.py:62 and :85: the same
        // PerlinNoise(octaves=5, seed) function), so one evaluation feeds both tables
        const double n5 = grad_noise(g5, 5, i, j);
        const double v = (n5 + 0.5 * grad_noise(g10, 10, i, j)) + 0.25 * grad_noise(g20, 20, i, j);
        const float fs = (float)v, fa = (float)n5;
        sp[c] = fs;
        an[c] = fa;
        smn = fminf(smn, fs);
        smx = fmaxf(smx, fs);
        amn = fminf(amn, fa);
        amx = fmaxf(amx, fa);
    }
    block_minmax(smn, smx, red);
    block_minmax(amn, amx, red);
    const float sr = smx - smn, ar = amx - amn;
    for (int c = threadIdx.x; c < N; c += kFieldThreads) {
        const float nrm = (sp[c] - smn) / sr;
        const float t = -10.0f * (nrm - 0.5f);
        // numpy's float32 exp is within an ulp of the correctly rounded value; the f64 exp
        // rounded to f32 is the correctly rounded value but for double-rounding cases
        const float speed = 1.0f / (1.0f + (float)exp((double)t));
        field[c] = make_float2(speed, (an[c] - amn) / ar);
    }
}

// Robot.process_demonstration's demonstration set (robot.py:694-698) with the augmentation of
// robot.py:771-824, one output point per thread: demo d's block is its T original states (f64 of
// the f32 CEM states), then per augmentation k the (T-1)*(steps+1) + 1 augmented states: for
// transition i and sub-step s < steps the float32 interpolation cur + f32(s+1)/(steps+1)*(nxt-cur)
// (numpy NEP 50: a python-float fraction times a float32 array stays float32, no fma) plus the
// state noise, at s = steps the current state plus noise, and finally the last state plus noise.
// noise [n_demo][n_aug][D], D = (T-1)(steps+1)*4 + 4: the augmentation's normal draws in the
// reference's order (per (i, s): state 2, action 2; then the last state 2, last action 2).
__global__ __launch_bounds__(kBlock) void k_demo_augment(int32_t n_demo, int32_t T, int32_t steps,
                                                         int32_t n_aug,
                                                         const float2* __restrict__ states,
                                                         const double* __restrict__ noise,
                                                         double2* __restrict__ out) {
    const int64_t per = steps + 1, A = (int64_t)(T - 1) * per + 1, Lp = T + n_aug * A;
    const int64_t D = (int64_t)(T - 1) * per * 4 + 4;
    const int64_t idx = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (idx >= (int64_t)n_demo * Lp) return;
    const int64_t d = idx / Lp;
    int64_t j = idx % Lp;
    const float2* st = states + d * T;
    double2 v;
    if (j < T) {
        const float2 q = st[j];
        v = make_double2((double)q.x, (double)q.y);
    } else {
        j -= T;
        const int64_t k = j / A, r = j % A;
        const double* g = noise + (d * n_aug + k) * D;
        if (r == A - 1) {
            const float2 q = st[T - 1];
            v = make_double2((double)q.x + g[D - 4], (double)q.y + g[D - 3]);
        } else {
            const int64_t i = r / per, sub = r % per;
            const float2 cur = st[i];
            double bx = cur.x, by = cur.y;
            if (sub < steps) {
                const float2 nxt = st[i + 1];
                const float f = (float)((double)(sub + 1) / (double)(steps + 1));
                const float dx = nxt.x - cur.x, dy = nxt.y - cur.y;
                const float tx = f * dx, ty = f * dy;
                bx = (double)(cur.x + tx);
                by = (double)(cur.y + ty);
            }
            const double* gn = g + (i * per + sub) * 4;
            v = make_double2(bx + gn[0], by + gn[1]);
        }
    }
    out[idx] = v;
}

// environment.py:166-171: the E best paths (np.argsort ascending, last E; ties by path index, a
// stable order), their float32 action mean and std over the elites in that order (numpy's float32
// reductions: sequential sums, / E, sqrt); best [n] = argmax of the rewards (first maximum,
// environment.py:173). Workgroup = problem; P <= kBlock.
__global__ __launch_bounds__(kBlock) void k_cem_elite(int32_t P, int32_t T, int32_t E,
                                                      const double* __restrict__ reward,
                                                      const float* __restrict__ actions,
                                                      float* __restrict__ mean,
                                                      float* __restrict__ stdv,
                                                      int32_t* __restrict__ best) {
    __shared__ double r[kBlock];
    __shared__ int order[kBlock];
    const int prob = blockIdx.x, tid = threadIdx.x;
    if (tid < P) r[tid] = reward[(int64_t)prob * P + tid];
    __syncthreads();
    if (tid < P) {
        const double v = r[tid];
        int rank = 0;
        for (int q = 0; q < P; ++q) rank += (r[q] < v || (r[q] == v && q < tid)) ? 1 : 0;
        order[rank] = tid;
    }
    __syncthreads();
    if (best && tid == 0) {
        int b = 0;
        for (int q = 1; q < P; ++q)
            if (r[q] > r[b]) b = q;
        best[prob] = b;
    }
    const float* acts = actions + (int64_t)prob * P * T * 2;
    const float inv_n = (float)E;
    for (int k = tid; k < T * 2; k += kBlock) {
        float sum = acts[(int64_t)order[P - E] * T * 2 + k];
        for (int e = 1; e < E; ++e) sum = sum + acts[(int64_t)order[P - E + e] * T * 2 + k];
        const float mu = sum / inv_n;
        float d0 = acts[(int64_t)order[P - E] * T * 2 + k] - mu;
        float sq = d0 * d0;
        for (int e = 1; e < E; ++e) {
            const float d = acts[(int64_t)order[P - E + e] * T * 2 + k] - mu;
            sq = sq + d * d;
        }
        mean[(int64_t)prob * T * 2 + k] = mu;
        stdv[(int64_t)prob * T * 2 + k] = sqrtf(sq / inv_n);
    }
}

// ReplayBuffer.push (robot.py:79-96) of n transitions given as f64 arrays.
__global__ __launch_bounds__(kBlock) void k_replay_push(int64_t n, const double2* __restrict__ s,
                                                        const double2* __restrict__ a,
                                                        const double* __restrict__ r,
                                                        const double2* __restrict__ s2,
                                                        const uint8_t* __restrict__ d,
                                                        float4* __restrict__ rows, int64_t cap,
                                                        int64_t base) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const int64_t slot = (base + i) % cap;
    const double2 x = s[i], y = a[i], z = s2[i];
    rows[2 * slot] = make_float4((float)x.x, (float)x.y, (float)y.x, (float)y.y);
    rows[2 * slot + 1] = make_float4((float)r[i], (float)z.x, (float)z.y, d[i] ? 1.f : 0.f);
}

// robot.py:753 min_j ||p_i - d_j|| for arbitrary points (scipy cdist semantics).
__global__ __launch_bounds__(kBlock) void k_demo_min(const double2* __restrict__ pts, int64_t n,
                                                     const double2* __restrict__ demo, int64_t m,
                                                     double* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const double2 s = pts[i];
    out[i] = sqrt(demo_min_global(demo, m, s.x, s.y));
}

// ---------------- exact bucketed nearest-demo index ----------------
// For a cell C of width w: U(C)^2 = min_q maxdist^2(q, C) bounds the nearest-demo distance of
// every query inside C, so the nearest point p* satisfies mindist(p*, C) <= U(C). The candidate
// list of C = { p : mindist^2(p, C) <= U^2 (1 + 1e-12) + 1e-12 } contains p* for every query in C;
// the query takes the same f64 minimum over it as over all points, so the result is
// bit-identical to the brute force (tests/test_gpu_env.py checks it).
// Two levels: the 1 x 1 dynamics cells over all points of the group (plan / scan / fill), then
// each dynamics cell's kRes x kRes index cells over its parent's list only (subplan / subscan /
// subfill): a subcell S of C has mindist(p, C) <= mindist(p, S) and U(S) <= U(C), so every
// candidate of S is a candidate of C, and U(S) taken over C's list is still a real point's
// maxdist, i.e. a valid bound. The queries use the index-cell lists.
NAV_DEV double cell_maxd2(double px, double py, double lx, double ly, double w = 1.0) {
    const double fx = fmax(fabs(px - lx), fabs(px - (lx + w)));
    const double fy = fmax(fabs(py - ly), fabs(py - (ly + w)));
    return fx * fx + fy * fy;
}

NAV_DEV double cell_mind2(double px, double py, double lx, double ly, double w = 1.0) {
    const double nx = fmax(0.0, fmax(lx - px, px - (lx + w)));
    const double ny = fmax(0.0, fmax(ly - py, py - (ly + w)));
    return nx * nx + ny * ny;
}

NAV_DEV double block_min(double v, double* red) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o, 64));
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) red[wv] = v;
    __syncthreads();
    v = red[0];
    for (int w = 1; w < kBlock / 64; ++w) v = fmin(v, red[w]);
    return v;
}

// grid = (cells / kPlanCells, groups): bound U^2 and candidate count of kPlanCells consecutive
// cells (one x column, consecutive y) of one group. Each point is loaded once per block and
// tested against all of the block's cells (the per-cell form re-read the group's points from L2
// for every cell: 232 GB of L2 reads at the bench's 64 x 10 000 cells, 9.4 ms); min and count are
// order-independent, so the result is the per-cell form's exactly.
constexpr int kPlanCells = 10;
static_assert(kCells % kPlanCells == 0 && NAV_WORLD_CELLS % kPlanCells == 0, "plan strips");
__global__ __launch_bounds__(kBlock) void k_demo_index_plan(const double2* __restrict__ demo,
                                                            const int64_t* __restrict__ off,
                                                            int64_t m_shared,
                                                            double* __restrict__ bound,
                                                            int32_t* __restrict__ count) {
    __shared__ double red[kBlock / 64];
    __shared__ int cnt[kPlanCells][kBlock / 64];
    const int cell0 = blockIdx.x * kPlanCells, g = blockIdx.y;
    const int64_t lo = off ? off[g] : 0, hi = off ? off[g + 1] : m_shared;
    const double lx = (double)(cell0 / NAV_WORLD_CELLS), ly0 = (double)(cell0 % NAV_WORLD_CELLS);
    double u[kPlanCells];
#pragma unroll
    for (int c = 0; c < kPlanCells; ++c) u[c] = __builtin_inf();
    for (int64_t j = lo + threadIdx.x; j < hi; j += kBlock) {
        const double2 q = demo[j];
#pragma unroll
        for (int c = 0; c < kPlanCells; ++c) u[c] = fmin(u[c], cell_maxd2(q.x, q.y, lx, ly0 + c));
    }
    double lim[kPlanCells];
#pragma unroll
    for (int c = 0; c < kPlanCells; ++c) {
        const double uc = block_min(u[c], red);
        lim[c] = uc * (1.0 + 1e-12) + 1e-12;
    }
    int n[kPlanCells] = {};
    for (int64_t j = lo + threadIdx.x; j < hi; j += kBlock) {
        const double2 q = demo[j];
#pragma unroll
        for (int c = 0; c < kPlanCells; ++c) n[c] += cell_mind2(q.x, q.y, lx, ly0 + c) <= lim[c] ? 1 : 0;
    }
#pragma unroll
    for (int c = 0; c < kPlanCells; ++c) {
        int v = n[c];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        if ((threadIdx.x & 63) == 0) cnt[c][threadIdx.x >> 6] = v;
    }
    __syncthreads();
    if (threadIdx.x < kPlanCells) {
        const int c = threadIdx.x;
        int t = 0;
        for (int w = 0; w < kBlock / 64; ++w) t += cnt[c][w];
        const int64_t k = (int64_t)g * kCells + cell0 + c;
        bound[k] = lim[c];
        count[k] = t;
    }
}

// exclusive scan of counts [n] into start [n + 1] (set-up time only; n = 10.24 M index cells at
// the bench config) in three launches over tiles of 4096 counts (4 per thread of a 1024-thread
// workgroup), using `start` itself as the scratch of the tile totals: (1) every tile's total into
// start[last index of the tile]; (2) one workgroup scans the ~2 500 totals into each tile's
// exclusive offset at start[first index of the tile] and writes start[n]; (3) every tile scans its
// counts from its offset (the tile's own scratch entries are overwritten last). Before: one
// workgroup walked every tile in turn (3.3 ms per scan, profiles/r03zk_kernel_stats.csv).
constexpr int kScanThreads = 1024;
constexpr int64_t kScanTile = 4 * kScanThreads;

// inclusive scan of v across the workgroup (kScanThreads), wave scans + the wave totals in LDS
NAV_DEV int64_t block_incl_scan(int64_t v, int64_t* wtot) {
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int64_t up = __shfl_up(v, o, 64);
        if (lane >= o) v += up;
    }
    if (lane == 63) wtot[wv] = v;
    __syncthreads();
    int64_t before = 0;
    for (int w = 0; w < wv; ++w) before += wtot[w];
    __syncthreads();  // wtot may be reused by the next call
    return before + v;
}

__global__ __launch_bounds__(kScanThreads) void k_scan_tile_sums(const int32_t* __restrict__ count,
                                                                 int64_t n,
                                                                 int64_t* __restrict__ start) {
    __shared__ int64_t wtot[kScanThreads / 64];
    const int64_t t0 = (int64_t)blockIdx.x * kScanTile, i0 = t0 + 4 * (int64_t)threadIdx.x;
    int64_t mine = 0;
#pragma unroll
    for (int u = 0; u < 4; ++u) mine += i0 + u < n ? count[i0 + u] : 0;
    const int64_t incl = block_incl_scan(mine, wtot);
    if (threadIdx.x == kScanThreads - 1) {
        const int64_t last = t0 + kScanTile < n ? t0 + kScanTile - 1 : n - 1;
        start[last] = incl;  // the tile's total
    }
}

__global__ __launch_bounds__(kScanThreads) void k_scan_tile_offsets(int64_t n,
                                                                    int64_t* __restrict__ start) {
    __shared__ int64_t wtot[kScanThreads / 64];
    __shared__ int64_t carry_s;
    const int64_t tiles = (n + kScanTile - 1) / kScanTile;
    int64_t carry = 0;
    for (int64_t b0 = 0; b0 < tiles; b0 += kScanThreads) {
        const int64_t b = b0 + threadIdx.x;
        const int64_t last = b < tiles ? (b * kScanTile + kScanTile < n ? b * kScanTile + kScanTile - 1
                                                                       : n - 1)
                                       : 0;
        const int64_t tot = b < tiles ? start[last] : 0;
        const int64_t incl = block_incl_scan(tot, wtot);
        if (b < tiles) start[b * kScanTile] = carry + incl - tot;  // the tile's offset
        if (threadIdx.x == kScanThreads - 1) carry_s = carry + incl;
        __syncthreads();
        carry = carry_s;
        __syncthreads();
    }
    if (threadIdx.x == 0) start[n] = carry;
}

__global__ __launch_bounds__(kScanThreads) void k_scan_apply(const int32_t* __restrict__ count,
                                                             int64_t n,
                                                             int64_t* __restrict__ start) {
    __shared__ int64_t wtot[kScanThreads / 64];
    __shared__ int64_t base_s;
    const int64_t t0 = (int64_t)blockIdx.x * kScanTile, i0 = t0 + 4 * (int64_t)threadIdx.x;
    if (threadIdx.x == 0) base_s = start[t0];
    int64_t c[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) c[u] = i0 + u < n ? count[i0 + u] : 0;
    const int64_t mine = c[0] + c[1] + c[2] + c[3];
    const int64_t incl = block_incl_scan(mine, wtot);  // synchronises: base_s is read
    int64_t run = base_s + incl - mine;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        if (i0 + u < n) start[i0 + u] = run;
        run += c[u];
    }
}

inline void scan_counts(const int32_t* count, int64_t n, int64_t* start, hipStream_t st) {
    const unsigned tiles = (unsigned)((n + kScanTile - 1) / kScanTile);
    if (n == 0) {
        hipLaunchKernelGGL(k_scan_tile_offsets, dim3(1), dim3(kScanThreads), 0, st, n, start);
        return;
    }
    hipLaunchKernelGGL(k_scan_tile_sums, dim3(tiles), dim3(kScanThreads), 0, st, count, n, start);
    hipLaunchKernelGGL(k_scan_tile_offsets, dim3(1), dim3(kScanThreads), 0, st, n, start);
    hipLaunchKernelGGL(k_scan_apply, dim3(tiles), dim3(kScanThreads), 0, st, count, n, start);
}

// grid = (cells / kPlanCells, groups): write the candidate indices (group-relative, ascending) of
// the plan's strip of cells, each point loaded once for all of the strip's cells
__global__ __launch_bounds__(kBlock) void k_demo_index_fill(const double2* __restrict__ demo,
                                                            const int64_t* __restrict__ off,
                                                            int64_t m_shared,
                                                            const double* __restrict__ bound,
                                                            const int64_t* __restrict__ start,
                                                            int32_t* __restrict__ cand) {
    __shared__ int wcnt[kPlanCells][kBlock / 64];
    __shared__ int64_t base[kPlanCells];
    const int cell0 = blockIdx.x * kPlanCells, g = blockIdx.y;
    const int64_t lo = off ? off[g] : 0, hi = off ? off[g + 1] : m_shared;
    const double lx = (double)(cell0 / NAV_WORLD_CELLS), ly0 = (double)(cell0 % NAV_WORLD_CELLS);
    const int64_t k0 = (int64_t)g * kCells + cell0;
    double lim[kPlanCells];
#pragma unroll
    for (int c = 0; c < kPlanCells; ++c) lim[c] = bound[k0 + c];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (threadIdx.x < kPlanCells) base[threadIdx.x] = start[k0 + threadIdx.x];
    __syncthreads();
    for (int64_t j0 = lo; j0 < hi; j0 += kBlock) {
        const int64_t j = j0 + threadIdx.x;
        double2 q = make_double2(0.0, 0.0);
        if (j < hi) q = demo[j];
        unsigned long long bal[kPlanCells];
#pragma unroll
        for (int c = 0; c < kPlanCells; ++c) {
            const bool take = j < hi && cell_mind2(q.x, q.y, lx, ly0 + c) <= lim[c];
            bal[c] = __ballot(take);
            if (lane == 0) wcnt[c][wv] = __popcll(bal[c]);
        }
        __syncthreads();
#pragma unroll
        for (int c = 0; c < kPlanCells; ++c) {
            if (!((bal[c] >> lane) & 1ull)) continue;
            int wbase = 0;
            for (int w = 0; w < wv; ++w) wbase += wcnt[c][w];
            cand[base[c] + wbase + __popcll(bal[c] & ((1ull << lane) - 1ull))] = (int32_t)(j - lo);
        }
        __syncthreads();
        if (threadIdx.x < kPlanCells) {
            int tot = 0;
            for (int w = 0; w < kBlock / 64; ++w) tot += wcnt[threadIdx.x][w];
            base[threadIdx.x] += tot;
        }
        __syncthreads();
    }
}

NAV_DEV double wave_min(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o, 64));
    return v;
}

// grid = (dynamics cells, groups), 4 waves: wave w takes index subcells w, w + 4, ... of its
// dynamics cell; bound and count of each from the parent's candidate list (lane-strided).
__global__ __launch_bounds__(kBlock) void k_demo_index_subplan(const double2* __restrict__ demo,
                                                               const int64_t* __restrict__ off,
                                                               const int64_t* __restrict__ start1,
                                                               const int32_t* __restrict__ cand1,
                                                               double* __restrict__ bound,
                                                               int32_t* __restrict__ count) {
    const int cell = blockIdx.x, g = blockIdx.y, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const double2* pts = demo + (off ? off[g] : 0);
    const int64_t k1 = (int64_t)g * kCells + cell;
    const int64_t a = start1[k1], b = start1[k1 + 1];
    const int cx = cell / NAV_WORLD_CELLS, cy = cell % NAV_WORLD_CELLS;
    constexpr double w = 1.0 / kRes;
    for (int sc = wv; sc < kRes * kRes; sc += kBlock / 64) {
        const int sx = sc / kRes, sy = sc % kRes;
        const double lx = cx + sx * w, ly = cy + sy * w;
        double u = __builtin_inf();
        for (int64_t t = a + lane; t < b; t += 64) {
            const double2 q = pts[cand1[t]];
            u = fmin(u, cell_maxd2(q.x, q.y, lx, ly, w));
        }
        u = wave_min(u);
        const double lim = u * (1.0 + 1e-12) + 1e-12;
        int c = 0;
        for (int64_t t = a + lane; t < b; t += 64) {
            const double2 q = pts[cand1[t]];
            c += cell_mind2(q.x, q.y, lx, ly, w) <= lim ? 1 : 0;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
        if (lane == 0) {
            const int64_t k = (int64_t)g * kIdxCells + (int64_t)(cx * kRes + sx) * kSide +
                              (cy * kRes + sy);
            bound[k] = lim;
            count[k] = c;
        }
    }
}

// the index cells' candidate lists, in their parent list's (ascending) order
__global__ __launch_bounds__(kBlock) void k_demo_index_subfill(const double2* __restrict__ demo,
                                                               const int64_t* __restrict__ off,
                                                               const int64_t* __restrict__ start1,
                                                               const int32_t* __restrict__ cand1,
                                                               const double* __restrict__ bound,
                                                               const int64_t* __restrict__ start,
                                                               int32_t* __restrict__ cand) {
    const int cell = blockIdx.x, g = blockIdx.y, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const double2* pts = demo + (off ? off[g] : 0);
    const int64_t k1 = (int64_t)g * kCells + cell;
    const int64_t a = start1[k1], b = start1[k1 + 1];
    const int cx = cell / NAV_WORLD_CELLS, cy = cell % NAV_WORLD_CELLS;
    constexpr double w = 1.0 / kRes;
    for (int sc = wv; sc < kRes * kRes; sc += kBlock / 64) {
        const int sx = sc / kRes, sy = sc % kRes;
        const double lx = cx + sx * w, ly = cy + sy * w;
        const int64_t k = (int64_t)g * kIdxCells + (int64_t)(cx * kRes + sx) * kSide +
                          (cy * kRes + sy);
        const double lim = bound[k];
        int64_t run = start[k];
        for (int64_t t0 = a; t0 < b; t0 += 64) {
            const int64_t t = t0 + lane;
            bool take = false;
            int32_t j = 0;
            if (t < b) {
                j = cand1[t];
                const double2 q = pts[j];
                take = cell_mind2(q.x, q.y, lx, ly, w) <= lim;
            }
            const unsigned long long bal = __ballot(take);
            if (take) cand[run + __popcll(bal & ((1ull << lane) - 1ull))] = j;
            run += __popcll(bal);
        }
    }
}

// The demo-proximity term through the index: lane = env, its cell = the index cell of s'.
__global__ __launch_bounds__(kBlock) void k_demo_reward_idx(nav_params p, int64_t n,
                                                            const double2* __restrict__ ns,
                                                            const double* __restrict__ gterm,
                                                            const uint8_t* __restrict__ flags,
                                                            DemoIdx d, float* __restrict__ rows,
                                                            int64_t cap, int64_t base,
                                                            double* __restrict__ reward_out) {
    const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (e >= n) return;
    const uint8_t f = flags[e];
    if (!(f & F_DEMO)) return;
    const double r = demo_reward_of(p, gterm[e], demo_min2_idx(d, e, ns[e]), (f & F_STUCK) != 0);
    const int64_t slot = (base + e) % cap;
    rows[slot * NAV_ROW + 4] = (float)r;
    if (reward_out) reward_out[e] = r;
}

// block_stats' reward column after a separate demo pass (nav_demo_reward(_indexed) with
// block_stats): the row of every 64 envs that hold a flagged env is summed again from the pushed
// rewards (the replay rows, now final) — the same wave tree over the same floats as the tick
// that runs the demo pass in its own launch, so every launch form reports the pushed reward.
__global__ __launch_bounds__(kBlock) void k_restat_reward(int64_t n, const uint8_t* __restrict__ flags,
                                                          const float* __restrict__ rows,
                                                          int64_t cap, int64_t base,
                                                          float* __restrict__ block_stats) {
    const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const bool live = e < n;
    const bool flagged = live && (flags[e] & F_DEMO);
    if (!__any(flagged)) return;  // wave-uniform
    const float r = live ? rows[((base + e) % cap) * NAV_ROW + 4] : 0.f;
    const float v = wave_sum(r);
    if ((threadIdx.x & 63) == 0) block_stats[(e >> 6) * 8] = v;
}

// One training tick per env (see navenv.h nav_agent_step). DEMO: the demo-proximity reward of
// flagged envs through the index in the same launch (nav_agent_step_indexed): the block's demo
// pass walks all its flagged envs' candidate lists together. One statistics row per wave.
template <bool DEMO>
__global__ __launch_bounds__(kBlock) void k_agent_step(nav_params p, nav_env_soa env,
                                                       const float2* __restrict__ field,
                                                       const double2* __restrict__ action,
                                                       float4* __restrict__ rows, int64_t cap,
                                                       int64_t base, nav_step_out out,
                                                       DemoIdx d, int32_t demo_pending,
                                                       double* __restrict__ reward_out) {
    const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    TickStats st{0.f, 0.f, 0.f, 0.f, 0.f};
    DemoPend pend{false, false, 0.0, make_double2(0.0, 0.0)};
    if (e < env.n)
        st = agent_tick<DEMO>(p, env, field, e, action[e], rows, cap, base, out,
                              demo_pending != 0, pend);
    if (DEMO) {
        __shared__ DemoScratch<kBlock, kBlock> scratch;
        const double r = demo_pass<kBlock, kBlock>(p, d, scratch, pend, e,
                                                   reinterpret_cast<float*>(rows), cap, base,
                                                   reward_out);
        if (pend.need) st.r = (float)r;  // the final reward of a flagged env
    }
    if (out.block_stats && e - (threadIdx.x & 63) < env.n) wave_stats(st, out.block_stats, e);
}

// Environment.step for K consecutive steps per launch (environment.py:122-127 applied K times):
// the state stays in registers, actions [K][n][2] stream in, next_out (nullable) [K][n][2]
// receives every step's committed state. Bytes per env-step 16 (+16 with next_out) + 32/K.
__global__ __launch_bounds__(kBlock) void k_env_step_k(int64_t n, int32_t K,
                                                       double2* __restrict__ state,
                                                       const float2* __restrict__ field,
                                                       const double2* __restrict__ action,
                                                       double2* __restrict__ next_out) {
    const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (e >= n) return;
    double2 s = state[e];
    double2 a = action[e];
    for (int32_t k = 0; k < K; ++k) {
        // the next step's action is in flight under this step's dynamics
        const double2 an = k + 1 < K ? action[(int64_t)(k + 1) * n + e] : a;
        const double2 nx = dynamics(field, s, a);
        if (in_world(nx)) s = nx;
        if (next_out) next_out[(int64_t)k * n + e] = s;
        a = an;
    }
    state[e] = s;
}

__global__ __launch_bounds__(kBlock) void k_compute_reward(nav_params p, int64_t n,
                                                           const double2* __restrict__ ns,
                                                           const double2* __restrict__ goal,
                                                           const double2* __restrict__ demo,
                                                           int64_t m, int32_t demo_flag,
                                                           double* reward, uint8_t* hit) {
    const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (e >= n) return;
    const double2 s = ns[e], g = goal[e];
    const double gt = -norm2(s.x - g.x, s.y - g.y);
    double r;
    uint8_t h = 0;
    if (gt >= -p.goal_threshold) {
        r = p.goal_reward;
        h = 1;
    } else if (m == 0) {
        r = gt;
    } else {
        const double mn = sqrt(demo_min_global(demo, m, s.x, s.y));
        r = gt + p.demo_factor * (demo_flag ? -mn : 0.0);
    }
    reward[e] = r;
    if (hit) hit[e] = h;
}

inline int blocks_for(int64_t n) { return (int)((n + kBlock - 1) / kBlock); }
inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

}  // namespace

extern "C" {

int nav_abi_version(void) { return NAV_ABI_VERSION; }

int nav_event_create(void** event) {
    if (!event) return NAV_EINVAL;
    const hipError_t e = hipEventCreateWithFlags(reinterpret_cast<hipEvent_t*>(event),
                                                 hipEventReleaseToDevice);
    return e == hipSuccess ? 0 : -(int)e;
}

int nav_event_destroy(void* event) {
    if (!event) return NAV_EINVAL;
    const hipError_t e = hipEventDestroy(reinterpret_cast<hipEvent_t>(event));
    return e == hipSuccess ? 0 : -(int)e;
}

int nav_event_record(void* event, void* stream) {
    if (!event) return NAV_EINVAL;
    const hipError_t e = hipEventRecord(reinterpret_cast<hipEvent_t>(event), S(stream));
    return e == hipSuccess ? 0 : -(int)e;
}

int nav_event_elapsed_ms(void* start, void* end, float* ms) {
    if (!start || !end || !ms) return NAV_EINVAL;
    hipError_t e = hipEventSynchronize(reinterpret_cast<hipEvent_t>(end));
    if (e == hipSuccess)
        e = hipEventElapsedTime(ms, reinterpret_cast<hipEvent_t>(start),
                                reinterpret_cast<hipEvent_t>(end));
    return e == hipSuccess ? 0 : -(int)e;
}

void nav_default_params(nav_params* p) {
    if (!p) return;
    p->world_size = 100.0;
    p->max_action = 5.0;
    p->init_region_size = 25.0;
    p->goal_threshold = 5.0;
    p->goal_reward = 50.0;
    p->stuck_threshold = 2.0;
    p->stuck_penalty = 50.0;
    p->demo_factor = 10.0;
    p->noise_decay = 0.75;
    p->path_length0 = 50;
    p->path_increase = 20;
    p->seed_lo = 1707366464u;
    p->seed_hi = 0u;
    p->max_goal_draws = 1 << 16;
}

static bool env_ok(const nav_env_soa* e) {
    return e && e->n >= 0 && e->n < (int64_t)1 << 31 && (e->n == 0 || (e->state && e->goal &&
           e->region && e->hist && e->meta && e->plan_index && e->path_length && e->episodes &&
           e->noise_scale));
}

int nav_env_init(const nav_params* p, const nav_env_soa* env, int32_t epg, int32_t demo_flag,
                 int32_t* draws_out, void* stream) {
    if (!p || !env_ok(env) || epg <= 0 || p->max_goal_draws <= 0) return NAV_EINVAL;
    if (env->n == 0) return 0;
    hipLaunchKernelGGL(k_env_init, dim3(blocks_for(env->n)), dim3(kBlock), 0, S(stream), *p, *env,
                       epg, demo_flag, draws_out);
    NAV_CHECK_LAUNCH();
    return 0;
}

int nav_env_reset(const nav_params* p, const nav_env_soa* env, const uint8_t* mask,
                  const double* uniforms, void* stream) {
    // needs state + region; the Philox draw also reads episodes
    if (!p || !env || env->n < 0 ||
        (env->n && (!env->state || !env->region || (!uniforms && !env->episodes))))
        return NAV_EINVAL;
    if (env->n == 0) return 0;
    hipLaunchKernelGGL(k_env_reset, dim3(blocks_for(env->n)), dim3(kBlock), 0, S(stream), *p,
                       *env, mask, reinterpret_cast<const double2*>(uniforms));
    NAV_CHECK_LAUNCH();
    return 0;
}

int nav_env_step(const nav_params* p, const nav_env_soa* env, const float* field,
                 const double* action, double* next_state, void* stream) {
    if (!p || !env || env->n < 0 || !field || (env->n && (!env->state || !action)))
        return NAV_EINVAL;
    if (env->n == 0) return 0;
    // Non-temporal state/action streams once the 48 B/env working set is past the 256 MB MALL
    // (>= 4 Mi envs): 219 -> 204 us at 2^24 envs (profiles/r01p_step_ab.log). Below that the
    // state stays cache-resident between steps, so default-policy accesses.
    const bool nt = env->n >= (int64_t(1) << 22);
    hipLaunchKernelGGL(nt ? k_env_step<true> : k_env_step<false>, dim3(blocks_for(env->n)),
                       dim3(kBlock), 0, S(stream), env->n,
                       reinterpret_cast<double2*>(env->state),
                       reinterpret_cast<const float2*>(field),
                       reinterpret_cast<const double2*>(action),
                       reinterpret_cast<double2*>(next_state));
    NAV_CHECK_LAUNCH();
    return 0;
}

int nav_env_step_k(const nav_params* p, const nav_env_soa* env, const float* field,
                   const double* actions, int32_t K, double* next_states, void* stream) {
    if (!p || !env || env->n < 0 || K < 0 || !field ||
        (env->n && K && (!env->state || !actions)))
        return NAV_EINVAL;
    if (env->n == 0 || K == 0) return 0;
    hipLaunchKernelGGL(k_env_step_k, dim3(blocks_for(env->n)), dim3(kBlock), 0, S(stream),
                       env->n, K, reinterpret_cast<double2*>(env->state),
                       reinterpret_cast<const float2*>(field),
                       reinterpret_cast<const double2*>(actions),
                       reinterpret_cast<double2*>(next_states));
    NAV_CHECK_LAUNCH();
    return 0;
}

int nav_dynamics(const float* field, const double* state, const double* action, double* out,
                 int64_t n, void* stream) {
    if (n < 0 || (n && (!field || !state || !action || !out))) return NAV_EINVAL;
    if (n == 0) return 0;
    hipLaunchKernelGGL(k_dynamics, dim3(blocks_for(n)), dim3(kBlock), 0, S(stream), n,
                       reinterpret_cast<const float2*>(field),
                       reinterpret_cast<const double2*>(state),
                       reinterpret_cast<const double2*>(action), reinterpret_cast<double2*>(out));
    NAV_CHECK_LAUNCH();
    return 0;
}

int nav_agent_step(const nav_params* p, const nav_env_soa* env, const float* field,
                   const double* action, const nav_replay* replay, int64_t replay_base,
                   const nav_step_out* out, int32_t demo_pending, void* stream) {
    // one slot per env per launch: a ring smaller than n would let two envs write one slot
    if (!p || !env_ok(env) || !field || !action || !replay || !replay->rows ||
        replay->capacity < env->n || replay->capacity <= 0 || replay_base < 0 || !out)
        return NAV_EINVAL;
    if (env->n == 0) return 0;
    hipLaunchKernelGGL(k_agent_step<false>, dim3(blocks_for(env->n)), dim3(kBlock), 0,
                       S(stream), *p, *env, reinterpret_cast<const float2*>(field),
                       reinterpret_cast<const double2*>(action),
                       reinterpret_cast<float4*>(replay->rows), replay->capacity,
                       replay_base % replay->capacity, *out, DemoIdx{}, demo_pending, nullptr);
    NAV_CHECK_LAUNCH();
    return 0;
}

int nav_agent_step_indexed(const nav_params* p, const nav_env_soa* env, const float* field,
                           const double* action, const nav_replay* replay, int64_t replay_base,
                           const nav_step_out* out, const double* demo_xy,
                           const int64_t* demo_off, int32_t envs_per_group,
                           const int64_t* cell_start, const int32_t* cand, double* reward_out,
                           void* stream) {
    if (!p || !env_ok(env) || !field || !action || !replay || !replay->rows ||
        replay->capacity < env->n || replay->capacity <= 0 || replay_base < 0 || !out ||
        (demo_off && envs_per_group <= 0))
        return NAV_EINVAL;
    if (env->n == 0) return 0;
    if (!demo_xy || !cell_start || !cand) return NAV_EINVAL;
    const DemoIdx d{reinterpret_cast<const double2*>(demo_xy), demo_off,
                    envs_per_group > 0 ? envs_per_group : 1, cell_start, cand};
    hipLaunchKernelGGL(k_agent_step<true>, dim3(blocks_for(env->n)), dim3(kBlock), 0,
                       S(stream), *p, *env, reinterpret_cast<const float2*>(field),
                       reinterpret_cast<const double2*>(action),
                       reinterpret_cast<float4*>(replay->rows), replay->capacity,
                       replay_base % replay->capacity, *out, d, 1, reward_out);
    NAV_CHECK_LAUNCH();
    return 0;
}

int nav_transition(const nav_params* p, const nav_env_soa* env, const double* state,
                   const double* action, const double* next_state, const nav_replay* replay,
                   int64_t replay_base, const nav_step_out* out, int32_t demo_pending,
                   void* stream) {
    if (!p || !env || env->n < 0 || !replay || !replay->rows || replay->capacity < env->n ||
        replay->capacity <= 0 || replay_base < 0 || !out)
        return NAV_EINVAL;
    if (env->n == 0) return 0;
    if (!env->goal || !env->hist || !env->meta || !env->plan_index || !env->path_length ||
        !state || !action || !next_state)
        return NAV_EINVAL;
    hipLaunchKernelGGL(k_transition, dim3(blocks_for(env->n)), dim3(kBlock), 0, S(stream), *p,
                       *env, reinterpret_cast<const double2*>(state),
                       reinterpret_cast<const double2*>(action),
                       reinterpret_cast<const double2*>(next_state),
                       reinterpret_cast<float4*>(replay->rows), replay->capacity,
                       replay_base % replay->capacity, *out, demo_pending);
    NAV_CHECK_LAUNCH();
    return 0;
}

int nav_check_if_stuck(const nav_params* p, const nav_env_soa* env, const double* state,
                       uint8_t* stuck, void* stream) {
    if (!p || !env || env->n < 0 || (env->n && (!env->hist || !env->meta || !state || !stuck)))
        return NAV_EINVAL;
    if (env->n == 0) return 0;
    hipLaunchKernelGGL(k_check_if_stuck, dim3(blocks_for(env->n)), dim3(kBlock), 0, S(stream),
                       *p, *env, reinterpret_cast<const double2*>(state), stuck);
    NAV_CHECK_LAUNCH();
    return 0;
}

int nav_rollout(const float* field, int64_t P, int32_t T, const double* start,
                const double* actions, double* paths, const double* goal, double* reward,
                void* stream) {
    if (P < 0 || T < 0 || (P && (!field || !start || !actions || !paths)) || (reward && !goal))
        return NAV_EINVAL;
    if (P == 0) return 0;
    hipLaunchKernelGGL(k_rollout, dim3(blocks_for(P)), dim3(kBlock), 0, S(stream),
                       reinterpret_cast<const float2*>(field), P, T,
                       reinterpret_cast<const double2*>(start),
                       reinterpret_cast<const double2*>(actions),
                       reinterpret_cast<double2*>(paths), goal, reward);
    NAV_CHECK_LAUNCH();
    return 0;
}

int nav_cem_rollout(const float* field, int32_t n_prob, int32_t P, int32_t T, int32_t iter,
                    const double* region, const double* uniforms, const double* goal,
                    const double* a0, const double* z, const float* mean, const float* stdv,
                    float* actions, float* paths, double* reward, void* stream) {
    if (!field || n_prob < 0 || P < 1 || T < 1 || iter < 0 || !region || !uniforms || !goal ||
        !actions || !reward || (iter == 0 && !a0) || (iter > 0 && (!z || !mean || !stdv)) ||
        (int64_t)n_prob * P * (T + 1) > ((int64_t)1 << 40))
        return NAV_EINVAL;
    if (n_prob == 0) return 0;
    hipLaunchKernelGGL(k_cem_rollout, dim3(blocks_for((int64_t)n_prob * P)), dim3(kBlock), 0,
                       S(stream), reinterpret_cast<const float2*>(field), n_prob, P, T, iter,
                       region, reinterpret_cast<const double2*>(uniforms),
                       reinterpret_cast<const double2*>(goal),
                       reinterpret_cast<const double2*>(a0), reinterpret_cast<const double2*>(z),
                       reinterpret_cast<const float2*>(mean), reinterpret_cast<const float2*>(stdv),
                       reinterpret_cast<float2*>(actions), reinterpret_cast<float2*>(paths),
                       reward);
    NAV_CHECK_LAUNCH();
    return 0;
}

int nav_cem_elite(int32_t n_prob, int32_t P, int32_t T, int32_t E, const double* reward,
                  const float* actions, float* mean, float* stdv, int32_t* best, void* stream) {
    if (n_prob < 0 || P < 1 || P > kBlock || T < 1 || E < 1 || E > P || !reward || !actions ||
        !mean || !stdv)
        return NAV_EINVAL;
    if (n_prob == 0) return 0;
    hipLaunchKernelGGL(k_cem_elite, dim3(n_prob), dim3(kBlock), 0, S(stream), P, T, E, reward,
                       actions, mean, stdv, best);
    NAV_CHECK_LAUNCH();
    return 0;
}

int nav_fields_generate(const double* g5, const double* g10, const double* g20, float* field,
                        void* stream) {
    if (!g5 || !g10 || !g20 || !field) return NAV_EINVAL;
    hipLaunchKernelGGL(k_fields, dim3(1), dim3(kFieldThreads), 0, S(stream), g5, g10, g20,
                       reinterpret_cast<float2*>(field));
    NAV_CHECK_LAUNCH();
    return 0;
}

int nav_demo_augment(int32_t n_demo, int32_t T, int32_t steps, int32_t n_aug,
                     const float* states, const double* noise, double* out, void* stream) {
    if (n_demo < 0 || T < 2 || steps < 0 || n_aug < 0 || (n_demo && (!states || !out)) ||
        (n_demo && n_aug && !noise))
        return NAV_EINVAL;
    const int64_t n = (int64_t)n_demo * (T + (int64_t)n_aug * ((int64_t)(T - 1) * (steps + 1) + 1));
    if (n == 0) return 0;
    hipLaunchKernelGGL(k_demo_augment, dim3(blocks_for(n)), dim3(kBlock), 0, S(stream), n_demo, T,
                       steps, n_aug, reinterpret_cast<const float2*>(states), noise,
                       reinterpret_cast<double2*>(out));
    NAV_CHECK_LAUNCH();
    return 0;
}

int nav_replay_push(const nav_replay* replay, int64_t base, int64_t n, const double* state,
                    const double* action, const double* reward, const double* next_state,
                    const uint8_t* done, void* stream) {
    if (!replay || !replay->rows || replay->capacity <= 0 || base < 0 || n < 0 ||
        (n && (!state || !action || !reward || !next_state || !done)))
        return NAV_EINVAL;
    if (n == 0) return 0;
    hipLaunchKernelGGL(k_replay_push, dim3(blocks_for(n)), dim3(kBlock), 0, S(stream), n,
                       reinterpret_cast<const double2*>(state),
                       reinterpret_cast<const double2*>(action), reward,
                       reinterpret_cast<const double2*>(next_state), done,
                       reinterpret_cast<float4*>(replay->rows), replay->capacity,
                       base % replay->capacity);
    NAV_CHECK_LAUNCH();
    return 0;
}

int nav_demo_reward(const nav_params* p, int64_t n, const double* next_state,
                    const double* goal_term, const uint8_t* flags, const double* demo_xy,
                    const int64_t* demo_off, int64_t m, int32_t epg, const nav_replay* replay,
                    int64_t replay_base, double* reward_out, float* block_stats, void* stream) {
    if (!p || n < 0 || !replay || !replay->rows || replay->capacity <= 0 || replay_base < 0)
        return NAV_EINVAL;
    if (n && (!next_state || !goal_term || !flags)) return NAV_EINVAL;
    if (demo_off && epg <= 0) return NAV_EINVAL;
    if (!demo_off && m > 0 && !demo_xy) return NAV_EINVAL;
    if (n == 0 || (!demo_off && m == 0)) return 0;
    if (n <= 8) {  // a lane per point (the N = 1 drop-in): 81 us -> a few per call
        hipLaunchKernelGGL(k_demo_reward_few, dim3((unsigned)n), dim3(kDemoBlock), 0, S(stream),
                           *p, reinterpret_cast<const double2*>(next_state), goal_term, flags,
                           demo_xy, demo_off, m, epg > 0 ? epg : 1, replay->rows,
                           replay->capacity, replay_base % replay->capacity, reward_out);
    } else {
        hipLaunchKernelGGL(k_demo_reward, dim3((unsigned)((n + kDemoEnvs - 1) / kDemoEnvs)),
                           dim3(kDemoBlock), 0, S(stream), *p, n,
                           reinterpret_cast<const double2*>(next_state), goal_term, flags, demo_xy,
                           demo_off, m, epg > 0 ? epg : 1,
                           replay->rows, replay->capacity, replay_base % replay->capacity,
                           reward_out);
    }
    NAV_CHECK_LAUNCH();
    if (block_stats) {
        hipLaunchKernelGGL(k_restat_reward, dim3(blocks_for(n)), dim3(kBlock), 0, S(stream), n,
                           flags, replay->rows, replay->capacity, replay_base % replay->capacity,
                           block_stats);
        NAV_CHECK_LAUNCH();
    }
    return 0;
}

int nav_demo_min(const double* points, int64_t n, const double* demo_xy, int64_t m,
                 double* out, void* stream) {
    if (n < 0 || m < 1 || (n && (!points || !demo_xy || !out))) return NAV_EINVAL;
    if (n == 0) return 0;
    hipLaunchKernelGGL(k_demo_min, dim3(blocks_for(n)), dim3(kBlock), 0, S(stream),
                       reinterpret_cast<const double2*>(points), n,
                       reinterpret_cast<const double2*>(demo_xy), m, out);
    NAV_CHECK_LAUNCH();
    return 0;
}

int nav_demo_index_plan(const double* demo_xy, const int64_t* demo_off, int32_t n_groups,
                        int64_t m, double* cell_bound, int32_t* cell_count, void* stream) {
    if (!demo_xy || n_groups < 1 || (!demo_off && (n_groups != 1 || m < 1)) || !cell_bound ||
        !cell_count)
        return NAV_EINVAL;
    hipLaunchKernelGGL(k_demo_index_plan, dim3(kCells / kPlanCells, n_groups), dim3(kBlock), 0,
                       S(stream),
                       reinterpret_cast<const double2*>(demo_xy), demo_off, m, cell_bound,
                       cell_count);
    NAV_CHECK_LAUNCH();
    return 0;
}

int nav_demo_index_scan(const int32_t* cell_count, int32_t n_groups, int64_t* cell_start,
                        void* stream) {
    if (!cell_count || !cell_start || n_groups < 1) return NAV_EINVAL;
    scan_counts(cell_count, (int64_t)n_groups * kCells, cell_start, S(stream));
    NAV_CHECK_LAUNCH();
    return 0;
}

int nav_demo_index_fill(const double* demo_xy, const int64_t* demo_off, int32_t n_groups,
                        int64_t m, const double* cell_bound, const int64_t* cell_start,
                        int32_t* cand, void* stream) {
    if (!demo_xy || n_groups < 1 || (!demo_off && n_groups != 1) || !cell_bound ||
        !cell_start || !cand)
        return NAV_EINVAL;
    hipLaunchKernelGGL(k_demo_index_fill, dim3(kCells / kPlanCells, n_groups), dim3(kBlock), 0,
                       S(stream),
                       reinterpret_cast<const double2*>(demo_xy), demo_off, m, cell_bound,
                       cell_start, cand);
    NAV_CHECK_LAUNCH();
    return 0;
}

int32_t nav_demo_index_res(void) { return kRes; }

int nav_demo_index_subplan(const double* demo_xy, const int64_t* demo_off, int32_t n_groups,
                           const int64_t* cell_start, const int32_t* cand, double* sub_bound,
                           int32_t* sub_count, void* stream) {
    if (!demo_xy || n_groups < 1 || (!demo_off && n_groups != 1) || !cell_start || !cand ||
        !sub_bound || !sub_count)
        return NAV_EINVAL;
    hipLaunchKernelGGL(k_demo_index_subplan, dim3(kCells, n_groups), dim3(kBlock), 0, S(stream),
                       reinterpret_cast<const double2*>(demo_xy), demo_off, cell_start, cand,
                       sub_bound, sub_count);
    NAV_CHECK_LAUNCH();
    return 0;
}

int nav_demo_index_subscan(const int32_t* sub_count, int32_t n_groups, int64_t* sub_start,
                           void* stream) {
    if (!sub_count || !sub_start || n_groups < 1) return NAV_EINVAL;
    scan_counts(sub_count, (int64_t)n_groups * kIdxCells, sub_start, S(stream));
    NAV_CHECK_LAUNCH();
    return 0;
}

int nav_demo_index_subfill(const double* demo_xy, const int64_t* demo_off, int32_t n_groups,
                           const int64_t* cell_start, const int32_t* cand,
                           const double* sub_bound, const int64_t* sub_start, int32_t* sub_cand,
                           void* stream) {
    if (!demo_xy || n_groups < 1 || (!demo_off && n_groups != 1) || !cell_start || !cand ||
        !sub_bound || !sub_start || !sub_cand)
        return NAV_EINVAL;
    hipLaunchKernelGGL(k_demo_index_subfill, dim3(kCells, n_groups), dim3(kBlock), 0, S(stream),
                       reinterpret_cast<const double2*>(demo_xy), demo_off, cell_start, cand,
                       sub_bound, sub_start, sub_cand);
    NAV_CHECK_LAUNCH();
    return 0;
}

int nav_demo_reward_indexed(const nav_params* p, int64_t n, const double* next_state,
                            const double* goal_term, const uint8_t* flags, const double* demo_xy,
                            const int64_t* demo_off, int32_t envs_per_group,
                            const int64_t* cell_start, const int32_t* cand,
                            const nav_replay* replay, int64_t replay_base, double* reward_out,
                            float* block_stats, void* stream) {
    if (!p || n < 0 || !replay || !replay->rows || replay->capacity <= 0 || replay_base < 0 ||
        (demo_off && envs_per_group <= 0))
        return NAV_EINVAL;
    if (n == 0) return 0;
    if (!next_state || !goal_term || !flags || !demo_xy || !cell_start || !cand)
        return NAV_EINVAL;
    const DemoIdx d{reinterpret_cast<const double2*>(demo_xy), demo_off,
                    envs_per_group > 0 ? envs_per_group : 1, cell_start, cand};
    hipLaunchKernelGGL(k_demo_reward_idx, dim3(blocks_for(n)), dim3(kBlock), 0, S(stream), *p,
                       n, reinterpret_cast<const double2*>(next_state), goal_term, flags, d,
                       replay->rows, replay->capacity, replay_base % replay->capacity,
                       reward_out);
    NAV_CHECK_LAUNCH();
    if (block_stats) {
        hipLaunchKernelGGL(k_restat_reward, dim3(blocks_for(n)), dim3(kBlock), 0, S(stream), n,
                           flags, replay->rows, replay->capacity, replay_base % replay->capacity,
                           block_stats);
        NAV_CHECK_LAUNCH();
    }
    return 0;
}

int nav_compute_reward(const nav_params* p, int64_t n, const double* next_state,
                       const double* goal, const double* demo_xy, int64_t m, int32_t demo_flag,
                       double* reward, uint8_t* goal_hit, void* stream) {
    if (!p || n < 0 || m < 0 || (n && (!next_state || !goal || !reward)) || (m && !demo_xy))
        return NAV_EINVAL;
    if (n == 0) return 0;
    hipLaunchKernelGGL(k_compute_reward, dim3(blocks_for(n)), dim3(kBlock), 0, S(stream), *p, n,
                       reinterpret_cast<const double2*>(next_state),
                       reinterpret_cast<const double2*>(goal),
                       reinterpret_cast<const double2*>(demo_xy), m, demo_flag, reward, goal_hit);
    NAV_CHECK_LAUNCH();
    return 0;
}

}  // extern "C"
