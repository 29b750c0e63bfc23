// nav_tick.h — the per-env training tick (environment.py:122-137 + robot.py:443-506, 509-538,
// 645-675, 727-762) as device functions, shared by the standalone tick kernels (env_kernels.hip)
// and the action-selection kernel that runs the tick in its epilogue (mlp_kernels.hip).
#pragma once
#include "nav_device.h"

namespace nav {

constexpr uint32_t M_GOAL = 1u, M_STUCK = 2u, M_DEMO = 4u;
constexpr uint8_t F_DONE = 1, F_GOAL = 2, F_STUCK = 4, F_ENDED = 8, F_DEMO = 16;
constexpr int kCells = NAV_WORLD_CELLS * NAV_WORLD_CELLS;
#ifndef NAV_DEMO_BATCH
#define NAV_DEMO_BATCH 16
#endif
constexpr int kDemoBatch = NAV_DEMO_BATCH;  // candidates per dependent-load trip (indexed reward)
// Resolution of the nearest-demo index: kRes x kRes index cells per dynamics cell (a power of 2,
// so s * kRes and the cell edges are exact). The query cell of s is (int)(s.x * kRes),
// (int)(s.y * kRes); kIdxCells index cells per group.
#ifndef NAV_DEMO_RES
#define NAV_DEMO_RES 4
#endif
constexpr int kRes = NAV_DEMO_RES;
static_assert(kRes >= 1 && (kRes & (kRes - 1)) == 0, "index resolution: a power of 2");
constexpr int kSide = NAV_WORLD_CELLS * kRes;
constexpr int64_t kIdxCells = (int64_t)kSide * kSide;

NAV_DEV bool in_index(double2 s) { return s.x >= 0.0 && s.x < 100.0 && s.y >= 0.0 && s.y < 100.0; }
NAV_DEV int64_t index_cell(int64_t g, double2 s) {
    return g * kIdxCells + (int64_t)(int)(s.x * kRes) * kSide + (int)(s.y * kRes);
}

// Robot.process_transition (robot.py:645-675) for env e given (s, a, s'): reward without the
// demo term (robot.py:727-762; the term is added by the demo pass for flagged envs),
// check_if_stuck on the pre-step state (robot.py:509-538, ring of 5 in hist [5][n]), done, and
// the updated meta word.
struct TransOut {
    double r, gt;
    bool goal_hit, demo_term, stuck, done;
    uint32_t meta;
};

// demo_pending: a demo-proximity pass follows for flagged envs (a non-empty demo set exists). The
// reference adds the demo term only when demonstration_states is non-empty (robot.py:749-751);
// with demo_flag set and no demo set the reward is the goal term alone and the stuck penalty is
// taken here.
// The env's tick inputs that do not depend on its action, loadable ahead of it (the fused act +
// tick launch issues them before its GEMM): state, goal, meta, plan / path counters, the stuck
// ring and the field value at the state.
struct TickIn {
    double2 s, g;
    uint32_t meta;
    int32_t plan, path;
    double2 hist[NAV_HIST];
    float2 f;
};
NAV_DEV TickIn tick_load(const nav_env_soa& env, const float2* __restrict__ field, int64_t e) {
    TickIn in;
    in.s = reinterpret_cast<const double2*>(env.state)[e];
    in.g = reinterpret_cast<const double2*>(env.goal)[e];
    in.meta = env.meta[e];
    in.plan = env.plan_index[e];
    in.path = env.path_length[e];
    const double2* hist = reinterpret_cast<const double2*>(env.hist);
#pragma unroll
    for (int k = 0; k < NAV_HIST; ++k) in.hist[k] = hist[(int64_t)k * env.n + e];
    in.f = field_at(field, in.s);
    return in;
}

NAV_DEV TransOut transition_in(const nav_params& p, const nav_env_soa& env, int64_t e,
                               const TickIn& in, double2 a, double2 ns, bool demo_pending);
NAV_DEV TransOut transition(const nav_params& p, const nav_env_soa& env, int64_t e, double2 s,
                            double2 a, double2 ns, uint32_t meta, int32_t plan, int32_t path,
                            bool demo_pending) {
    TickIn in;
    in.s = s;
    in.g = reinterpret_cast<const double2*>(env.goal)[e];
    in.meta = meta;
    in.plan = plan;
    in.path = path;
    const double2* hist = reinterpret_cast<const double2*>(env.hist);
    // the ring is read only when it is full (cnt >= NAV_HIST)
    if ((int)((meta >> 8) & 7u) >= NAV_HIST) {
#pragma unroll
        for (int k = 0; k < NAV_HIST; ++k) in.hist[k] = hist[(int64_t)k * env.n + e];
    }
    return transition_in(p, env, e, in, a, ns, demo_pending);
}
NAV_DEV TransOut transition_in(const nav_params& p, const nav_env_soa& env, int64_t e,
                               const TickIn& in, double2 a, double2 ns, bool demo_pending) {
    (void)a;
    double2* hist = reinterpret_cast<double2*>(env.hist);
    const double2 s = in.s, g = in.g;
    const uint32_t meta = in.meta;
    const int32_t plan = in.plan, path = in.path;
    TransOut t;
    bool goal_reached = (meta & M_GOAL) != 0;
    t.gt = -norm2(ns.x - g.x, ns.y - g.y);
    t.goal_hit = t.gt >= -p.goal_threshold;
    t.demo_term = false;
    if (t.goal_hit) {
        goal_reached = true;
        t.r = p.goal_reward;
    } else {
        t.r = t.gt;
        t.demo_term = demo_pending && (meta & M_DEMO) != 0;
    }
    int cnt = (int)((meta >> 8) & 7u), head = (int)((meta >> 12) & 7u);
    t.stuck = false;
    if (cnt >= NAV_HIST) {
        bool all = true;
#pragma unroll
        for (int k = 0; k < NAV_HIST; ++k) {
            const double2 h = in.hist[k];
            const double d = norm2(s.x - h.x, s.y - h.y);
            all = all && (d < p.stuck_threshold);
        }
        if (all) {
            t.stuck = true;
            cnt = 0;
        } else {
            head = head == NAV_HIST - 1 ? 0 : head + 1;
            cnt -= 1;
        }
    }
    {
        int sl = head + cnt;
        if (sl >= NAV_HIST) sl -= NAV_HIST;
        hist[(int64_t)sl * env.n + e] = s;
        cnt += 1;
    }
    bool stuck_flag = (meta & M_STUCK) != 0;
    if (t.stuck) {
        stuck_flag = true;
        if (!t.demo_term) t.r -= p.stuck_penalty;
    }
    t.done = plan == path - 1;  // robot.py:672
    t.meta = (goal_reached ? M_GOAL : 0u) | (stuck_flag ? M_STUCK : 0u) | (meta & M_DEMO) |
             ((uint32_t)cnt << 8) | ((uint32_t)head << 12);
    return t;
}

NAV_DEV uint8_t flag_byte(const TransOut& t, bool ended) {
    return (uint8_t)((t.done ? F_DONE : 0) | (t.goal_hit ? F_GOAL : 0) | (t.stuck ? F_STUCK : 0) |
                     (ended ? F_ENDED : 0) | (t.demo_term ? F_DEMO : 0));
}

// ReplayBuffer.push (robot.py:79-96) of (s, a, r, s', done) as one 32-B row.
NAV_DEV void push_row(float4* __restrict__ rows, int64_t slot, double2 s, double2 a, double r,
                      double2 ns, bool done) {
    rows[2 * slot] = make_float4((float)s.x, (float)s.y, (float)a.x, (float)a.y);
    rows[2 * slot + 1] = make_float4((float)r, (float)ns.x, (float)ns.y, done ? 1.f : 0.f);
}

NAV_DEV double demo_min_global(const double2* __restrict__ d, int64_t m, double x, double y) {
    double best = __builtin_inf();
    for (int64_t j = 0; j < m; ++j) {
        const double2 q = d[j];
        const double dx = x - q.x, dy = y - q.y;
        const double v = dx * dx + dy * dy;
        best = v < best ? v : best;
    }
    return best;
}

NAV_DEV double sqd(double x, double y, double px, double py) {
    const double dx = x - px, dy = y - py;
    return dx * dx + dy * dy;
}

// The demo set of env e through the exact bucketed index (nav_demo_index_*): squared distance to
// the nearest demonstration point of its group (robot.py:753), the candidates of the index cell
// of s' (brute force outside the indexed world).
struct DemoIdx {
    const double2* demo;
    const int64_t* off;
    int32_t epg;
    const int64_t* start;
    const int32_t* cand;
};

NAV_DEV double demo_min2_idx(const DemoIdx& d, int64_t e, double2 s) {
    const int64_t g = d.off ? e / d.epg : 0;
    const double2* pts = d.demo + (d.off ? d.off[g] : 0);
    double best = __builtin_inf();
    if (in_index(s)) {
        const int64_t k = index_cell(g, s);
        const int64_t a = d.start[k], b = d.start[k + 1];
        // kDemoBatch candidates per trip: their indices, then their points, are independent loads
        // (two dependent round trips per batch instead of per candidate; a wave runs as many
        // trips as its longest candidate list). Slots past the list repeat candidate a — a
        // duplicate cannot change a min, so the result is the same bits as one by one.
        double bu[kDemoBatch];
#pragma unroll
        for (int u = 0; u < kDemoBatch; ++u) bu[u] = __builtin_inf();
        for (int64_t j = a; j < b; j += kDemoBatch) {
            int32_t c[kDemoBatch];
#pragma unroll
            for (int u = 0; u < kDemoBatch; ++u) c[u] = d.cand[j + u < b ? j + u : a];
            double2 q[kDemoBatch];
#pragma unroll
            for (int u = 0; u < kDemoBatch; ++u) q[u] = pts[c[u]];
#pragma unroll
            for (int u = 0; u < kDemoBatch; ++u) bu[u] = fmin(bu[u], sqd(s.x, s.y, q[u].x, q[u].y));
        }
#pragma unroll
        for (int u = 0; u < kDemoBatch; ++u) best = fmin(best, bu[u]);
    } else {  // outside the indexed cells: brute force
        best = demo_min_global(pts, (d.off ? d.off[g + 1] - d.off[g] : 0), s.x, s.y);
    }
    return best;
}

// robot.py:749-757 reward of a flagged env: goal term + demo_factor * -min dist, minus the stuck
// penalty (the order nav_demo_reward uses).
NAV_DEV double demo_reward_of(const nav_params& p, double gterm, double min2, bool stuck) {
    double r = gterm + p.demo_factor * (-sqrt(min2));
    if (stuck) r -= p.stuck_penalty;
    return r;
}

// The demo term of one env, deferred by the tick to the block's demo pass (its replay row is
// written with the goal-term reward first; the pass overwrites the reward word).
struct DemoPend {
    bool need, stuck;
    double gt;
    double2 ns;
};

// Everything one training tick does for env e given its action (see navenv.h nav_agent_step):
// Environment.step (environment.py:122-127) -> Robot.process_transition (robot.py:645-675) ->
// replay push -> the next tick's end-of-episode check and Robot.reset + Environment.reset
// (robot.py:479-506, environment.py:130-137). DEMO: a demo pass follows in the same launch; the
// env's demo term (robot.py:749-757) is returned in `pend` for it. Returns the per-env statistics
// (reward w/o demo term, done, goal, stuck, ended) for the block reduction.
struct TickStats {
    float r, done, goal, stuck, ended;
};

template <bool DEMO>
NAV_DEV TickStats agent_tick_in(const nav_params& p, const nav_env_soa& env, int64_t e,
                                const TickIn& in, double2 a, float4* __restrict__ rows,
                                int64_t cap, int64_t base, const nav_step_out& out,
                                bool demo_pending, DemoPend& pend);
template <bool DEMO>
NAV_DEV TickStats agent_tick(const nav_params& p, const nav_env_soa& env,
                             const float2* __restrict__ field, int64_t e, double2 a,
                             float4* __restrict__ rows, int64_t cap, int64_t base,
                             const nav_step_out& out, bool demo_pending, DemoPend& pend) {
    return agent_tick_in<DEMO>(p, env, e, tick_load(env, field, e), a, rows, cap, base, out,
                               demo_pending, pend);
}
// the tick from its preloaded inputs (tick_load) and the action
template <bool DEMO>
NAV_DEV TickStats agent_tick_in(const nav_params& p, const nav_env_soa& env, int64_t e,
                                const TickIn& in, double2 a, float4* __restrict__ rows,
                                int64_t cap, int64_t base, const nav_step_out& out,
                                bool demo_pending, DemoPend& pend) {
    double2* state = reinterpret_cast<double2*>(env.state);
    const double2 s = in.s;
    int32_t plan = in.plan;
    const int32_t path = in.path;

    // environment.py:122-127
    double2 ns = dynamics_f(in.f, s, a);
    if (!in_world(ns)) ns = s;
    TransOut t = transition_in(p, env, e, in, a, ns, DEMO || demo_pending);
    if (DEMO) {
        pend.need = t.demo_term;
        pend.stuck = t.stuck;
        pend.gt = t.gt;
        pend.ns = ns;
    }
    push_row(rows, (base + e) % cap, s, a, t.r, ns, t.done);

    // next tick: robot.py:479-487 end check -> Robot.reset (492-506) + Environment.reset
    const bool ended = t.done || (t.meta & (M_GOAL | M_STUCK));
    if (ended) {
        const int32_t ep = env.episodes[e] + 1;
        env.episodes[e] = ep;
        env.path_length[e] = path + p.path_increase;
        env.noise_scale[e] = env.noise_scale[e] * p.noise_decay;
        plan = 1;  // Robot.reset sets 0, the next tick's increment makes it 1
        t.meta &= ~(M_GOAL | M_STUCK);
        const uint4 w = philox(0u, (uint32_t)e, NAV_TAG_RESET, (uint32_t)ep, p.seed_lo,
                               p.seed_hi);
        const double4 rg = reinterpret_cast<const double4*>(env.region)[e];
        const double reg[4] = {rg.x, rg.y, rg.z, rg.w};
        state[e] = region_sample(reg, u01(w.x, w.y), u01(w.z, w.w));
    } else {
        plan += 1;
        state[e] = ns;
    }
    env.plan_index[e] = plan;
    env.meta[e] = t.meta;
    if (out.next_state) reinterpret_cast<double2*>(out.next_state)[e] = ns;
    if (out.goal_term) out.goal_term[e] = t.gt;
    if (out.flags) out.flags[e] = flag_byte(t, ended);
    TickStats st;
    st.r = (float)t.r;
    st.done = t.done ? 1.f : 0.f;
    st.goal = t.goal_hit ? 1.f : 0.f;
    st.stuck = t.stuck ? 1.f : 0.f;
    st.ended = ended ? 1.f : 0.f;
    return st;
}

// ---- block-cooperative demo pass (the indexed demo term of a block's flagged envs) ----
// One lane per env walking its own candidate list makes a wave as slow as its longest list (the
// CEM demo sets: mean 36 candidates per flagged env, per-wave max ~175, p90 350, cells up to 992).
// Here the block's candidate lists are concatenated (inclusive prefix of the lengths in LDS) and
// every thread of the block takes kDemoFlat consecutive entries per trip, whichever envs they
// belong to: a block's time is its total candidate count / block size. Per-env minima are combined
// with LDS 64-bit atomic min on the bit patterns (non-negative doubles order as unsigned
// integers), so the result is the same f64 minimum over the same candidate set, bit for bit.
#ifndef NAV_DEMO_FLAT
#define NAV_DEMO_FLAT 8
#endif
constexpr int kDemoFlat = NAV_DEMO_FLAT;
// sub-phase marks of the demo pass in the phase-trace build of the tick launch (marks 62, 63)
#if defined(NAV_PHASE_TRACE) && defined(NAV_TRACE_MARK)
#define DEMO_MARK(k) NAV_TRACE_MARK(k)
#else
#define DEMO_MARK(k) \
    do {            \
    } while (0)
#endif

template <int NE, int NT>
struct DemoScratch {
    int32_t incl[NE];       // inclusive prefix of the candidate-list lengths
    int32_t wsum[NE / 64];  // per-wave totals of the scan
    int64_t first[NE];      // index into cand of the env's first candidate
    int64_t pbase[NE];      // demo offset of the env's group
    double sx[NE], sy[NE];  // the env's s'
    unsigned long long best[NE];
};

// All NT threads of the block call this (it synchronises). Threads 0..NE-1 own env slots; `pend`
// of a non-owner or an env past n has need = false. Writes the final reward of every flagged env
// into its replay row (word 4) and reward_out, and returns it to the owner (0 elsewhere).
template <int NE, int NT>
NAV_DEV double demo_pass(const nav_params& p, const DemoIdx& d, DemoScratch<NE, NT>& S,
                       const DemoPend& pend, int64_t e, float* __restrict__ rows, int64_t cap,
                       int64_t base, double* __restrict__ reward_out) {
    static_assert(NE % 64 == 0 && NE <= NT, "env slots: whole waves, at most one per thread");
    const int tid = threadIdx.x, lane = tid & 63;
    const bool owner = tid < NE;
    bool brute = false;
    int len = 0;
    int64_t g = 0;
    if (owner) {
        int64_t first = 0;
        if (pend.need) {
            g = d.off ? e / d.epg : 0;
            const double2 s = pend.ns;
            if (in_index(s)) {
                const int64_t k = index_cell(g, s);
                first = d.start[k];
                len = (int)(d.start[k + 1] - first);
            } else {
                brute = true;  // outside the indexed cells
            }
        }
        S.first[tid] = first;
        S.pbase[tid] = d.off ? d.off[g] : 0;
        S.sx[tid] = pend.ns.x;
        S.sy[tid] = pend.ns.y;
        S.best[tid] = 0x7ff0000000000000ull;  // +inf
        // inclusive scan of len within the wave
        int v = len;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int u = __shfl_up(v, o, 64);
            if (lane >= o) v += u;
        }
        if (lane == 63) S.wsum[tid >> 6] = v;
        len = v;  // wave-inclusive prefix
    }
    __syncthreads();
    if (owner) {
        int add = 0;
        for (int w = 0; w < (tid >> 6); ++w) add += S.wsum[w];
        S.incl[tid] = len + add;
    }
    __syncthreads();
    DEMO_MARK(62);  // cell starts gathered, lengths scanned
    const int T = S.incl[NE - 1];
    for (int t0 = tid * kDemoFlat; t0 < T; t0 += NT * kDemoFlat) {
        // owner slot of entry t0: the first slot whose inclusive prefix exceeds it
        int lo = 0, hi = NE - 1;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (S.incl[mid] > t0) hi = mid;
            else lo = mid + 1;
        }
        int o = lo;
        int lo_b = o ? S.incl[o - 1] : 0, hi_b = S.incl[o];
        int ow[kDemoFlat];
        int64_t ci[kDemoFlat];
#pragma unroll
        for (int u = 0; u < kDemoFlat; ++u) {
            const int t = t0 + u;
            if (t < T) {
                while (t >= hi_b) {
                    lo_b = hi_b;
                    ++o;
                    hi_b = S.incl[o];
                }
                ow[u] = o;
                ci[u] = S.first[o] + (t - lo_b);
            } else {  // past the end: repeat the previous entry (a duplicate cannot change a min)
                ow[u] = ow[u > 0 ? u - 1 : 0];
                ci[u] = ci[u > 0 ? u - 1 : 0];
            }
        }
        int32_t c[kDemoFlat];
#pragma unroll
        for (int u = 0; u < kDemoFlat; ++u) c[u] = d.cand[ci[u]];
        double2 q[kDemoFlat];
#pragma unroll
        for (int u = 0; u < kDemoFlat; ++u) q[u] = d.demo[S.pbase[ow[u]] + c[u]];
        int cur_o = ow[0];
        double cur = sqd(S.sx[cur_o], S.sy[cur_o], q[0].x, q[0].y);
#pragma unroll
        for (int u = 1; u < kDemoFlat; ++u) {
            const double v = sqd(S.sx[ow[u]], S.sy[ow[u]], q[u].x, q[u].y);
            if (ow[u] == cur_o) {
                cur = fmin(cur, v);
            } else {
                atomicMin(&S.best[cur_o], (unsigned long long)__double_as_longlong(cur));
                cur_o = ow[u];
                cur = v;
            }
        }
        atomicMin(&S.best[cur_o], (unsigned long long)__double_as_longlong(cur));
    }
    DEMO_MARK(63);  // this thread's trips done
    __syncthreads();
    if (owner && pend.need) {
        double m2;
        if (brute) {
            const double2* pts = d.demo + S.pbase[tid];
            m2 = demo_min_global(pts, d.off ? d.off[g + 1] - d.off[g] : 0, pend.ns.x, pend.ns.y);
        } else {
            m2 = __longlong_as_double((long long)S.best[tid]);
        }
        const double r = demo_reward_of(p, pend.gt, m2, pend.stuck);
        rows[((base + e) % cap) * NAV_ROW + 4] = (float)r;
        if (reward_out) reward_out[e] = r;
        return r;
    }
    return 0.0;
}

// Per-64-env statistics row (one wave = 64 consecutive envs): wave shuffles, lane 0 writes row
// e0/64 of block_stats [ceil(n/64)][8] = sum reward, n_done, n_goal, n_stuck, n_ended, 0, 0, 0
// (the reward as pushed: with the demo term when the demo pass ran in the same launch).
// Deterministic (fixed xor tree), no LDS and no barrier. Call from every lane of the wave.
NAV_DEV void wave_stats(const TickStats& st, float* block_stats, int64_t e0) {
    const float v0 = wave_sum(st.r), v1 = wave_sum(st.done), v2 = wave_sum(st.goal);
    const float v3 = wave_sum(st.stuck), v4 = wave_sum(st.ended);
    const int lane = threadIdx.x & 63;
    if (lane < 8) {
        float v = 0.f;
        v = lane == 0 ? v0 : (lane == 1 ? v1 : (lane == 2 ? v2 : (lane == 3 ? v3 : (lane == 4 ? v4 : 0.f))));
        block_stats[(e0 >> 6) * 8 + lane] = v;
    }
}

}  // namespace nav
