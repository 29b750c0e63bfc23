/*
 * nav_oracle.c — TEST INFRASTRUCTURE ONLY (parity checker + cpu_baseline leg; see nav_oracle.h).
 *
 * Plain-C fp64 restatement of the reference's environment / agent per-step algorithm, written from
 * the reference's behaviour, not copied from it. Build: oracle/Makefile (-O2 -ffp-contract=off so
 * every product and sum rounds exactly where numpy's separate ufunc calls round).
 */
#include "nav_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ======================= numpy legacy RandomState ======================= */
/* numpy/random/src/mt19937 + legacy distributions (numpy 2.2.6): the RNG under every draw the
 * reference makes (environment.py:29-53, 136, 157-159; robot.py:111, 640, 802-815). */
#define MT_N 624
#define MT_M 397

size_t orc_mt_sizeof(void) { return sizeof(orc_mt_t); }

void orc_mt_seed(orc_mt_t* s, uint32_t seed) {
    /* RandomState.seed(int) -> mt19937_seed (Knuth multiplier init) */
    for (int i = 0; i < MT_N; ++i) {
        s->key[i] = seed;
        seed = 1812433253u * (seed ^ (seed >> 30)) + (uint32_t)(i + 1);
    }
    s->pos = MT_N;
    s->has_gauss = 0;
    s->gauss = 0.0;
}

static void mt_regen(orc_mt_t* s) {
    uint32_t* k = s->key;
    for (int i = 0; i < MT_N; ++i) {
        uint32_t y = (k[i] & 0x80000000u) | (k[(i + 1) % MT_N] & 0x7fffffffu);
        uint32_t v = k[(i + MT_M) % MT_N] ^ (y >> 1);
        if (y & 1u) v ^= 0x9908b0dfu;
        k[i] = v;
    }
    s->pos = 0;
}

uint32_t orc_mt_next32(orc_mt_t* s) {
    if (s->pos == MT_N) mt_regen(s);
    uint32_t y = s->key[s->pos++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

double orc_mt_double(orc_mt_t* s) {
    uint32_t a = orc_mt_next32(s) >> 5, b = orc_mt_next32(s) >> 6;
    return (a * 67108864.0 + b) / 9007199254740992.0;
}

double orc_mt_gauss(orc_mt_t* s) {
    if (s->has_gauss) {
        double t = s->gauss;
        s->has_gauss = 0;
        s->gauss = 0.0;
        return t;
    }
    double x1, x2, r2;
    do {
        x1 = 2.0 * orc_mt_double(s) - 1.0;
        x2 = 2.0 * orc_mt_double(s) - 1.0;
        r2 = x1 * x1 + x2 * x2;
    } while (r2 >= 1.0 || r2 == 0.0);
    double f = sqrt(-2.0 * log(r2) / r2);
    s->gauss = f * x1;
    s->has_gauss = 1;
    return f * x2;
}

static uint64_t mask_of(uint64_t m) {
    m |= m >> 1; m |= m >> 2; m |= m >> 4; m |= m >> 8; m |= m >> 16; m |= m >> 32;
    return m;
}

int64_t orc_mt_randint(orc_mt_t* s, int64_t low, int64_t high) {
    /* legacy _rand_int64 with use_masked=True; ranges < 2^32 draw 32-bit words */
    uint64_t rng = (uint64_t)(high - 1 - low);
    if (rng == 0) return low;
    uint64_t mask = mask_of(rng), v;
    do { v = orc_mt_next32(s) & mask; } while (v > rng);
    return low + (int64_t)v;
}

static uint64_t mt_interval(orc_mt_t* s, uint64_t max) {
    if (max == 0) return 0;
    uint64_t mask = mask_of(max), v;
    do { v = orc_mt_next32(s) & mask; } while (v > max);
    return v;
}

void orc_mt_permutation(orc_mt_t* s, int64_t n, int64_t* out) {
    /* permutation(n) = arange + legacy Fisher-Yates shuffle, i = n-1 .. 1 */
    for (int64_t i = 0; i < n; ++i) out[i] = i;
    for (int64_t i = n - 1; i >= 1; --i) {
        int64_t j = (int64_t)mt_interval(s, (uint64_t)i);
        int64_t t = out[i]; out[i] = out[j]; out[j] = t;
    }
}

/* ======================= Philox4x32-10 ======================= */
void orc_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
    uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
    uint32_t k0 = key[0], k1 = key[1];
    for (int r = 0; r < 10; ++r) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        c1 = (uint32_t)p1; c3 = (uint32_t)p0; c0 = n0; c2 = n2;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

double orc_u01(uint32_t hi, uint32_t lo) {
    return ((hi >> 5) * 67108864.0 + (lo >> 6)) / 9007199254740992.0;
}

/* ======================= Environment ======================= */
static double clipd(double v, double lo, double hi) {
    /* np.clip: NaN propagates */
    if (v != v) return v;
    return v < lo ? lo : (v > hi ? hi : v);
}

double orc_norm2(double a0, double a1) {
    /* np.linalg.norm(v) = sqrt(v.dot(v)); OpenBLAS ddot's scalar tail accumulates with fma */
    return sqrt(fma(a1, a1, a0 * a0));
}

static int cell_of(double v) {
    int c = (int)v; /* int() truncation, v >= 0 */
    return c < 0 ? 0 : (c > 99 ? 99 : c);
}

void orc_dynamics(const float* speed, const float* angle, const double* s, const double* a_in,
                  double* out) {
    /* environment.py:98-119 */
    double a0 = clipd(a_in[0], -5.0, 5.0), a1 = clipd(a_in[1], -5.0, 5.0);
    double mag = orc_norm2(a0, a1);
    double ang = atan2(a1, a0);
    int cx = cell_of(s[0]), cy = cell_of(s[1]);
    /* NEP 50: float32 field * 2 * pi stays float32 */
    float rot = (angle[cx * 100 + cy] * 2.0f) * (float)M_PI;
    double rang = ang + (double)rot;
    double sp = (double)speed[cx * 100 + cy];
    double nx = s[0] + (sp * mag) * cos(rang);
    double ny = s[1] + (sp * mag) * sin(rang);
    double hi = 100.0 - 1.0001;
    out[0] = clipd(nx, 0.0, hi);
    out[1] = clipd(ny, 0.0, hi);
}

int orc_step(const float* speed, const float* angle, double* s, const double* a) {
    /* environment.py:122-127: commit only inside the world (fails only for NaN after the clip) */
    double n[2];
    orc_dynamics(speed, angle, s, a, n);
    if (0.0 <= n[0] && n[0] < 100.0 && 0.0 <= n[1] && n[1] < 100.0) {
        s[0] = n[0];
        s[1] = n[1];
        return 1;
    }
    return 0;
}

void orc_reset_u(const double* region, double u0, double u1, double* out) {
    /* environment.py:135-137: uniform([l, b], [r, t]) = low + (high - low) * u */
    out[0] = region[0] + (region[1] - region[0]) * u0;
    out[1] = region[2] + (region[3] - region[2]) * u1;
}

void orc_reset_mt(orc_mt_t* rs, const double* region, double* out) {
    double u0 = orc_mt_double(rs);
    double u1 = orc_mt_double(rs);
    orc_reset_u(region, u0, u1, out);
}

static void region_of(int r, double u, double* region) {
    /* environment.py:29-49; region = (left, right, bottom, top) */
    const double W = 100.0, S = 25.0;
    double l, rr, b, t;
    double v = 0.0 + (W - S - 0.0) * u;
    if (r == 0) { l = 0; rr = S; b = v; t = b + S; }
    else if (r == 1) { l = v; rr = l + S; b = W - S; t = W; }
    else if (r == 2) { l = W - S; rr = W; b = v; t = b + S; }
    else { l = v; rr = l + S; b = 0; t = S; }
    region[0] = l; region[1] = rr; region[2] = b; region[3] = t;
}

int orc_init_and_goal_mt(orc_mt_t* rs, double* region, double* goal, int* side) {
    /* environment.py:28-56 */
    int r = (int)orc_mt_randint(rs, 0, 4);
    double u = orc_mt_double(rs);
    region_of(r, u, region);
    double mx = 0.5 * (region[0] + region[1]), my = 0.5 * (region[2] + region[3]);
    double dist = 0.0;
    int draws = 0;
    while (dist < 90.0) {
        goal[0] = 5.0 + 90.0 * orc_mt_double(rs);
        goal[1] = 5.0 + 90.0 * orc_mt_double(rs);
        dist = orc_norm2(goal[0] - mx, goal[1] - my);
        ++draws;
    }
    if (side) *side = r;
    return draws;
}

/* ======================= Robot per-step math ======================= */
double orc_demo_min(const double* d, int64_t m, double x, double y) {
    /* robot.py:753: np.min(cdist([s], demos)); scipy's euclidean = sqrt(dx*dx + dy*dy), no fma.
     * sqrt is monotone and correctly rounded, so min-then-sqrt equals sqrt-then-min exactly. */
    double best = INFINITY;
    for (int64_t j = 0; j < m; ++j) {
        double dx = x - d[2 * j], dy = y - d[2 * j + 1];
        double q = dx * dx + dy * dy;
        if (q < best) best = q;
    }
    return sqrt(best);
}

double orc_compute_reward(const double* ns, const double* goal, const double* demo, int64_t m,
                          int demo_flag, int* goal_reached, double goal_thr, double goal_reward,
                          double demo_factor) {
    /* robot.py:727-762 for path = [next_state] */
    double g = -orc_norm2(ns[0] - goal[0], ns[1] - goal[1]);
    if (g >= -goal_thr) {
        *goal_reached = 1;
        return goal_reward;
    }
    if (m == 0) return g;
    double mn = orc_demo_min(demo, m, ns[0], ns[1]);
    double prox = demo_flag ? -mn : 0.0;
    return g + demo_factor * prox;
}

int orc_check_if_stuck(double* hist, int* count, int* head, const double* s, double thr) {
    /* robot.py:509-538: compare with the last STUCK_STEPS (=5) states; stuck clears the history,
     * otherwise the oldest is dropped; the current state is always appended. */
    int stuck = 0;
    if (*count >= 5) {
        int all = 1;
        for (int k = 0; k < 5; ++k) {
            double d = orc_norm2(s[0] - hist[2 * k], s[1] - hist[2 * k + 1]);
            if (!(d < thr)) all = 0;
        }
        if (all) {
            stuck = 1;
            *count = 0;
        } else {
            *head = (*head + 1) % 5;
            *count -= 1;
        }
    }
    int slot = (*head + *count) % 5;
    hist[2 * slot] = s[0];
    hist[2 * slot + 1] = s[1];
    *count += 1;
    return stuck;
}

/* ======================= Vectorised path ======================= */
enum { TAG_INIT = 1, TAG_RESET = 2, TAG_NOISE = 3 };

void orc_default_params(orc_params_t* p) {
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

static void philox_words(const orc_params_t* p, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                         uint32_t w[4]) {
    uint32_t ctr[4] = {c0, c1, c2, c3}, key[2] = {p->seed_lo, p->seed_hi};
    orc_philox(ctr, key, w);
}

int orc_vec_init_one(const orc_params_t* p, uint32_t sid, double* region, double* goal) {
    uint32_t w[4];
    philox_words(p, 0, sid, TAG_INIT, 0, w);
    int r = (int)(w[0] & 3u);
    region_of(r, orc_u01(w[2], w[3]), region);
    double mx = 0.5 * (region[0] + region[1]), my = 0.5 * (region[2] + region[3]);
    for (int k = 1; k <= p->max_goal_draws; ++k) {
        philox_words(p, (uint32_t)k, sid, TAG_INIT, 0, w);
        goal[0] = 5.0 + 90.0 * orc_u01(w[0], w[1]);
        goal[1] = 5.0 + 90.0 * orc_u01(w[2], w[3]);
        if (orc_norm2(goal[0] - mx, goal[1] - my) >= 90.0) return k;
    }
    return 0;
}

void orc_vec_reset_one(const orc_params_t* p, uint32_t env, uint32_t ep, const double* region,
                       double* out) {
    uint32_t w[4];
    philox_words(p, 0, env, TAG_RESET, ep, w);
    orc_reset_u(region, orc_u01(w[0], w[1]), orc_u01(w[2], w[3]), out);
}

void orc_vec_noise_one(const orc_params_t* p, uint32_t env, uint32_t step, double* z) {
    uint32_t w[4];
    philox_words(p, 0, env, TAG_NOISE, step, w);
    double u1 = orc_u01(w[0], w[1]), u2 = orc_u01(w[2], w[3]);
    double rad = sqrt(-2.0 * log(1.0 - u1));
    double th = 6.283185307179586 * u2;
    z[0] = rad * cos(th);
    z[1] = rad * sin(th);
}

void orc_act_epilogue(const double* s, const double* g, const float* res, double sigma,
                      const double* z, double max_action, double* out) {
    /* robot.py:556-567 (training) / 586-593 (testing: z = NULL) */
    for (int i = 0; i < 2; ++i) {
        double b = s[i] - g[i];
        double c = b + (double)res[i];
        if (z) c = c + (sigma * max_action) * z[i];
        out[i] = clipd(c, -max_action, max_action);
    }
}

/* ---- exact nearest-demo index for the CPU port (the cpu_baseline leg does the GPU's algorithm):
 * per cell C a candidate list holding, for every query in C, its nearest demo point.
 * Any demo point q bounds the nearest distance of every x in C by U = maxdist(q, C), and the
 * nearest point p* has mindist(p*, C) <= U, so {p : mindist^2(p, C) <= U^2} suffices; the min over
 * it is the same f64 value as over all points (tests/test_oracle_golden.py checks it).
 * Two levels, as nav_demo_index_*: the 1 x 1 dynamics cells (points bucketed into those cells,
 * rings of buckets searched), then ORC_DEMO_RES x ORC_DEMO_RES index cells per dynamics cell whose
 * lists come from the parent's list (a subcell's candidates are candidates of its parent). */
static double cell_maxd2(double px, double py, double lx, double ly, double w) {
    double fx = fmax(fabs(px - lx), fabs(px - (lx + w)));
    double fy = fmax(fabs(py - ly), fabs(py - (ly + w)));
    return fx * fx + fy * fy;
}

static double cell_mind2(double px, double py, double lx, double ly, double w) {
    double nx = fmax(0.0, fmax(lx - px, px - (lx + w)));
    double ny = fmax(0.0, fmax(ly - py, py - (ly + w)));
    return nx * nx + ny * ny;
}

static int bucket_of(double v) {
    int b = (int)floor(v);
    return b < 0 ? 0 : (b > 99 ? 99 : b);
}

int32_t orc_demo_index_res(void) { return ORC_DEMO_RES; }

/* level 1 over the 100 x 100 dynamics cells: cell_start [10001]; cand NULL = count only */
static int64_t index_level1(const double* demo, int64_t m, int64_t* cell_start, int32_t* cand,
                            int64_t cap) {
    /* buckets (CSR) of the in-world points; points outside [0,100)^2 go to a side list that
     * every cell checks (augmentation noise can push a demo point off the world) */
    int64_t* bstart = (int64_t*)calloc(10001, sizeof(int64_t));
    int32_t* bpts = (int32_t*)malloc((size_t)(m > 0 ? m : 1) * sizeof(int32_t));
    int32_t* outside = (int32_t*)malloc((size_t)(m > 0 ? m : 1) * sizeof(int32_t));
    int64_t n_out = 0;
    for (int64_t j = 0; j < m; ++j) {
        double x = demo[2 * j], y = demo[2 * j + 1];
        if (x >= 0.0 && x < 100.0 && y >= 0.0 && y < 100.0)
            bstart[bucket_of(x) * 100 + bucket_of(y) + 1]++;
        else
            outside[n_out++] = (int32_t)j;
    }
    for (int k = 0; k < 10000; ++k) bstart[k + 1] += bstart[k];
    int64_t* fill = (int64_t*)malloc(10000 * sizeof(int64_t));
    memcpy(fill, bstart, 10000 * sizeof(int64_t));
    for (int64_t j = 0; j < m; ++j) {
        double x = demo[2 * j], y = demo[2 * j + 1];
        if (x >= 0.0 && x < 100.0 && y >= 0.0 && y < 100.0)
            bpts[fill[bucket_of(x) * 100 + bucket_of(y)]++] = (int32_t)j;
    }
    free(fill);
    int64_t total = 0;
    for (int cell = 0; cell < 10000; ++cell) {
        const int cx = cell / 100, cy = cell % 100;
        const double lx = (double)cx, ly = (double)cy;
        double u = INFINITY;
        for (int64_t o = 0; o < n_out; ++o)
            u = fmin(u, cell_maxd2(demo[2 * outside[o]], demo[2 * outside[o] + 1], lx, ly, 1.0));
        /* rings of buckets around the cell until one ring past the first non-empty one */
        int hit = -1;
        for (int r = 0; r < 100; ++r) {
            int any = 0;
            for (int bx = cx - r; bx <= cx + r; ++bx) {
                if (bx < 0 || bx > 99) continue;
                for (int by = cy - r; by <= cy + r; ++by) {
                    if (by < 0 || by > 99) continue;
                    if (abs(bx - cx) != r && abs(by - cy) != r) continue;
                    const int b = bx * 100 + by;
                    for (int64_t t = bstart[b]; t < bstart[b + 1]; ++t) {
                        const int32_t j = bpts[t];
                        u = fmin(u, cell_maxd2(demo[2 * j], demo[2 * j + 1], lx, ly, 1.0));
                        any = 1;
                    }
                }
            }
            if (any && hit < 0) hit = r;
            if (hit >= 0 && r >= hit + 1) break;
        }
        const double lim = u * (1.0 + 1e-12) + 1e-12;
        /* a point in a bucket at Chebyshev distance d is at least d - 1 from the cell */
        const int R = isinf(lim) ? 100 : (int)ceil(sqrt(lim)) + 1;
        const int64_t first = total;
        for (int bx = cx - R; bx <= cx + R; ++bx) {
            if (bx < 0 || bx > 99) continue;
            for (int by = cy - R; by <= cy + R; ++by) {
                if (by < 0 || by > 99) continue;
                const int b = bx * 100 + by;
                for (int64_t t = bstart[b]; t < bstart[b + 1]; ++t) {
                    const int32_t j = bpts[t];
                    if (cell_mind2(demo[2 * j], demo[2 * j + 1], lx, ly, 1.0) <= lim) {
                        if (cand && total < cap) cand[total] = j;
                        ++total;
                    }
                }
            }
        }
        for (int64_t o = 0; o < n_out; ++o) {
            const int32_t j = outside[o];
            if (cell_mind2(demo[2 * j], demo[2 * j + 1], lx, ly, 1.0) <= lim) {
                if (cand && total < cap) cand[total] = j;
                ++total;
            }
        }
        cell_start[cell] = first;
        cell_start[cell + 1] = total;
    }
    free(bstart);
    free(bpts);
    free(outside);
    return total;
}

/* the query index: cell_start [(100 R)^2 + 1] (nullable), cand [cap] (nullable = count only) */
int64_t orc_demo_index_build(const double* demo, int64_t m, int64_t* cell_start, int32_t* cand,
                             int64_t cap) {
    int64_t* s1 = (int64_t*)malloc(10001 * sizeof(int64_t));
    const int64_t t1 = index_level1(demo, m, s1, NULL, 0);
    int32_t* c1 = (int32_t*)malloc((size_t)(t1 > 0 ? t1 : 1) * sizeof(int32_t));
    index_level1(demo, m, s1, c1, t1);
    const int R = ORC_DEMO_RES, side = 100 * ORC_DEMO_RES;
    const double w = 1.0 / R;
    int64_t total = 0;
    for (int ix = 0; ix < side; ++ix) {
        for (int iy = 0; iy < side; ++iy) {
            const int k1 = (ix / R) * 100 + iy / R;
            const double lx = (double)(ix / R) + (ix % R) * w, ly = (double)(iy / R) + (iy % R) * w;
            double u = INFINITY;
            for (int64_t t = s1[k1]; t < s1[k1 + 1]; ++t)
                u = fmin(u, cell_maxd2(demo[2 * c1[t]], demo[2 * c1[t] + 1], lx, ly, w));
            const double lim = u * (1.0 + 1e-12) + 1e-12;
            const int64_t first = total;
            for (int64_t t = s1[k1]; t < s1[k1 + 1]; ++t) {
                const int32_t j = c1[t];
                if (cell_mind2(demo[2 * j], demo[2 * j + 1], lx, ly, w) <= lim) {
                    if (cand && total < cap) cand[total] = j;
                    ++total;
                }
            }
            if (cell_start) {
                cell_start[(int64_t)ix * side + iy] = first;
                cell_start[(int64_t)ix * side + iy + 1] = total;
            }
        }
    }
    free(s1);
    free(c1);
    return total;
}

/* robot.py:753 min distance through the index (brute force off the indexed world) */
double orc_demo_min_idx(const double* demo, int64_t m, const int64_t* cell_start,
                        const int32_t* cand, double x, double y) {
    if (!(x >= 0.0 && x < 100.0 && y >= 0.0 && y < 100.0)) return orc_demo_min(demo, m, x, y);
    const int64_t k = (int64_t)(int)(x * ORC_DEMO_RES) * (100 * ORC_DEMO_RES) +
                      (int)(y * ORC_DEMO_RES);
    double best = INFINITY;
    for (int64_t t = cell_start[k]; t < cell_start[k + 1]; ++t) {
        const int32_t j = cand[t];
        double dx = x - demo[2 * j], dy = y - demo[2 * j + 1];
        double q = dx * dx + dy * dy;
        if (q < best) best = q;
    }
    return sqrt(best);
}

static int tick_impl(const orc_params_t* p, const float* speed, const float* angle,
                     const double* demo, int64_t m, const int64_t* idx_start,
                     const int32_t* idx_cand, uint32_t env, double* state, const double* goal,
                     const double* region, double* hist, uint32_t* meta, int32_t* plan_index,
                     int32_t* path_length, int32_t* episodes, double* noise_scale,
                     const double* action, double* next_out, float* row, double* reward_out,
                     const double* reset_state) {
    uint32_t mt = *meta;
    int goal_reached = (int)(mt & 1u), stuck_flag = (int)((mt >> 1) & 1u);
    int demo_flag = (int)((mt >> 2) & 1u);
    int cnt = (int)((mt >> 8) & 7u), head = (int)((mt >> 12) & 7u);

    double s[2] = {state[0], state[1]}, ns[2] = {state[0], state[1]};
    orc_step(speed, angle, ns, action); /* environment.py:122-127 */

    /* robot.py:645-675 process_transition */
    double r;
    if (idx_start && m > 0) { /* compute_reward (robot.py:727-762) with the indexed minimum */
        double g = -orc_norm2(ns[0] - goal[0], ns[1] - goal[1]);
        if (g >= -p->goal_threshold) {
            goal_reached = 1;
            r = p->goal_reward;
        } else {
            double mn = orc_demo_min_idx(demo, m, idx_start, idx_cand, ns[0], ns[1]);
            r = g + p->demo_factor * (demo_flag ? -mn : 0.0);
        }
    } else {
        r = orc_compute_reward(ns, goal, demo, m, demo_flag, &goal_reached, p->goal_threshold,
                               p->goal_reward, p->demo_factor);
    }
    /* hist is laid out [5][2] for this env */
    int stuck = orc_check_if_stuck(hist, &cnt, &head, s, p->stuck_threshold);
    if (stuck) {
        stuck_flag = 1;
        r -= p->stuck_penalty;
    }
    int done = (*plan_index == *path_length - 1);
    row[0] = (float)s[0]; row[1] = (float)s[1];
    row[2] = (float)action[0]; row[3] = (float)action[1];
    row[4] = (float)r;
    row[5] = (float)ns[0]; row[6] = (float)ns[1];
    row[7] = done ? 1.0f : 0.0f;
    next_out[0] = ns[0]; next_out[1] = ns[1];
    if (reward_out) *reward_out = r;

    /* the next tick's get_next_action_type (robot.py:479-487) + Robot.reset (robot.py:492-506)
     * + Environment.reset (environment.py:130-132), fused: the reset tick takes no env step. */
    int ended = done || goal_reached || stuck_flag;
    int flags = (done ? 1 : 0) | (goal_reached ? 2 : 0) | (stuck ? 4 : 0) | (ended ? 8 : 0);
    if (ended) {
        *episodes += 1;
        *plan_index = 1; /* Robot.reset sets 0; the next tick's increment makes it 1 */
        goal_reached = 0;
        stuck_flag = 0;
        *noise_scale = *noise_scale * p->noise_decay;
        *path_length += p->path_increase;
        if (reset_state) {
            state[0] = reset_state[0];
            state[1] = reset_state[1];
        } else {
            orc_vec_reset_one(p, env, (uint32_t)*episodes, region, state);
        }
    } else {
        *plan_index += 1;
        state[0] = ns[0];
        state[1] = ns[1];
    }
    *meta = (uint32_t)goal_reached | ((uint32_t)stuck_flag << 1) | ((uint32_t)demo_flag << 2) |
            ((uint32_t)cnt << 8) | ((uint32_t)head << 12);
    return flags;
}

int orc_vec_agent_tick(const orc_params_t* p, const float* speed, const float* angle,
                       const double* demo, int64_t m, uint32_t env, double* state,
                       const double* goal, const double* region, double* hist, uint32_t* meta,
                       int32_t* plan_index, int32_t* path_length, int32_t* episodes,
                       double* noise_scale, const double* action, double* next_out, float* row,
                       double* reward_out, const double* reset_state) {
    return tick_impl(p, speed, angle, demo, m, NULL, NULL, env, state, goal, region, hist, meta,
                     plan_index, path_length, episodes, noise_scale, action, next_out, row,
                     reward_out, reset_state);
}

int orc_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

void orc_set_threads(int n) {
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
#else
    (void)n;
#endif
}

void orc_vec_agent_step_batch(const orc_params_t* p, const float* speed, const float* angle,
                              const double* demo, int64_t m, int64_t n, double* state,
                              const double* goal, const double* region, double* hist,
                              uint32_t* meta, int32_t* plan_index, int32_t* path_length,
                              int32_t* episodes, double* noise_scale, const double* action,
                              double* next_out, float* rows, int64_t cap, int64_t base,
                              int64_t env0, const int64_t* idx_start, const int32_t* idx_cand) {
    /* hist here is [n][5][2] (env-major; the device layout differs, the values do not);
     * idx_start / idx_cand (nullable): the demo set's orc_demo_index_build index */
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
    for (int64_t e = 0; e < n; ++e) {
        int64_t slot = (base + e) % cap;
        tick_impl(p, speed, angle, demo, m, idx_start, idx_cand, (uint32_t)(env0 + e),
                  state + 2 * e, goal + 2 * e, region + 4 * e, hist + 10 * e, meta + e,
                  plan_index + e, path_length + e, episodes + e, noise_scale + e, action + 2 * e,
                  next_out + 2 * e, rows + 8 * slot, NULL, NULL);
    }
}

/* Single-env loop on one core for the cpu_baseline's per-env figures: K steps of
 * Environment.step alone (tick = 0) or of the whole agent tick (tick = 1: step, process_transition
 * with the demo term through the index, episode control, replay push into a 1024-row ring),
 * actions cycled from actions [n_act][2]. Returns a checksum of the final state. */
double orc_single_env_run(const orc_params_t* p, const float* speed, const float* angle,
                          const double* demo, int64_t m, const int64_t* idx_start,
                          const int32_t* idx_cand, const double* actions, int64_t n_act,
                          int64_t K, int tick) {
    double state[2] = {50.0, 50.0}, goal[2], region[4], hist[10] = {0}, ns[2];
    uint32_t meta = 4u;
    int32_t plan = 5, path = p->path_length0, ep = 5;
    double noise = 1.0;
    static float rows[1024 * 8];
    orc_vec_init_one(p, 0, region, goal);
    for (int64_t k = 0; k < K; ++k) {
        const double* a = actions + 2 * (k % n_act);
        if (tick)
            tick_impl(p, speed, angle, demo, m, idx_start, idx_cand, 0u, state, goal, region, hist,
                      &meta, &plan, &path, &ep, &noise, a, ns, rows + 8 * (k & 1023), NULL, NULL);
        else
            orc_step(speed, angle, state, a);
    }
    return state[0] + state[1];
}
