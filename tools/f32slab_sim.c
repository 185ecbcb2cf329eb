/*
 * f32slab_sim.c — experiment (test infrastructure, never shipped): how often
 * would an f32 slab test with a proven error bound leave a traversal decision
 * of Node::intersection (bvh.rs:151-186) undecided, so that the exact f64 slab
 * test must be run?  Built from the oracle's own traversal (oracle.c,
 * node_closest) with its two observation hooks; tools/f32slab_sim.py drives it.
 *
 * Mode bit 0 clear: per ray inv_k = RN32(1/d_k), oi_k = RN32(RN32(o_k) inv_k);
 * per plane q'_k = RN32(fma(b, inv_k, -oi_k)), b an exact f32 box coordinate;
 * |q' - q64| <= eps |q'| + E_k with E_k = |oi_k| 2^-21.
 * Mode bit 0 set (double-float origin): o = o32 + o_lo, oli_k = RN32(RN32(o_lo)
 * inv_k); q'_k = RN32(fma(RN32(b - o32_k), inv_k, -oli_k)); E_k = |oli_k| 2^-21
 * (|o_lo| <= 2^-24 |o|: the absolute term shrinks 2^24-fold, so a ray leaving a
 * surface EPSILON above it still resolves the faces through its origin).
 * eps = 2^-21 is 4x the first-order bound 2^-23; the slack covers the second-
 * order terms and the f32 roundings of the margins.  A min / max over such
 * values keeps the bound eps |result'| + max E_k.  Mode bit 1: the hit test
 * compares only pairs of different axes (x_k <= y_k holds exactly on one axis,
 * which a flat box, min = max, would otherwise leave undecided).
 * Every classification is checked against the exact f64 test of the same
 * child; a violation is counted and must stay 0.
 */
#define _GNU_SOURCE
#include <stdint.h>
#include <stdio.h>

static void sim_node_fwd(const void* b, const void* n, double ox, double oy, double oz, double dx, double dy,
                         double dz, int lh, double lt, int rh, double rt, double bt);
static void sim_pop_fwd(const void* b, int64_t ci, double ox, double oy, double oz, double dx, double dy, double dz,
                        double v, double b2);
#define ORACLE_NODE_HOOK(b, n, o, d, lh, lt, rh, rt, bt) \
    sim_node_fwd(b, n, (o).x, (o).y, (o).z, (d).x, (d).y, (d).z, lh, lt, rh, rt, bt)
#define ORACLE_POP_HOOK(b, ci, o, d, v, b2) sim_pop_fwd(b, ci, (o).x, (o).y, (o).z, (d).x, (d).y, (d).z, v, b2)

#include "../oracle/oracle.c"

enum {
    kNodes, kKids, kMissC, kHitC, kUnc, kVisitUnc, kOrderUnc, kNodeExact, kPops, kPopUnc, kViol, kIneligible, kViolMiss, kViolHit, kViolIv, kViolPop,
    kSimWords
};
static uint64_t g_cnt[kSimWords];
static int g_mode = 0;
void sim_mode(int m) { g_mode = m; }

static const float kEps = 0x1p-21f;

typedef struct { float inv[3], oi[3], o32[3], oli[3], Ek[3], E; int ok; } R32;

static R32 ray32(double ox, double oy, double oz, double dx, double dy, double dz) {
    R32 r;
    const double o[3] = {ox, oy, oz}, d[3] = {dx, dy, dz};
    r.ok = 1;
    r.E = 0.0f;
    for (int k = 0; k < 3; ++k) {
        const double ad = fabs(d[k]);
        if (!(ad >= 0x1p-60 && ad <= 0x1p60) || !(fabs(o[k]) <= 0x1p60)) r.ok = 0;
        r.inv[k] = (float)(1.0 / d[k]);
        r.oi[k] = (float)o[k] * r.inv[k];
        r.o32[k] = (float)o[k];
        r.oli[k] = (float)(o[k] - (double)r.o32[k]) * r.inv[k];
        const float e = ((g_mode & 1) ? fabsf(r.oli[k]) : fabsf(r.oi[k])) * kEps + 0x1p-100f;
        r.Ek[k] = e;
        if (e > r.E) r.E = e;
    }
    return r;
}

/* f32 classification of one child box: 0 certain miss, 1 certain hit (v near *vp), 2 undecided */
static int cls32(const R32* r, const AABB* a, float* vp) {
    const double mn[3] = {a->min.x, a->min.y, a->min.z}, mx[3] = {a->max.x, a->max.y, a->max.z};
    float x[3], y[3];
    float tn = -INFINITY, tf = INFINITY;
    for (int k = 0; k < 3; ++k) {
        float qa, qb;
        if (g_mode & 1) {
            qa = fmaf((float)mn[k] - r->o32[k], r->inv[k], -r->oli[k]);
            qb = fmaf((float)mx[k] - r->o32[k], r->inv[k], -r->oli[k]);
        } else {
            qa = fmaf((float)mn[k], r->inv[k], -r->oi[k]);
            qb = fmaf((float)mx[k], r->inv[k], -r->oi[k]);
        }
        x[k] = fminf(qa, qb); y[k] = fmaxf(qa, qb);
        tn = fmaxf(tn, x[k]);
        tf = fminf(tf, y[k]);
    }
    const float mn_ = fmaf(kEps, fabsf(tn), r->E), mf = fmaf(kEps, fabsf(tf), r->E);
    *vp = fmaxf(tn, 0.0f);
    if (tf + mf < 0.0f) return 0;
    if (!(g_mode & 2)) {
        if (tn - mn_ > tf + mf) return 0;
        if (tn + mn_ <= tf - mf && tf - mf >= 0.0f) return 1;
        return 2;
    }
    int hit = tf - mf >= 0.0f, miss = 0;
    if (g_mode & 4) {  /* per-axis absolute terms */
        hit = 1;
        for (int j = 0; j < 3; ++j) {
            const float mj = fmaf(kEps, fabsf(y[j]), r->Ek[j]);
            if (y[j] + mj < 0.0f) return 0;
            if (!(y[j] - mj >= 0.0f)) hit = 0;
        }
    }
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            if (i == j) continue;
            const float ei = (g_mode & 4) ? r->Ek[i] : r->E, ej = (g_mode & 4) ? r->Ek[j] : r->E;
            const float mi = fmaf(kEps, fabsf(x[i]), ei), mj = fmaf(kEps, fabsf(y[j]), ej);
            if (!(x[i] + mi <= y[j] - mj)) hit = 0;
            if (x[i] - mi > y[j] + mj) miss = 1;
        }
    if (miss) return 0;
    if (hit && (g_mode & 8)) {  /* t_near certainly <= 0: v = max(t_near, 0) is exactly 0 */
        int z = 1;
        for (int i = 0; i < 3; ++i)
            if (!(x[i] + fmaf(kEps, fabsf(x[i]), (g_mode & 4) ? r->Ek[i] : r->E) <= 0.0f)) z = 0;
        if (z) return 3;
    }
    return hit ? 1 : 2;
}

static void sim_node_fwd(const void* bv, const void* nv, double ox, double oy, double oz, double dx, double dy,
                         double dz, int lh, double lt, int rh, double rt, double bt) {
    const BVH* b = (const BVH*)bv;
    const Node* n = (const Node*)nv;
    if (n->left < 0 && n->right < 0) return;  /* a leaf: no child tests */
    uint64_t c[kSimWords] = {0};
    c[kNodes] = 1;
    const R32 r = ray32(ox, oy, oz, dx, dy, dz);
    if (!r.ok) c[kIneligible] = 1;
    int st[2] = {0, 0}, vis[2] = {0, 0}, uv[2] = {0, 0};
    float lo[2] = {0, 0}, hi[2] = {0, 0};
    const int eh[2] = {lh, rh};
    const double et[2] = {lt, rt};
    const int64_t kid[2] = {n->left, n->right};
    for (int s = 0; s < 2; ++s) {
        if (kid[s] < 0) continue;
        c[kKids]++;
        float v;
        st[s] = cls32(&r, &b->nodes[kid[s]].aabb, &v);
        const float m = fmaf(kEps, v, r.E);
        lo[s] = v - m; hi[s] = v + m;
        if (st[s] == 3) { st[s] = 1; lo[s] = hi[s] = 0.0f; }
        if (st[s] == 0) { c[kMissC]++; if (eh[s]) { c[kViol]++; c[kViolMiss]++; } }
        else if (st[s] == 1) {
            c[kHitC]++;
            if (!eh[s]) { c[kViol]++; c[kViolHit]++; if (g_cnt[kViolHit] < 3) { g_cnt[kViolHit]++; fprintf(stderr, "hit: E=%g o=(%.17g %.17g %.17g) d=(%.17g %.17g %.17g) box=(%.9g %.9g %.9g)-(%.9g %.9g %.9g) ok=%d\n", r.E, ox, oy, oz, dx, dy, dz, b->nodes[kid[s]].aabb.min.x, b->nodes[kid[s]].aabb.min.y, b->nodes[kid[s]].aabb.min.z, b->nodes[kid[s]].aabb.max.x, b->nodes[kid[s]].aabb.max.y, b->nodes[kid[s]].aabb.max.z, r.ok); } } else if (!((double)lo[s] <= et[s] && et[s] <= (double)hi[s])) { c[kViol]++; c[kViolIv]++; if (c[kViolIv] == 1 && g_cnt[kViolIv] < 5) fprintf(stderr, "iv: v=%.17g lo=%.9g hi=%.9g E=%g o=(%g %g %g) d=(%g %g %g) box=(%.9g %.9g %.9g)-(%.9g %.9g %.9g)\n", et[s], lo[s], hi[s], r.E, ox, oy, oz, dx, dy, dz, b->nodes[kid[s]].aabb.min.x, b->nodes[kid[s]].aabb.min.y, b->nodes[kid[s]].aabb.min.z, b->nodes[kid[s]].aabb.max.x, b->nodes[kid[s]].aabb.max.y, b->nodes[kid[s]].aabb.max.z); }
        } else c[kUnc]++;
        if (st[s] == 1) {  /* visit <=> hit && v < bt */
            if ((double)hi[s] < bt) vis[s] = 1;
            else if ((double)lo[s] >= bt) vis[s] = 0;
            else uv[s] = 1;
        } else if (st[s] == 2) uv[s] = 1;
    }
    int exact = uv[0] || uv[1] || !r.ok;
    if (uv[0] || uv[1]) c[kVisitUnc]++;
    if (!exact && vis[0] && vis[1]) {  /* near-first order: left first <=> v_l < v_r */
        if (!(hi[0] < lo[1] || lo[0] >= hi[1])) { c[kOrderUnc]++; exact = 1; }
    }
    if (exact) c[kNodeExact]++;
#pragma omp critical(sim)
    for (int i = 0; i < kSimWords; ++i) g_cnt[i] += c[i];
}

static void sim_pop_fwd(const void* bv, int64_t ci, double ox, double oy, double oz, double dx, double dy, double dz,
                        double v, double b2) {
    const BVH* b = (const BVH*)bv;
    const R32 r = ray32(ox, oy, oz, dx, dy, dz);
    float vv;
    (void)cls32(&r, &b->nodes[ci].aabb, &vv);
    const float m = fmaf(kEps, vv, r.E);
    const float lo = vv - m, hi = vv + m;
    uint64_t unc = !((double)hi < b2 || (double)lo >= b2);
    uint64_t viol = !((double)lo <= v && v <= (double)hi);
#pragma omp critical(sim)
    { g_cnt[kPops]++; g_cnt[kPopUnc] += unc; g_cnt[kViol] += viol; g_cnt[kViolPop] += viol; }
}

void sim_read(uint64_t* out) {
    for (int i = 0; i < kSimWords; ++i) { out[i] = g_cnt[i]; g_cnt[i] = 0; }
}
