/*
 * oracle.c — plain-C restatement of uncerso/cpu-raytracing-rt's hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h): the checker and the CPU baseline,
 * never linked into the product.  Every function cites the reference
 * file:line it restates.  Compiled with -ffp-contract=off: the reference is
 * Rust, which never contracts a*b+c into an FMA.
 *
 * Third-party arithmetic restated (not vendored in /root/reference):
 *  - cgmath ^0.18 (Cargo.toml:7): dot = (x*x'+y*y')+z*z'; normalize = v*(1/|v|);
 *    Quaternion::rotate_vector: t = q.v x v + v*q.s; q.v x t * 2 + v;
 *    conjugate = (s, -v); Matrix3::determinant = cofactor expansion down
 *    column 0; Matrix3*Vector3 = (row_i . v).
 *  - rand ^0.8.5 (Cargo.toml:9): Standard f64 = (u64>>11)*2^-53;
 *    UniformFloat::sample_single (half-open) = ((u64>>12 | 1.0) - 1)*scale+low,
 *    retry while >= high; new_inclusive scale = (hi-lo)/(1-2^-52);
 *    UniformInt widening-multiply rejection; Bernoulli p_int = (p*2^64) as u64.
 *    The ChaCha12 ThreadRng STREAM is replaced by a counter-based
 *    Philox4x32-10 stream per (pixel, sample): the reference's stream is
 *    OS-seeded and irreproducible (main.rs:95), so only the transforms and
 *    distributions are restated, not the bits.
 */
#define _GNU_SOURCE
#include "oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ======================================================================= */
/* types.rs:5-14                                                            */
/* ======================================================================= */
#define R_PI 3.14159265358979323846264338327950288 /* std::f64::consts::PI */
static const double R_EPSILON = 2.220446049250313080847263336181640625e-16 * 512.0; /* types.rs:14 */

typedef struct { double x, y, z; } V3;
typedef struct { double s; V3 v; } Q; /* cgmath Quaternion { s, v } */
typedef struct { V3 min, max; } AABB;

static inline V3 v3(double x, double y, double z) { V3 r = {x, y, z}; return r; }
static inline V3 vadd(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline V3 vsub(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline V3 vmul(V3 a, V3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline V3 vdiv(V3 a, V3 b) { return v3(a.x / b.x, a.y / b.y, a.z / b.z); }
static inline V3 vscale(V3 a, double s) { return v3(a.x * s, a.y * s, a.z * s); }
static inline V3 vdivs(V3 a, double s) { return v3(a.x / s, a.y / s, a.z / s); }
static inline V3 vneg(V3 a) { return v3(-a.x, -a.y, -a.z); }
static inline double vdot(V3 a, V3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
static inline V3 vcross(V3 a, V3 b) {
    return v3((a.y * b.z) - (a.z * b.y), (a.z * b.x) - (a.x * b.z), (a.x * b.y) - (a.y * b.x));
}
static inline double vmag(V3 a) { return sqrt(vdot(a, a)); }
static inline V3 vnormalize(V3 a) { return vscale(a, 1.0 / vmag(a)); }
static inline double vget(V3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }
static inline V3 vld(const double* p) { return v3(p[0], p[1], p[2]); }
static inline void vst(double* p, V3 a) { p[0] = a.x; p[1] = a.y; p[2] = a.z; }
static inline Q qconj(Q q) { Q r = {q.s, vneg(q.v)}; return r; }
static inline V3 qrot(Q q, V3 v) { /* cgmath Quaternion * Vector3 */
    V3 tmp = vadd(vcross(q.v, v), vscale(v, q.s));
    return vadd(vscale(vcross(q.v, tmp), 2.0), v);
}
static inline Q qld(const double* p) { Q q = {p[0], v3(p[1], p[2], p[3])}; return q; }

/* ======================================================================= */
/* aabb.rs                                                                  */
/* ======================================================================= */
static inline double fmin_r(double a, double b) { return a < b ? a : b; } /* aabb.rs:34-36 */
static inline double fmax_r(double a, double b) { return b < a ? a : b; } /* aabb.rs:38-40 */
static inline AABB aabb_empty(void) { /* aabb.rs:16-21 */
    AABB a = {v3(INFINITY, INFINITY, INFINITY), v3(-INFINITY, -INFINITY, -INFINITY)};
    return a;
}
static inline void aabb_extend(AABB* a, V3 v) { /* aabb.rs:23-26 */
    a->min = v3(fmin_r(a->min.x, v.x), fmin_r(a->min.y, v.y), fmin_r(a->min.z, v.z));
    a->max = v3(fmax_r(a->max.x, v.x), fmax_r(a->max.y, v.y), fmax_r(a->max.z, v.z));
}
static inline void aabb_extend_aabb(AABB* a, const AABB* b) { /* aabb.rs:28-31 */
    a->min = v3(fmin_r(a->min.x, b->min.x), fmin_r(a->min.y, b->min.y), fmin_r(a->min.z, b->min.z));
    a->max = v3(fmax_r(a->max.x, b->max.x), fmax_r(a->max.y, b->max.y), fmax_r(a->max.z, b->max.z));
}
static inline double safe_min(double a, double b) { /* aabb.rs:90-98 */
    if (!isfinite(a)) return b;
    if (!isfinite(b)) return a;
    return fmin_r(a, b);
}
static inline double safe_max(double a, double b) { /* aabb.rs:100-108 */
    if (!isfinite(a)) return b;
    if (!isfinite(b)) return a;
    return fmax_r(a, b);
}
static inline int aabb_inside(const AABB* a, V3 o) { /* aabb.rs:80-87 */
    for (int i = 0; i < 3; ++i)
        if (vget(o, i) < vget(a->min, i) || vget(a->max, i) < vget(o, i)) return 0;
    return 1;
}
/* AABB::intersects (aabb.rs:51-78): returns 1 and *t on Some. */
static int aabb_intersects(const AABB* a, V3 o, V3 d, double* t) {
    for (int i = 0; i < 3; ++i)
        if (vget(d, i) == 0.0 && (vget(o, i) < vget(a->min, i) || vget(a->max, i) < vget(o, i))) return 0;
    if (aabb_inside(a, o)) { *t = 0.0; return 1; }
    V3 tmin = vdiv(vsub(a->min, o), d);
    V3 tmax = vdiv(vsub(a->max, o), d);
    V3 t1 = v3(safe_min(tmin.x, tmax.x), safe_min(tmin.y, tmax.y), safe_min(tmin.z, tmax.z));
    V3 t2 = v3(safe_max(tmin.x, tmax.x), safe_max(tmin.y, tmax.y), safe_max(tmin.z, tmax.z));
    double tn = safe_max(safe_max(t1.x, t1.y), t1.z);
    double tf = safe_min(safe_min(t2.x, t2.y), t2.z);
    if (tn > tf) return 0;
    if (0.0 <= tn) { *t = tn; return 1; }
    if (0.0 <= tf) { *t = tf; return 1; }
    return 0;
}

/* ======================================================================= */
/* intersections.rs:10-40, primitives/{plane,box,ellipsoid,triangle}.rs    */
/* ======================================================================= */
typedef struct { double t; V3 ng, ns; int inside; } Hit;
typedef struct { int n; Hit h[2]; } Hits; /* Intersections::{None,One,Two} */

static inline Hit hit_geom(double t, V3 n, int inside) { Hit h = {t, n, n, inside}; return h; }
static inline Hit hit_rotated(Hit h, Q q) { /* intersections.rs:32-39 */
    Hit r = {h.t, vnormalize(qrot(q, h.ng)), vnormalize(qrot(q, h.ns)), h.inside};
    return r;
}

/* plane.rs:11-21 */
static int plane_hit(V3 nrm, V3 o, V3 d, Hit* out) {
    double nd = vdot(nrm, d);
    double t = -vdot(nrm, o) / nd;
    if (t < 0.0) return 0;
    *out = hit_geom(t, vscale(nrm, nd <= 0.0 ? 1.0 : -1.0), 0);
    return 1;
}

/* box.rs:50-115 */
typedef struct { double t; double normal; int dim; } BPI;
static inline V3 bpi_normal(BPI p) { /* box.rs:64-72 */
    if (p.dim == 0) return v3(p.normal, 0.0, 0.0);
    if (p.dim == 1) return v3(0.0, p.normal, 0.0);
    return v3(0.0, 0.0, p.normal);
}
/* returns 0 None, 1 One(exit), 2 Two(entry, exit) */
static int box_coef(V3 s, V3 o, V3 d, BPI* entry, BPI* exit_) { /* box.rs:75-106 */
    int have = 0;
    BPI mx = {0, 0, 0}, mn = {0, 0, 0};
    for (int i = 0; i < 3; ++i) {
        double di = vget(d, i), oi = vget(o, i), si = vget(s, i);
        if (di == 0.0 && si < fabs(oi)) return 0;
        if (di == 0.0) continue; /* box_planes_intersect -> None (box.rs:109-111) */
        double t1 = (si - oi) / di;
        double t2 = (-si - oi) / di;
        double a, b, nrm;
        if (t1 < t2) { a = t1; b = t2; nrm = 1.0; } else { a = t2; b = t1; nrm = -1.0; }
        BPI p1 = {a, nrm, i}, p2 = {b, nrm, i};
        if (!have) { mx = p1; mn = p2; have = 1; }
        else {
            mx = (p1.t < mx.t) ? mx : p1; /* BoxPlaneIntersection::max, box.rs:57-59 */
            mn = (p2.t < mn.t) ? p2 : mn; /* BoxPlaneIntersection::min, box.rs:60-62 */
        }
    }
    if (!have) return 0;
    if (mn.t < mx.t) return 0;
    if (0.0 <= mx.t) { *entry = mx; *exit_ = mn; return 2; }
    if (0.0 <= mn.t) { *exit_ = mn; return 1; }
    return 0;
}
static Hits box_all(V3 s, V3 o, V3 d) { /* box.rs:35-46 */
    Hits r; r.n = 0;
    BPI e, x;
    int k = box_coef(s, o, d, &e, &x);
    if (k == 1) { r.n = 1; r.h[0] = hit_geom(x.t, bpi_normal(x), 1); }
    else if (k == 2) { r.n = 2; r.h[0] = hit_geom(e.t, bpi_normal(e), 0); r.h[1] = hit_geom(x.t, bpi_normal(x), 1); }
    return r;
}
static int box_hit(V3 s, V3 o, V3 d, Hit* out) { /* box.rs:21-33 */
    BPI e, x;
    int k = box_coef(s, o, d, &e, &x);
    if (k == 1) { *out = hit_geom(x.t, bpi_normal(x), 1); return 1; }
    if (k == 2) { *out = hit_geom(e.t, bpi_normal(e), 0); return 1; }
    return 0;
}

/* ellipsoid.rs:49-76; returns 0/1/2 with t1 (entry) / t2 (exit) */
static int ell_coef(V3 r, V3 o, V3 d, double* t1o, double* t2o) {
    V3 oo = vdiv(o, r), dd = vdiv(d, r);
    double c = vdot(oo, oo), b = vdot(oo, dd), a = vdot(dd, dd);
    double disc = b * b - a * (c - 1.0);
    if (disc < 0.0) return 0;
    double ds = sqrt(disc);
    double t1 = (-b + ds) / a, t2 = (-b - ds) / a;
    if (t2 < t1) { double tmp = t1; t1 = t2; t2 = tmp; }
    if (0.0 <= t1) { *t1o = t1; *t2o = t2; return 2; }
    if (0.0 <= t2) { *t2o = t2; return 1; }
    return 0;
}
static inline V3 ell_normal(V3 r, V3 o, V3 d, double t) { /* p/r/r normalised (ellipsoid.rs:26,29) */
    V3 p = vadd(o, vscale(d, t));
    return vnormalize(vdiv(vdiv(p, r), r));
}
static Hits ell_all(V3 r, V3 o, V3 d) { /* ellipsoid.rs:34-46 */
    Hits h; h.n = 0;
    double t1 = 0, t2 = 0;
    int k = ell_coef(r, o, d, &t1, &t2);
    if (k == 1) { h.n = 1; h.h[0] = hit_geom(t2, vneg(ell_normal(r, o, d, t2)), 1); }
    else if (k == 2) {
        h.n = 2;
        h.h[0] = hit_geom(t1, ell_normal(r, o, d, t1), 0);
        h.h[1] = hit_geom(t2, vneg(ell_normal(r, o, d, t2)), 1);
    }
    return h;
}
static int ell_hit(V3 r, V3 o, V3 d, Hit* out) { /* ellipsoid.rs:21-32 */
    double t1 = 0, t2 = 0;
    int k = ell_coef(r, o, d, &t1, &t2);
    if (k == 1) { *out = hit_geom(t2, vneg(ell_normal(r, o, d, t2)), 1); return 1; }
    if (k == 2) { *out = hit_geom(t1, ell_normal(r, o, d, t1), 0); return 1; }
    return 0;
}

/* triangle.rs */
typedef struct {
    V3 a, ba, ca, ng; double inv_area; V3 na, nb, nc;
} Triangle;
static Triangle tri_props(V3 a, V3 b, V3 c) { /* triangle.rs:41-47 */
    Triangle t;
    t.a = a; t.ba = vsub(b, a); t.ca = vsub(c, a);
    V3 sized = vcross(t.ba, t.ca);
    double area = sqrt(vdot(sized, sized)) / 2.0;
    t.ng = vnormalize(sized);
    t.inv_area = 1.0 / area;
    return t;
}
static Triangle tri_new_smooth(V3 a, V3 b, V3 c, V3 na, V3 nb, V3 nc) { /* triangle.rs:20-23 */
    Triangle t = tri_props(a, b, c);
    t.na = na; t.nb = nb; t.nc = nc;
    return t;
}
static Triangle tri_new_geom(V3 a, V3 b, V3 c) { /* triangle.rs:25-28 */
    Triangle t = tri_props(a, b, c);
    t.na = t.ng; t.nb = t.ng; t.nc = t.ng;
    return t;
}
/* Triangle::intersection (triangle.rs:49-80) */
static int tri_hit(const Triangle* tr, V3 o, V3 d, Hit* out) {
    V3 m0 = tr->ba, m1 = tr->ca, m2 = vneg(d); /* Mat3::from_cols(ba, ca, -dir) */
    /* cgmath Matrix3::determinant, m[c][r] */
    double det = m0.x * (m1.y * m2.z - m2.y * m1.z)
               - m1.x * (m0.y * m2.z - m2.y * m0.z)
               + m2.x * (m0.y * m1.z - m1.y * m0.z);
    if (fabs(det) < 1e-11) return 0;
    V3 x0 = vdivs(vcross(m1, m2), det);
    V3 x1 = vdivs(vcross(m2, m0), det);
    V3 x2 = vdivs(vcross(m0, m1), det);
    V3 w = vsub(o, tr->a);
    double u = vdot(x0, w), v = vdot(x1, w), t = vdot(x2, w); /* transpose then row . w */
    if (u < 0.0 || v < 0.0 || 1.0 < u + v || t < 0.0) return 0;
    V3 n = tr->ng;
    V3 sn = vnormalize(vadd(vadd(tr->na, vscale(vsub(tr->nb, tr->na), u)), vscale(vsub(tr->nc, tr->na), v)));
    int inside = vdot(d, n) > 0.0;
    out->t = t;
    out->ng = inside ? vneg(n) : n;
    out->ns = inside ? vneg(sn) : sn;
    out->inside = inside;
    return 1;
}

/* ======================================================================= */
/* scene.rs — primitives and the scene model                                */
/* ======================================================================= */
typedef struct {
    int type; V3 shape; V3 pos; Q rot; uint32_t mat; AABB aabb; int64_t gid;
} Shape;
typedef struct {
    Triangle tri; uint32_t mat; AABB aabb; int64_t gid;
} Tri;

typedef struct { AABB aabb; int64_t left, right; uint64_t start, end; } Node; /* bvh.rs:48-54 */
typedef struct { Node* nodes; uint64_t n_nodes; uint64_t n; Shape* s; Tri* t; uint32_t depth; } BVH;

struct oracle_scene {
    rt_material* mats; uint32_t n_mats;
    Shape* planes; uint32_t n_planes;
    BVH boxes, ells, tris;       /* scene.rs:56-62 */
    BVH lboxes, lells, ltris;    /* scene.rs:64-69 */
};

static AABB rotated_aabb(AABB a, Q r) { /* scene.rs:255-268 */
    V3 mn = a.min, mx = a.max;
    AABB b = aabb_empty();
    aabb_extend(&b, qrot(r, v3(mn.x, mn.y, mn.z)));
    aabb_extend(&b, qrot(r, v3(mn.x, mn.y, mx.z)));
    aabb_extend(&b, qrot(r, v3(mn.x, mx.y, mn.z)));
    aabb_extend(&b, qrot(r, v3(mn.x, mx.y, mx.z)));
    aabb_extend(&b, qrot(r, v3(mx.x, mn.y, mn.z)));
    aabb_extend(&b, qrot(r, v3(mx.x, mn.y, mx.z)));
    aabb_extend(&b, qrot(r, v3(mx.x, mx.y, mn.z)));
    aabb_extend(&b, qrot(r, v3(mx.x, mx.y, mx.z)));
    return b;
}

/* ---- BVH build (bvh.rs:11-17, 75-140, 224-256) ------------------------- */
typedef struct { const int64_t* key; } SortCtx;  /* total_order_key of each primitive's midpoint on one axis */
static inline double axis_of(V3 v, int axis) { return vget(v, axis); }
static inline int64_t total_order_key(double x) { /* f64::total_cmp */
    int64_t b; memcpy(&b, &x, 8);
    b ^= (int64_t)(((uint64_t)(b >> 63)) >> 1);
    return b;
}
/* midpoint_comparator (bvh.rs:137-140); ties broken by the list index so the
   tree is deterministic (the reference's sort_unstable tie order is not). */
static int cmp_mid(const void* pa, const void* pb, void* pctx) {
    const SortCtx* c = (const SortCtx*)pctx;
    uint64_t ia = *(const uint64_t*)pa, ib = *(const uint64_t*)pb;
    int64_t ka = c->key[ia], kb = c->key[ib];
    if (ka < kb) return -1;
    if (ka > kb) return 1;
    return ia < ib ? -1 : (ia > ib ? 1 : 0);
}
/* Sort by cmp_mid: a parallel merge sort (OpenMP tasks) above 1M elements.
   cmp_mid is a total order (midpoint key, then list index), so every correct
   sort gives the same permutation as qsort_r. */
static void psort(uint64_t* a, uint64_t n, const int64_t* key, uint64_t* tmp) {
    SortCtx ctx = {key};
    if (n < (1u << 20)) { qsort_r(a, n, sizeof(uint64_t), cmp_mid, &ctx); return; }
    const uint64_t h = n / 2;
#pragma omp task
    psort(a, h, key, tmp);
#pragma omp task
    psort(a + h, n - h, key, tmp + h);
#pragma omp taskwait
    uint64_t i = 0, j = h, k = 0;
    while (i < h && j < n) tmp[k++] = cmp_mid(&a[j], &a[i], &ctx) < 0 ? a[j++] : a[i++];
    while (i < h) tmp[k++] = a[i++];
    while (j < n) tmp[k++] = a[j++];
    memcpy(a, tmp, n * sizeof(uint64_t));
}
static inline double aabb_score(const AABB* a) { /* bvh.rs:115-118 */
    V3 s = vsub(a->max, a->min);
    return s.x * s.y + s.x * s.z + s.y * s.z;
}
typedef struct {
    const AABB* boxes; uint64_t* idx; Node* nodes; uint64_t n_nodes, cap;
    AABB* fwd; AABB* bwd; uint32_t max_depth;
    const int64_t* keys[3];  /* midpoint sort keys per axis (computed once per build) */
} Builder;
static void sort_mid(Builder* b, uint64_t lo, uint64_t n, int axis) {
    if (n < (1u << 20)) {
        SortCtx ctx = {b->keys[axis]};
        qsort_r(b->idx + lo, n, sizeof(uint64_t), cmp_mid, &ctx);
        return;
    }
    uint64_t* tmp = (uint64_t*)malloc(n * sizeof(uint64_t));
    psort(b->idx + lo, n, b->keys[axis], tmp);
    free(tmp);
}
static uint64_t push_node(Builder* b, Node n) {
    if (b->n_nodes == b->cap) {
        b->cap = b->cap ? b->cap * 2 : 64;
        b->nodes = (Node*)realloc(b->nodes, b->cap * sizeof(Node));
    }
    b->nodes[b->n_nodes] = n;
    return b->n_nodes++;
}
/* Subtrees of at least this many primitives build their two children as
   parallel OpenMP tasks (the 10M-triangle C5 tree: minutes -> about a minute). */
enum { kParMin = 65536 };
static void build_sub(const Builder* parent, uint64_t lo, uint64_t hi, uint32_t depth, Builder* out);
static uint64_t splice(Builder* b, Builder* sub);
static uint64_t build_nodes(Builder* b, uint64_t lo, uint64_t hi, uint32_t depth) { /* bvh.rs:75-113 */
    uint64_t n = hi - lo;
    if (depth > b->max_depth) b->max_depth = depth;
    AABB box = aabb_empty();
    for (uint64_t i = lo; i < hi; ++i) aabb_extend_aabb(&box, &b->boxes[b->idx[i]]);
    if (n <= 4) {
        Node leaf = {box, -1, -1, lo, hi};
        return push_node(b, leaf);
    }
    uint64_t best_first = n;
    double best_score = aabb_score(&box) * (double)n;
    int best_axis = -1;
    for (int axis = 0; axis < 3; ++axis) { /* subdivision_score (bvh.rs:120-135) */
        sort_mid(b, lo, n, axis);
        /* AABBSplitsBuilder::make_splits (bvh.rs:238-255) */
        AABB acc = aabb_empty();
        for (uint64_t i = 0; i + 1 < n; ++i) { aabb_extend_aabb(&acc, &b->boxes[b->idx[lo + i]]); b->fwd[i] = acc; }
        acc = aabb_empty();
        for (uint64_t k = 0; k + 1 < n; ++k) { aabb_extend_aabb(&acc, &b->boxes[b->idx[hi - 1 - k]]); b->bwd[k] = acc; }
        for (uint64_t i = 0; i + 1 < n; ++i) {
            uint64_t lc = i + 1, rc = n - lc;
            double score = aabb_score(&b->fwd[i]) * (double)lc + aabb_score(&b->bwd[(n - 1) - i - 1]) * (double)rc;
            if (score < best_score) { best_first = lc; best_score = score; best_axis = axis; }
        }
    }
    if (best_axis < 0) { /* SubdivisionType::SameNode (bvh.rs:93-96) */
        Node leaf = {box, -1, -1, lo, hi};
        return push_node(b, leaf);
    }
    sort_mid(b, lo, n, best_axis);
    Node placeholder = {box, -1, -1, 0, 0};
    uint64_t me = push_node(b, placeholder);
    uint64_t l, r;
    if (n >= kParMin) { /* both subtrees at once (OpenMP tasks), spliced in pre-order */
        Builder L, R;
#pragma omp task shared(L)
        build_sub(b, lo, lo + best_first, depth + 1, &L);
#pragma omp task shared(R)
        build_sub(b, lo + best_first, hi, depth + 1, &R);
#pragma omp taskwait
        l = splice(b, &L);
        r = splice(b, &R);
    } else {
        l = build_nodes(b, lo, lo + best_first, depth + 1);
        r = build_nodes(b, lo + best_first, hi, depth + 1);
    }
    b->nodes[me].left = (int64_t)l;
    b->nodes[me].right = (int64_t)r;
    return me;
}
/* A subtree built on its own (node indices from 0, own sort scratch).  The
   tree is the sequential build's: every node's split depends only on its own
   primitive range, and pre-order is parent, left subtree, right subtree. */
static void build_sub(const Builder* parent, uint64_t lo, uint64_t hi, uint32_t depth, Builder* out) {
    const uint64_t n = hi - lo;
    Builder b = {parent->boxes, parent->idx, NULL, 0, 0, NULL, NULL, 0, {parent->keys[0], parent->keys[1], parent->keys[2]}};
    b.fwd = (AABB*)malloc(sizeof(AABB) * (n > 1 ? n - 1 : 1));
    b.bwd = (AABB*)malloc(sizeof(AABB) * (n > 1 ? n - 1 : 1));
    build_nodes(&b, lo, hi, depth);
    free(b.fwd); free(b.bwd);
    b.fwd = b.bwd = NULL;
    *out = b;
}
static uint64_t splice(Builder* b, Builder* sub) { /* append sub's nodes; returns its root's index */
    const uint64_t off = b->n_nodes;
    for (uint64_t i = 0; i < sub->n_nodes; ++i) {
        Node nd = sub->nodes[i];
        if (nd.left >= 0) { nd.left += (int64_t)off; nd.right += (int64_t)off; }
        push_node(b, nd);
    }
    if (sub->max_depth > b->max_depth) b->max_depth = sub->max_depth;
    free(sub->nodes);
    return off;
}
static void bvh_build(BVH* bvh, const AABB* boxes, uint64_t n, uint64_t* perm_out) {
    bvh->n = n; bvh->nodes = NULL; bvh->n_nodes = 0; bvh->depth = 0;
    for (uint64_t i = 0; i < n; ++i) perm_out[i] = i;
    if (n == 0) return; /* BVH::new(vec![]) builds a leaf over nothing; never traversed (bvh.rs:29) */
    /* the midpoint comparator's keys (bvh.rs:137-140: (min + max) / 2 per axis,
       f64::total_cmp order), once per primitive instead of per comparison */
    int64_t* keys = (int64_t*)malloc(sizeof(int64_t) * 3 * n);
    for (uint64_t i = 0; i < n; ++i)
        for (int axis = 0; axis < 3; ++axis)
            keys[axis * n + i] = total_order_key((axis_of(boxes[i].min, axis) + axis_of(boxes[i].max, axis)) / 2.0);
    Builder root = {boxes, perm_out, NULL, 0, 0, NULL, NULL, 0, {keys, keys + n, keys + 2 * n}};
    Builder b;
    if (n >= kParMin) {
#pragma omp parallel
#pragma omp single
        build_sub(&root, 0, n, 1, &b);
    } else {
        build_sub(&root, 0, n, 1, &b);
    }
    free(keys);
    bvh->nodes = b.nodes; bvh->n_nodes = b.n_nodes; bvh->depth = b.max_depth;
}
static void bvh_build_shapes(BVH* bvh, Shape* list, uint64_t n) {
    AABB* boxes = (AABB*)calloc(n ? n : 1, sizeof(AABB));
    uint64_t* perm = (uint64_t*)malloc(sizeof(uint64_t) * (n ? n : 1));
    for (uint64_t i = 0; i < n; ++i) boxes[i] = list[i].aabb;
    bvh_build(bvh, boxes, n, perm);
    bvh->s = (Shape*)malloc(sizeof(Shape) * (n ? n : 1));
    for (uint64_t i = 0; i < n; ++i) bvh->s[i] = list[perm[i]];
    bvh->t = NULL;
    free(boxes); free(perm);
}
static void bvh_build_tris(BVH* bvh, Tri* list, uint64_t n) {
    AABB* boxes = (AABB*)calloc(n ? n : 1, sizeof(AABB));
    uint64_t* perm = (uint64_t*)malloc(sizeof(uint64_t) * (n ? n : 1));
    for (uint64_t i = 0; i < n; ++i) boxes[i] = list[i].aabb;
    bvh_build(bvh, boxes, n, perm);
    bvh->t = (Tri*)malloc(sizeof(Tri) * (n ? n : 1));
    for (uint64_t i = 0; i < n; ++i) bvh->t[i] = list[perm[i]];
    bvh->s = NULL;
    free(boxes); free(perm);
}
static void bvh_free(BVH* b) { free(b->nodes); free(b->s); free(b->t); }

static int is_light(const rt_material* m) { /* scene.rs:225-227 */
    return m->emission[0] != 0.0 || m->emission[1] != 0.0 || m->emission[2] != 0.0;
}

/* Scene::new / make_scenes (scene.rs:180-223) */
oracle_scene* oracle_scene_create(const rt_scene_desc* d) {
    if (!d) return NULL;
    oracle_scene* s = (oracle_scene*)calloc(1, sizeof(oracle_scene));
    s->n_mats = d->n_materials;
    s->mats = (rt_material*)malloc(sizeof(rt_material) * (d->n_materials ? d->n_materials : 1));
    if (d->n_materials) memcpy(s->mats, d->materials, sizeof(rt_material) * d->n_materials);
    uint32_t ns = d->n_shapes;
    Shape* planes = (Shape*)malloc(sizeof(Shape) * (ns ? ns : 1));
    Shape* boxes = (Shape*)malloc(sizeof(Shape) * (ns ? ns : 1));
    Shape* ells = (Shape*)malloc(sizeof(Shape) * (ns ? ns : 1));
    uint32_t np = 0, nb = 0, ne = 0;
    for (uint32_t i = 0; i < ns; ++i) {
        const rt_shape* sh = &d->shapes[i];
        Shape x;
        x.type = (int)sh->type; x.shape = vld(sh->shape); x.pos = vld(sh->position); x.rot = qld(sh->rotation);
        x.mat = sh->material; x.gid = i;
        if (sh->type == RT_SHAPE_PLANE) { /* Primitive::new_without_aabb (scene.rs:126-136) */
            x.aabb = aabb_empty();
            planes[np++] = x;
        } else { /* Box::new / Ellipsoid::new (box.rs:12-17, ellipsoid.rs:12-17) + Primitive::new (scene.rs:109-122) */
            AABB local = aabb_empty();
            aabb_extend(&local, x.shape);
            aabb_extend(&local, vneg(x.shape));
            AABB w = rotated_aabb(local, x.rot);
            w.min = vadd(w.min, x.pos);
            w.max = vadd(w.max, x.pos);
            x.aabb = w;
            if (sh->type == RT_SHAPE_BOX) boxes[nb++] = x; else ells[ne++] = x;
        }
    }
    uint64_t nt = d->n_triangles;
    Tri* tris = (Tri*)malloc(sizeof(Tri) * (nt ? nt : 1));
    for (uint64_t j = 0; j < nt; ++j) {
        const double* vv = d->tri_vertices + 9 * j;
        Tri t;
        t.mat = d->tri_material ? d->tri_material[j] : 0;
        t.gid = (int64_t)ns + (int64_t)j;
        if (d->tri_mode == RT_TRI_GLTF) {
            /* Triangle::new_with_smooth_normal + instantiate (gltf/scene_builder.rs:42-55,342-356) */
            const double* nn = d->tri_normals + 9 * j;
            t.tri = tri_new_smooth(vld(vv), vld(vv + 3), vld(vv + 6), vld(nn), vld(nn + 3), vld(nn + 6));
            AABB bb = aabb_empty();
            aabb_extend(&bb, t.tri.a);
            aabb_extend(&bb, vadd(t.tri.a, t.tri.ba));
            aabb_extend(&bb, vadd(t.tri.a, t.tri.ca));
            t.aabb = bb;
        } else {
            /* Triangle::new_with_geometry_normals (scene_parser.rs:71-73) then
               TrianglePrimitive::new (scene.rs:139-165) */
            Triangle m = tri_new_geom(vld(vv), vld(vv + 3), vld(vv + 6));
            V3 pos = d->tri_position ? vld(d->tri_position + 3 * j) : v3(0, 0, 0);
            Q rot = d->tri_rotation ? qld(d->tri_rotation + 4 * j) : (Q){1.0, {0, 0, 0}};
            V3 a = vadd(qrot(rot, m.a), pos);
            V3 b = vadd(qrot(rot, vadd(m.ba, m.a)), pos);
            V3 c = vadd(qrot(rot, vadd(m.ca, m.a)), pos);
            V3 na = qrot(rot, m.na), nb = qrot(rot, m.nb), nc = qrot(rot, m.nc);
            t.tri = tri_new_smooth(a, b, c, na, nb, nc);
            AABB bb = aabb_empty();
            aabb_extend(&bb, a); aabb_extend(&bb, b); aabb_extend(&bb, c);
            t.aabb = bb;
        }
        tris[j] = t;
    }
    /* lights are copies (scene.rs:209-213, copy_if_light :229-241) */
    Shape* lb = (Shape*)malloc(sizeof(Shape) * (nb ? nb : 1));
    Shape* le = (Shape*)malloc(sizeof(Shape) * (ne ? ne : 1));
    Tri* lt = (Tri*)malloc(sizeof(Tri) * (nt ? nt : 1));
    uint32_t nlb = 0, nle = 0; uint64_t nlt = 0;
    for (uint32_t i = 0; i < nb; ++i) if (is_light(&s->mats[boxes[i].mat])) lb[nlb++] = boxes[i];
    for (uint32_t i = 0; i < ne; ++i) if (is_light(&s->mats[ells[i].mat])) le[nle++] = ells[i];
    for (uint64_t i = 0; i < nt; ++i) if (is_light(&s->mats[tris[i].mat])) lt[nlt++] = tris[i];
    bvh_build_shapes(&s->lboxes, lb, nlb);
    bvh_build_shapes(&s->lells, le, nle);
    bvh_build_tris(&s->ltris, lt, nlt);
    bvh_build_shapes(&s->ells, ells, ne);
    bvh_build_shapes(&s->boxes, boxes, nb);
    bvh_build_tris(&s->tris, tris, nt);
    s->planes = planes; s->n_planes = np;
    free(boxes); free(ells); free(tris); free(lb); free(le); free(lt);
    return s;
}
void oracle_scene_destroy(oracle_scene* s) {
    if (!s) return;
    bvh_free(&s->boxes); bvh_free(&s->ells); bvh_free(&s->tris);
    bvh_free(&s->lboxes); bvh_free(&s->lells); bvh_free(&s->ltris);
    free(s->planes); free(s->mats); free(s);
}
static const BVH* bvh_k(const oracle_scene* s, int k) {
    switch (k) {
    case 0: return &s->boxes; case 1: return &s->ells; case 2: return &s->tris;
    case 3: return &s->lboxes; case 4: return &s->lells; default: return &s->ltris;
    }
}
void oracle_scene_bvh_info(const oracle_scene* s, uint64_t nodes[6], uint32_t depth[6]) {
    for (int k = 0; k < 6; ++k) { nodes[k] = bvh_k(s, k)->n_nodes; depth[k] = bvh_k(s, k)->depth; }
}
uint64_t oracle_scene_bvh_dump(const oracle_scene* s, int k, int64_t* links, double* bounds) {
    const BVH* b = bvh_k(s, k);
    for (uint64_t i = 0; i < b->n_nodes; ++i) {
        const Node* n = &b->nodes[i];
        if (links) {
            links[4 * i + 0] = n->left; links[4 * i + 1] = n->right;
            links[4 * i + 2] = (int64_t)n->start; links[4 * i + 3] = (int64_t)n->end;
        }
        if (bounds) { vst(bounds + 6 * i, n->aabb.min); vst(bounds + 6 * i + 3, n->aabb.max); }
    }
    return b->n_nodes;
}
int64_t oracle_scene_bvh_prim(const oracle_scene* s, int k, uint64_t i) {
    const BVH* b = bvh_k(s, k);
    if (i >= b->n) return -1;
    return b->s ? b->s[i].gid : b->t[i].gid;
}

/* ======================================================================= */
/* Counters (canonical byte model)                            */
/* ======================================================================= */
typedef struct {
    uint64_t paths, segments, aabb, tri, shape, shaded, lq, lhits;
} Counters;

/* ======================================================================= */
/* Queries: intersections.rs, bvh.rs traversal                              */
/* ======================================================================= */
static inline void model_ray(const Shape* p, V3 o, V3 d, V3* mo, V3* md) { /* intersections.rs:93-99 */
    Q r = qconj(p->rot);
    *mo = qrot(r, vsub(o, p->pos));
    *md = qrot(r, d);
}
static int shape_hit(const Shape* p, V3 o, V3 d, Hit* h, Counters* c) { /* intersections.rs:101-104 */
    V3 mo, md;
    model_ray(p, o, d, &mo, &md);
    c->shape++;
    if (p->type == RT_SHAPE_PLANE) return plane_hit(p->shape, mo, md, h);
    if (p->type == RT_SHAPE_BOX) return box_hit(p->shape, mo, md, h);
    return ell_hit(p->shape, mo, md, h);
}
static Hits shape_all(const Shape* p, V3 o, V3 d, Counters* c) { /* intersections.rs:106-108 */
    V3 mo, md;
    model_ray(p, o, d, &mo, &md);
    c->shape++;
    if (p->type == RT_SHAPE_BOX) return box_all(p->shape, mo, md);
    if (p->type == RT_SHAPE_ELLIPSOID) return ell_all(p->shape, mo, md);
    Hits r; r.n = 0; Hit h;
    if (plane_hit(p->shape, mo, md, &h)) { r.n = 1; r.h[0] = h; }
    return r;
}
static inline int aabb_test(const AABB* a, V3 o, V3 d, double* t, Counters* c) {
    c->aabb++;
    return aabb_intersects(a, o, d, t);
}

typedef struct { int valid; Hit h; uint64_t prim; } Best; /* Option<(Intersection, &T)> */

/* Node::intersection (bvh.rs:151-186), recursive exactly as the reference */
static void node_closest(const BVH* b, uint64_t ni, V3 o, V3 d, Best* best, Counters* c) {
    const Node* n = &b->nodes[ni];
    for (uint64_t i = n->start; i < n->end; ++i) {
        Hit h; int ok;
        if (b->s) ok = shape_hit(&b->s[i], o, d, &h, c);
        else { c->tri++; ok = tri_hit(&b->t[i].tri, o, d, &h); }
        if (!ok) continue;
        if (!best->valid || h.t < best->h.t) { best->valid = 1; best->h = h; best->prim = i; } /* bvh.rs:213-222 */
    }
    double lt = 0, rt = 0;
    int lh = 0, rh = 0;
    if (n->left >= 0) lh = aabb_test(&b->nodes[n->left].aabb, o, d, &lt, c);
    if (n->right >= 0) rh = aabb_test(&b->nodes[n->right].aabb, o, d, &rt, c);
    double bt = best->valid ? best->h.t : INFINITY;
    double li = lh ? (lt < bt ? lt : bt) : bt;
    double ri = rh ? (rt < bt ? rt : bt) : bt;
#ifdef ORACLE_NODE_HOOK /* experiment builds only (tools/f32slab_sim.c): observes, changes nothing */
    ORACLE_NODE_HOOK(b, n, o, d, lh, lt, rh, rt, bt);
#endif
    if (li < bt) {
        if (ri < bt) {
            if (li < ri) {
                node_closest(b, (uint64_t)n->left, o, d, best, c);
                double b2 = best->valid ? best->h.t : INFINITY;
#ifdef ORACLE_POP_HOOK
                ORACLE_POP_HOOK(b, n->right, o, d, ri, b2);
#endif
                if (ri < b2) node_closest(b, (uint64_t)n->right, o, d, best, c);
            } else {
                node_closest(b, (uint64_t)n->right, o, d, best, c);
                double b2 = best->valid ? best->h.t : INFINITY;
#ifdef ORACLE_POP_HOOK
                ORACLE_POP_HOOK(b, n->left, o, d, li, b2);
#endif
                if (li < b2) node_closest(b, (uint64_t)n->left, o, d, best, c);
            }
        } else {
            node_closest(b, (uint64_t)n->left, o, d, best, c);
        }
    } else if (ri < bt) {
        node_closest(b, (uint64_t)n->right, o, d, best, c);
    }
}
static Best bvh_closest(const BVH* b, V3 o, V3 d, Counters* c) { /* bvh.rs:27-36 */
    Best best; best.valid = 0;
    if (b->n > 0) {
        double t;
        if (aabb_test(&b->nodes[0].aabb, o, d, &t, c)) node_closest(b, 0, o, d, &best, c);
    }
    return best;
}

/* The light-pdf accumulator passed as the intersect_lights callback
   (ray_sampler.rs:135-137). */
typedef struct { double impact; V3 dir; Counters* c; } PdfAcc;

static inline double prob_tri(const Triangle* t) { return t->inv_area; } /* intersection_probability.rs:9-13 */
static inline double prob_box(V3 s) { /* intersection_probability.rs:15-23 */
    double sum = (s.y * s.z + s.x * s.z) + s.x * s.y;
    return 1.0 / sum / 8.0;
}
static inline double prob_ell(V3 r, V3 ng) { /* intersection_probability.rs:25-35 */
    V3 coef = vmul(v3(r.y * r.z, r.x * r.z, r.x * r.y), ng);
    return 1.0 / (4.0 * R_PI * sqrt(vdot(coef, coef)));
}
static inline void pdf_cb(PdfAcc* acc, const Hit* h, double prob) {
    /* to_direction_probability (ray_sampler.rs:172-174) */
    double tdp = h->t * h->t / fabs(vdot(acc->dir, h->ng));
    acc->impact += prob * tdp;
    acc->c->lhits++;
}
/* Node::intersections (bvh.rs:188-210) */
static void node_all(const BVH* b, uint64_t ni, V3 o, V3 d, PdfAcc* acc) {
    const Node* n = &b->nodes[ni];
    Counters* c = acc->c;
    for (uint64_t i = n->start; i < n->end; ++i) {
        if (b->s) {
            const Shape* p = &b->s[i];
            Hits hs = shape_all(p, o, d, c);
            for (int k = 0; k < hs.n; ++k) {
                Hit h = hit_rotated(hs.h[k], p->rot); /* intersections.rs:88-89 */
                pdf_cb(acc, &h, p->type == RT_SHAPE_BOX ? prob_box(p->shape) : prob_ell(p->shape, h.ng));
            }
        } else {
            c->tri++;
            Hit h;
            if (tri_hit(&b->t[i].tri, o, d, &h)) pdf_cb(acc, &h, prob_tri(&b->t[i].tri)); /* intersections.rs:90 */
        }
    }
    double t;
    if (n->left >= 0 && aabb_test(&b->nodes[n->left].aabb, o, d, &t, c)) node_all(b, (uint64_t)n->left, o, d, acc);
    if (n->right >= 0 && aabb_test(&b->nodes[n->right].aabb, o, d, &t, c)) node_all(b, (uint64_t)n->right, o, d, acc);
}
static void bvh_all(const BVH* b, V3 o, V3 d, PdfAcc* acc) { /* bvh.rs:38-45 */
    if (b->n > 0) {
        double t;
        if (aabb_test(&b->nodes[0].aabb, o, d, &t, acc->c)) node_all(b, 0, o, d, acc);
    }
}

/* Closest hit over the whole scene: intersect (intersections.rs:42-62).
   Returns 1 with world hit, material and global id. */
typedef struct { Hit h; uint32_t mat; int64_t gid; } SceneHit;
static int scene_intersect(const oracle_scene* s, V3 o, V3 d, SceneHit* out, Counters* c) {
    int valid = 0;
    Hit best = {0};
    uint32_t mat = 0; int64_t gid = -1;
    Q rot = {1.0, {0, 0, 0}};
    for (uint32_t i = 0; i < s->n_planes; ++i) { /* :45-49 */
        Hit h;
        if (!shape_hit(&s->planes[i], o, d, &h, c)) continue;
        if (!valid || h.t < best.t) { valid = 1; best = h; mat = s->planes[i].mat; gid = s->planes[i].gid; rot = s->planes[i].rot; }
    }
    const BVH* sb[2] = {&s->boxes, &s->ells};
    for (int k = 0; k < 2; ++k) { /* :51-52 */
        Best r = bvh_closest(sb[k], o, d, c);
        if (!r.valid) continue;
        if (!valid || r.h.t < best.t) {
            const Shape* p = &sb[k]->s[r.prim];
            valid = 1; best = r.h; mat = p->mat; gid = p->gid; rot = p->rot;
        }
    }
    { /* :53, DONT_ROTATE :64 */
        Best r = bvh_closest(&s->tris, o, d, c);
        if (r.valid && (!valid || r.h.t < best.t)) {
            const Tri* p = &s->tris.t[r.prim];
            valid = 1; best = r.h; mat = p->mat; gid = p->gid;
            rot.s = 1.0; rot.v = v3(0.0, 0.0, 0.0);
        }
    }
    if (!valid) return 0;
    if (!(best.t * vmag(d) <= INFINITY)) return 0; /* :56 with max_dist = +inf */
    out->h = hit_rotated(best, rot);
    out->mat = mat; out->gid = gid;
    c->shaded++;
    return 1;
}

static double light_pdf(const oracle_scene* s, V3 pos, V3 dir, Counters* c) { /* ray_sampler.rs:132-139 */
    V3 o = vadd(pos, vscale(dir, R_EPSILON));
    PdfAcc acc = {0.0, dir, c};
    c->lq++;
    bvh_all(&s->lboxes, o, dir, &acc); /* intersect_lights (intersections.rs:87-91) */
    bvh_all(&s->lells, o, dir, &acc);
    bvh_all(&s->ltris, o, dir, &acc);
    double len = (double)(s->lells.n + s->lboxes.n + s->ltris.n);
    return acc.impact / len;
}

/* ======================================================================= */
/* RNG: Philox4x32-10 stream + rand 0.8.5 transforms                        */
/* ======================================================================= */
void oracle_philox4x32_10(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4]) {
    uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
    uint32_t k0 = key_in[0], k1 = key_in[1];
    for (int r = 0; r < 10; ++r) {
        if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}
typedef struct { uint32_t ctr[4]; uint32_t key[2]; uint32_t buf[4]; int idx; } Rng;
static void rng_init(Rng* r, uint64_t seed, uint64_t pixel, uint32_t sample) {
    r->ctr[0] = 0; r->ctr[1] = sample; r->ctr[2] = (uint32_t)pixel; r->ctr[3] = (uint32_t)(pixel >> 32);
    r->key[0] = (uint32_t)seed; r->key[1] = (uint32_t)(seed >> 32);
    r->idx = 4;
}
static inline uint32_t next_u32(Rng* r) {
    if (r->idx == 4) { oracle_philox4x32_10(r->ctr, r->key, r->buf); r->ctr[0]++; r->idx = 0; }
    return r->buf[r->idx++];
}
/* Start the next draw on a fresh 4-word block (the rest of the current one is
   skipped).  Called at every hit before shading draws anything, so each
   shading step consumes its words from a block boundary: lanes in the same
   branch then need new blocks at the same points on the device (coherent
   Philox refills).  Skipping words of a counter-based stream leaves the draws
   independent and uniform. */
static inline void rng_align(Rng* r) { r->idx = 4; }
static inline uint64_t next_u64(Rng* r) { /* BlockRng::next_u64: lo word then hi word */
    uint64_t lo = next_u32(r);
    uint64_t hi = next_u32(r);
    return lo | (hi << 32);
}
static inline double bits_f64(uint64_t b) { double x; memcpy(&x, &b, 8); return x; }
static inline uint64_t f64_bits(double x) { uint64_t b; memcpy(&b, &x, 8); return b; }
static inline double gen_f64(Rng* r) { /* Standard f64: (u64 >> 11) * 2^-53 */
    return (double)(next_u64(r) >> 11) * (1.0 / 9007199254740992.0);
}
static inline double value0_1(Rng* r) { /* (u64 >> 12).into_float_with_exponent(0) - 1.0 */
    return bits_f64((next_u64(r) >> 12) | 0x3FF0000000000000ull) - 1.0;
}
static double gen_range_f64(Rng* r, double low, double high) { /* UniformFloat::sample_single */
    double scale = high - low;
    for (;;) {
        double res = value0_1(r) * scale + low;
        if (res < high) return res;
    }
}
static double incl_scale(double low, double high) { /* UniformFloat::new_inclusive */
    const double max_rand = bits_f64(0x3FFFFFFFFFFFFFFFull) - 1.0; /* (u64::MAX>>12 | 1.0) - 1 */
    double scale = (high - low) / max_rand;
    while (scale * max_rand + low > high) scale = bits_f64(f64_bits(scale) - 1);
    return scale;
}
static double gen_range_incl_f64(Rng* r, double low, double high) {
    double scale = incl_scale(low, high);
    return value0_1(r) * scale + low;
}
/* UniformInt widening-multiply rejection (rand 0.8.5 uniform.rs sample_single_inclusive)
   with the EXACT acceptance zone MAX - (MAX - range + 1) % range, the form rand itself
   uses for u8/u16, instead of its conservative (range << lz) - 1 for wider types.
   Same uniform output distribution; for power-of-two ranges (1 light, the sign bit)
   it never rejects, so every lane consumes the same words (coherent device refills),
   where the conservative zone rejects half the draws. */
static uint64_t usize_zone(uint64_t range) { return UINT64_MAX - (0 - range) % range; }
static uint64_t gen_range_usize(Rng* r, uint64_t n) { /* UniformInt<usize>::sample_single(0, n) */
    uint64_t range = n; /* high-1 - low + 1 */
    if (range == 0) return next_u64(r);
    uint64_t zone = usize_zone(range);
    for (;;) {
        uint64_t v = next_u64(r);
        unsigned __int128 m = (unsigned __int128)v * range;
        uint64_t hi = (uint64_t)(m >> 64), lo = (uint64_t)m;
        if (lo <= zone) return hi;
    }
}
/* Bernoulli(0.5) from ONE word: P(w < 2^31) = 1/2 exactly, the distribution of
   gen_bool(0.5) (whose u64 draw this stream layout does not spend).  With one
   word for the Mix coin (and none for a single light's index), every diffuse
   sampler fits the two Philox blocks the device generates before it branches. */
static inline int gen_half(Rng* r) { return next_u32(r) < 0x80000000u; }
static int gen_bool(Rng* r, double p) { /* Bernoulli::new(p) + sample */
    if (p == 1.0) return 1; /* ALWAYS_TRUE: no draw */
    uint64_t p_int = (p >= 0.0 && p < 1.0) ? (uint64_t)(p * 18446744073709551616.0) : 0; /* NaN: reference panics */
    return next_u64(r) < p_int;
}

/* ======================================================================= */
/* ray_sampler.rs                                                           */
/* ======================================================================= */
/* The diffuse sampler's stream layout (Mix::sample :87-93): after the Mix coin both
   branches take the same three u64 draws A, B, C and differ only in how they map them
   (the device then draws them once per wave, render.hip "samplers").  Every
   distribution is the reference's:
     cosine (:69-76, uniform_on_sphere :159-170): gen_f64 of A, B, C;
     box light (uniform_on_box :142-157): choice = gen_range of A, sign = the lowest bit
       of A (value0_1 reads only A's top 52 bits, so the two are independent), u1 / u2
       = the inclusive [-1, 1] draws of B / C;
     ellipsoid light: uniform_on_sphere of A, B, C; triangle light: u, v of A, B;
     the light index (more than one light) is drawn after C. */
static inline double f64_of(uint64_t u) { return (double)(u >> 11) * (1.0 / 9007199254740992.0); }
static inline double unit_of(uint64_t u) { return bits_f64((u >> 12) | 0x3FF0000000000000ull) - 1.0; }
static V3 sphere_of(uint64_t A, uint64_t B, uint64_t C) { /* uniform_on_sphere :159-170 (a normalised cube point) */
    return vnormalize(v3(f64_of(A) * 2.0 - 1.0, f64_of(B) * 2.0 - 1.0, f64_of(C) * 2.0 - 1.0));
}
static V3 uniform_on_sphere(Rng* r) {
    uint64_t A = next_u64(r), B = next_u64(r), C = next_u64(r);
    return sphere_of(A, B, C);
}
static V3 cosine_of(V3 n, V3 v) { /* :69-76 with v = uniform_on_sphere */
    V3 d = vadd(v, n);
    const double eps = R_EPSILON * 16.0;
    if (fabs(d.x) <= eps && fabs(d.y) <= eps && fabs(d.z) <= eps) return n; /* abs_diff_eq(zero) */
    return vnormalize(d);
}
static V3 cosine_sample(V3 n, Rng* r) { return cosine_of(n, uniform_on_sphere(r)); } /* :69-76 */
static inline double cosine_pdf(V3 n, V3 d) { /* :78-83 */
    if (vdot(n, d) <= 0.0) return 0.0;
    return vdot(n, d) / R_PI;
}
static V3 uniform_on_box(V3 s, uint64_t A, uint64_t B, uint64_t C, Rng* r) { /* :142-157 */
    double w4x = s.y * s.z, w4y = s.x * s.z, w4z = s.x * s.y;
    double high = (w4x + w4y) + w4z, scale = high - 0.0, choice;
    for (;;) { /* gen_range_f64(r, 0.0, high) on A (never rejects: value0_1 * scale < scale) */
        choice = unit_of(A) * scale + 0.0;
        if (choice < high) break;
        A = next_u64(r);
    }
    double sign = (A & 1u) ? 1.0 : -1.0;
    double s11 = incl_scale(-1.0, 1.0);
    double u1 = unit_of(B) * s11 + -1.0; /* gen_range_incl_f64(-1.0, 1.0) */
    double u2 = unit_of(C) * s11 + -1.0;
    V3 p;
    if (choice < w4x) p = v3(sign, u1, u2);
    else if (choice < w4x + w4y) p = v3(u1, sign, u2);
    else p = v3(u1, u2, sign);
    return vmul(p, s);
}
static V3 light_sample(const oracle_scene* s, V3 pos, uint64_t A, uint64_t B, uint64_t C, Rng* r) { /* :101-130 */
    uint64_t len = s->lells.n + s->lboxes.n + s->ltris.n;
    /* gen_range(0..1) is 0 whatever it draws: no draw for a single light (a choice of
       this build's stream layout, like rng_align; the distribution is the same) */
    uint64_t index = len == 1 ? 0 : gen_range_usize(r, len);
    V3 world;
    if (index < s->lboxes.n) {
        const Shape* l = &s->lboxes.s[index];
        world = vadd(qrot(l->rot, uniform_on_box(l->shape, A, B, C, r)), l->pos);
    } else if (index < s->lboxes.n + s->lells.n) {
        const Shape* l = &s->lells.s[index - s->lboxes.n];
        world = vadd(qrot(l->rot, vmul(sphere_of(A, B, C), l->shape)), l->pos);
    } else {
        const Triangle* t = &s->ltris.t[index - s->lboxes.n - s->lells.n].tri;
        double s01 = incl_scale(0.0, 1.0);
        double u = unit_of(A) * s01 + 0.0; /* gen_range_incl_f64(0.0, 1.0) */
        double v = unit_of(B) * s01 + 0.0;
        if (u + v > 1.0) { u = 1.0 - u; v = 1.0 - v; }
        world = vadd(vadd(vscale(t->ba, u), vscale(t->ca, v)), t->a);
    }
    return vnormalize(vsub(world, pos));
}
static inline int lights_empty(const oracle_scene* s) { return s->lells.n == 0 && s->lboxes.n == 0 && s->ltris.n == 0; }

/* ---- literal draws (mode 2) -------------------------------------------- */
/* The reference's own sequence of rand 0.8.5 calls per diffuse bounce, on the
   same Philox word stream, with none of this build's layout choices (no block
   alignment at hits, no shared A/B/C draws, no exact UniformInt zone, an index
   draw even for one light).  Used only to pin, statistically, that the build's
   layout (modes 0/1, the device's) is the same estimator
   (tests/test_oracle.py::test_layout_matches_literal_draw_order). */
static int gen_bool_half_ref(Rng* r) { /* rng.gen_bool(0.5) (ray_sampler.rs:88): Bernoulli p_int = 2^63 */
    return next_u64(r) < 0x8000000000000000ull;
}
static uint64_t gen_range_usize_ref(Rng* r, uint64_t n) {
    /* rng.gen_range(0..n) (ray_sampler.rs:102): UniformInt<usize>::sample_single_inclusive(0, n-1)
       with rand's conservative zone (range << leading_zeros) - 1 for types wider than u16 */
    const uint64_t range = n, zone = (range << __builtin_clzll(range)) - 1;
    for (;;) {
        uint64_t v = next_u64(r);
        unsigned __int128 m = (unsigned __int128)v * range;
        if ((uint64_t)m <= zone) return (uint64_t)(m >> 64);
    }
}
static int32_t gen_range_i32_incl_ref(Rng* r, int32_t low, int32_t high) {
    /* rng.gen_range(0..=1) (ray_sampler.rs:147, an i32 literal): UniformInt<i32> draws u32
       words, conservative zone */
    const uint32_t range = (uint32_t)(high - low) + 1u, zone = (range << __builtin_clz(range)) - 1u;
    for (;;) {
        uint64_t m = (uint64_t)next_u32(r) * range;
        if ((uint32_t)m <= zone) return low + (int32_t)(uint32_t)(m >> 32);
    }
}
static V3 uniform_on_box_ref(V3 s, Rng* r) { /* ray_sampler.rs:142-157, call for call */
    double w4x = s.y * s.z, w4y = s.x * s.z, w4z = s.x * s.y;
    double choice = gen_range_f64(r, 0.0, (w4x + w4y) + w4z);
    double sign = (double)(gen_range_i32_incl_ref(r, 0, 1) * 2 - 1);
    double u1 = gen_range_incl_f64(r, -1.0, 1.0);
    double u2 = gen_range_incl_f64(r, -1.0, 1.0);
    V3 p;
    if (choice < w4x) p = v3(sign, u1, u2);
    else if (choice < w4x + w4y) p = v3(u1, sign, u2);
    else p = v3(u1, u2, sign);
    return vmul(p, s);
}
static V3 light_sample_ref(const oracle_scene* s, V3 pos, Rng* r) { /* ray_sampler.rs:101-130, call for call */
    uint64_t index = gen_range_usize_ref(r, s->lells.n + s->lboxes.n + s->ltris.n);
    V3 world;
    if (index < s->lboxes.n) {
        const Shape* l = &s->lboxes.s[index];
        world = vadd(qrot(l->rot, uniform_on_box_ref(l->shape, r)), l->pos);
    } else if (index < s->lboxes.n + s->lells.n) {
        const Shape* l = &s->lells.s[index - s->lboxes.n];
        world = vadd(qrot(l->rot, vmul(uniform_on_sphere(r), l->shape)), l->pos);
    } else {
        const Triangle* t = &s->ltris.t[index - s->lboxes.n - s->lells.n].tri;
        double u = gen_range_incl_f64(r, 0.0, 1.0);
        double v = gen_range_incl_f64(r, 0.0, 1.0);
        if (u + v > 1.0) { u = 1.0 - u; v = 1.0 - v; }
        world = vadd(vadd(vscale(t->ba, u), vscale(t->ca, v)), t->a);
    }
    return vnormalize(vsub(world, pos));
}

/* ======================================================================= */
/* raytrace.rs                                                              */
/* ======================================================================= */
static inline double powi2(double x) { return x * x; }                    /* powi(x, 2) */
static inline double powi5(double x) { double x2 = x * x; return x * (x2 * x2); } /* powi(x, 5) */

typedef struct {
    const oracle_scene* s; const rt_render_params* p; Rng* rng; Counters* c;
    int32_t* hits; /* [ray_depth] for this (pixel, sample) or NULL */
    int literal;   /* mode 2: the reference's own rand call sequence (see "literal draws") */
} Ctx;

static inline void reflected_ray(V3 o, V3 d, const Hit* h, V3* ro, V3* rd) { /* raytrace.rs:67-73 */
    V3 dir = vsub(d, vscale(vscale(h->ns, 2.0), vdot(h->ns, d)));
    *ro = vadd(vadd(o, vscale(d, h->t)), vscale(dir, R_EPSILON));
    *rd = dir;
}
static inline int refracted_ray(V3 o, V3 d, const Hit* h, double k, V3* ro, V3* rd) { /* raytrace.rs:75-88 */
    double cos1 = -vdot(h->ns, d);
    double sin2 = k * sqrt(1.0 - cos1 * cos1);
    if (sin2 > 1.0) return 0;
    double cos2 = sqrt(1.0 - sin2 * sin2);
    V3 dir = vadd(vscale(d, k), vscale(h->ns, k * cos1 - cos2));
    *ro = vadd(vadd(o, vscale(d, h->t)), vscale(dir, R_EPSILON));
    *rd = dir;
    return 1;
}
static inline double reflection_power(double n1, double n2, V3 d, const Hit* h) { /* raytrace.rs:62-65 */
    double r0 = powi2((n1 - n2) / (n1 + n2));
    return r0 + (1.0 - r0) * powi5(1.0 + vdot(d, h->ns));
}
static inline double clamp01(double x) { /* f64::clamp (NaN stays NaN) */
    if (x < 0.0) return 0.0;
    if (x > 1.0) return 1.0;
    return x;
}

/* Diffuse direction + pdf (raytrace.rs:17-30): returns 0 if the level ends
   with emission only (below the surface or pdf == 0). */
static int diffuse_sample(Ctx* x, V3 pos, V3 n, V3* dir_out, double* pdf_out) {
    const oracle_scene* s = x->s;
    V3 dir;
    int empty = lights_empty(s);
    if (empty) dir = cosine_sample(n, x->rng);
    else if (x->literal) /* Mix::sample :87-93 as written: coin, then the chosen sampler's own draws */
        dir = gen_bool_half_ref(x->rng) ? cosine_sample(n, x->rng) : light_sample_ref(s, pos, x->rng);
    else { /* Mix::sample :87-93, with the shared draws A, B, C (see uniform_on_box) */
        int coin = gen_half(x->rng);
        uint64_t A = next_u64(x->rng), B = next_u64(x->rng), C = next_u64(x->rng);
        dir = coin ? cosine_of(n, sphere_of(A, B, C)) : light_sample(s, pos, A, B, C, x->rng);
    }
    if (vdot(dir, n) <= 0.0) return 0;
    double pdf = empty ? cosine_pdf(n, dir)
                       : (cosine_pdf(n, dir) + light_pdf(s, pos, dir, x->c)) / 2.0; /* Mix::pdf :95-97 */
    if (pdf == 0.0) return 0;
    *dir_out = dir; *pdf_out = pdf;
    return 1;
}

static V3 raytrace_impl(Ctx* x, V3 o, V3 d, uint32_t left) { /* raytrace.rs:12-60 */
    if (left == 0) return v3(0, 0, 0);
    SceneHit sh;
    x->c->segments++;
    uint32_t bounce = x->p->ray_depth - left;
    int hit = scene_intersect(x->s, o, d, &sh, x->c);
    if (x->hits) x->hits[bounce] = hit ? (int32_t)sh.gid : RT_HIT_MISS;
    if (!hit) return vld(x->p->bg_color);
    if (!x->literal) rng_align(x->rng);
    const rt_material* m = &x->s->mats[sh.mat];
    const Hit* h = &sh.h;
    V3 e = vld(m->emission), col = vld(m->color);
    V3 rest;
    if (m->kind == RT_MAT_DIFFUSE) {
        V3 pos = vadd(o, vscale(d, h->t));
        V3 dir; double pdf;
        if (!diffuse_sample(x, pos, h->ns, &dir, &pdf)) rest = v3(0, 0, 0);
        else {
            V3 L = raytrace_impl(x, vadd(pos, vscale(dir, R_EPSILON)), dir, left - 1);
            rest = vdivs(vdivs(vscale(vmul(col, L), vdot(dir, h->ns)), R_PI), pdf);
        }
    } else if (m->kind == RT_MAT_DIELECTRIC) {
        double n1 = 1.0, n2 = m->ior;
        if (h->inside) { double t = n1; n1 = n2; n2 = t; }
        V3 fo, fd, ro, rd;
        reflected_ray(o, d, h, &fo, &fd);
        if (!refracted_ray(o, d, h, n1 / n2, &ro, &rd)) rest = raytrace_impl(x, fo, fd, left - 1);
        else {
            double power = reflection_power(n1, n2, d, h);
            if (gen_bool(x->rng, clamp01(power))) rest = raytrace_impl(x, fo, fd, left - 1);
            else {
                V3 L = raytrace_impl(x, ro, rd, left - 1);
                rest = h->inside ? L : vmul(L, col);
            }
        }
    } else {
        V3 fo, fd;
        reflected_ray(o, d, h, &fo, &fd);
        rest = vmul(raytrace_impl(x, fo, fd, left - 1), col);
    }
    return vadd(e, rest);
}

/* Iterative throughput form of the same estimator — the algorithm of the
   device kernel, operation for operation. */
static V3 raytrace_iter(Ctx* x, V3 o, V3 d) {
    V3 L = v3(0, 0, 0), T = v3(1.0, 1.0, 1.0);
    uint32_t depth = x->p->ray_depth;
    for (uint32_t b = 0; b < depth; ++b) {
        SceneHit sh;
        x->c->segments++;
        int hit = scene_intersect(x->s, o, d, &sh, x->c);
        if (x->hits) x->hits[b] = hit ? (int32_t)sh.gid : RT_HIT_MISS;
        if (!hit) { L = vadd(L, vmul(T, vld(x->p->bg_color))); break; }
        rng_align(x->rng);
        const rt_material* m = &x->s->mats[sh.mat];
        const Hit* h = &sh.h;
        V3 col = vld(m->color);
        L = vadd(L, vmul(T, vld(m->emission)));
        if (m->kind == RT_MAT_DIFFUSE) {
            V3 pos = vadd(o, vscale(d, h->t));
            V3 dir; double pdf;
            if (!diffuse_sample(x, pos, h->ns, &dir, &pdf)) break;
            /* col * cos / pi / pdf reassociated as col * (cosine_pdf / pdf), the device's
               one-division form (render.hip diffuse_weight): radiance only, so hit ids are
               unchanged and the recursive form above stays within rtol 1e-12 */
            double f = cosine_pdf(h->ns, dir) / pdf;
            V3 w = v3(col.x * f, col.y * f, col.z * f);
            T = vmul(T, w);
            /* The last bounce: the recursive form still evaluates dot * col (x) 0 / pi / pdf
               with raytrace_impl(.., 0) == 0 (raytrace.rs:13,32-33), which is NaN exactly
               when the direction or the pdf is NaN (e.g. a NaN light pdf: a query ray that
               starts inside a rotated light box by rounding, t^2/|d.n| = 0/0); the NaN then
               reaches the pixel through every enclosing level.  T is not read again here,
               so the rule is explicit. */
            if (b + 1 == depth && (isnan(vdot(dir, h->ns)) || isnan(pdf))) { L = v3(NAN, NAN, NAN); break; }
            o = vadd(pos, vscale(dir, R_EPSILON));
            d = dir;
        } else if (m->kind == RT_MAT_DIELECTRIC) {
            double n1 = 1.0, n2 = m->ior;
            if (h->inside) { double t = n1; n1 = n2; n2 = t; }
            V3 fo, fd, ro, rd;
            reflected_ray(o, d, h, &fo, &fd);
            if (!refracted_ray(o, d, h, n1 / n2, &ro, &rd)) { o = fo; d = fd; }
            else {
                double power = reflection_power(n1, n2, d, h);
                if (gen_bool(x->rng, clamp01(power))) { o = fo; d = fd; }
                else {
                    if (!h->inside) T = vmul(T, col);
                    o = ro; d = rd;
                }
            }
        } else {
            V3 fo, fd;
            reflected_ray(o, d, h, &fo, &fd);
            T = vmul(T, col);
            o = fo; d = fd;
        }
    }
    return L;
}

/* ======================================================================= */
/* camera.rs + main.rs:85-114                                               */
/* ======================================================================= */
typedef struct { V3 pos, right, up, fwd; double tx, ty, w, h; } Camera;
static Camera camera_new(const rt_render_params* p) { /* camera.rs:17-46 */
    Camera c;
    double fw = (double)p->width, fh = (double)p->height;
    if (p->fov_axis == RT_FOV_Y) {
        c.ty = tan(p->fov / 2.0);
        double aspect = fh / fw;
        c.tx = c.ty / aspect;
    } else {
        c.tx = tan(p->fov / 2.0);
        double aspect = fw / fh;
        c.ty = c.tx / aspect;
    }
    c.pos = vld(p->cam_position); c.right = vld(p->cam_right); c.up = vld(p->cam_up); c.fwd = vld(p->cam_forward);
    c.w = fw; c.h = fh;
    return c;
}
static void fuzzy_ray(const Camera* c, uint32_t x, uint32_t y, Rng* r, V3* o, V3* d) { /* camera.rs:48-55 */
    double px = (double)x + gen_range_f64(r, 0.0, 1.0);
    double py = (double)y + gen_range_f64(r, 0.0, 1.0);
    double xx = (2.0 * px / c->w - 1.0) * c->tx;
    double yy = -(2.0 * py / c->h - 1.0) * c->ty;
    *d = vadd(vadd(vscale(c->right, xx), vscale(c->up, yy)), vscale(c->fwd, 1.0));
    *o = c->pos;
}

int oracle_render(const oracle_scene* s, const rt_render_params* p, int mode, int threads,
                  uint32_t row_begin, uint32_t row_end,
                  double* out, int32_t* hit_ids, rt_stats* stats) {
    return oracle_render_chunked(s, p, mode, threads, row_begin, row_end, 0, out, hit_ids, stats);
}

static int render_impl(const oracle_scene* s, const rt_render_params* p, int mode, int threads,
                       uint32_t row_begin, uint32_t row_end, uint32_t chunk_spp,
                       double* out, double* out_sq, int32_t* hit_ids, rt_stats* stats) {
    if (!s || !p || !out || p->width == 0 || p->height == 0 || mode < 0 || mode > 2) return RT_ERR_INVALID;
    if (chunk_spp == 0 || chunk_spp > p->spp) chunk_spp = p->spp;
    if (row_end > p->height) row_end = p->height;
    if (row_begin >= row_end) return RT_ERR_INVALID;
    Camera cam = camera_new(p);
    const uint64_t W = p->width;
    const uint64_t first = (uint64_t)row_begin * W, last = (uint64_t)row_end * W;
    const uint32_t spp = p->spp, depth = p->ray_depth;
    int nthreads = 1;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
    nthreads = omp_get_max_threads();
#endif
    Counters* tc = (Counters*)calloc((size_t)nthreads, sizeof(Counters));
#pragma omp parallel for schedule(dynamic, 64)
    for (uint64_t idx = first; idx < last; ++idx) { /* main.rs:94-111 */
        int tid = 0;
#ifdef _OPENMP
        tid = omp_get_thread_num();
#endif
        Counters* c = &tc[tid];
        uint32_t x = (uint32_t)(idx % W), y = (uint32_t)(idx / W);
        V3 sum = v3(0, 0, 0), run = v3(0, 0, 0), sq = v3(0, 0, 0);
        for (uint32_t smp = 0; smp < spp; ++smp) {
            Rng rng;
            rng_init(&rng, p->seed, idx, smp);
            int32_t* hrow = hit_ids ? hit_ids + (idx * spp + smp) * depth : NULL;
            if (hrow) for (uint32_t b = 0; b < depth; ++b) hrow[b] = RT_HIT_NONE;
            Ctx cx = {s, p, &rng, c, hrow, mode == 2};
            V3 o, d;
            fuzzy_ray(&cam, x, y, &rng, &o, &d);
            d = vnormalize(d); /* raytrace.rs:9 */
            c->paths++;
            V3 L = mode == 1 ? raytrace_iter(&cx, o, d) : raytrace_impl(&cx, o, d, depth);
            run = vadd(run, L);
            if (out_sq) sq = vadd(sq, vmul(L, L));
            if ((smp + 1) % chunk_spp == 0 || smp + 1 == spp) { /* end of a run (one run = main.rs's sum) */
                sum = smp < chunk_spp ? run : vadd(sum, run);
                run = v3(0, 0, 0);
            }
        }
        vst(out + 3 * idx, vdivs(sum, (double)spp)); /* main.rs:104 before tonemapping */
        if (out_sq) vst(out_sq + 3 * idx, vdivs(sq, (double)spp));
    }
    if (stats) {
        memset(stats, 0, sizeof(*stats));
        for (int t = 0; t < nthreads; ++t) {
            stats->paths += tc[t].paths; stats->segments += tc[t].segments;
            stats->aabb_tests += tc[t].aabb; stats->tri_tests += tc[t].tri;
            stats->shape_tests += tc[t].shape; stats->shaded_hits += tc[t].shaded;
            stats->light_queries += tc[t].lq; stats->light_hits += tc[t].lhits;
        }
    }
    free(tc);
    return 0;
}

int oracle_render_chunked(const oracle_scene* s, const rt_render_params* p, int mode, int threads,
                          uint32_t row_begin, uint32_t row_end, uint32_t chunk_spp,
                          double* out, int32_t* hit_ids, rt_stats* stats) {
    return render_impl(s, p, mode, threads, row_begin, row_end, chunk_spp, out, NULL, hit_ids, stats);
}

int oracle_render_moments(const oracle_scene* s, const rt_render_params* p, int mode, int threads,
                          uint32_t row_begin, uint32_t row_end, double* out_mean, double* out_sq, rt_stats* stats) {
    if (!out_sq) return RT_ERR_INVALID;
    return render_impl(s, p, mode, threads, row_begin, row_end, 0, out_mean, out_sq, NULL, stats);
}

void oracle_intersect_rays(const oracle_scene* s, const double* rays, uint32_t n, rt_hit* out) {
    Counters c = {0};
    for (uint32_t i = 0; i < n; ++i) {
        SceneHit sh;
        V3 o = vld(rays + 6 * i), d = vld(rays + 6 * i + 3);
        memset(&out[i], 0, sizeof(rt_hit));
        if (scene_intersect(s, o, d, &sh, &c)) {
            out[i].t = sh.h.t; vst(out[i].geometry_normal, sh.h.ng); vst(out[i].shading_normal, sh.h.ns);
            out[i].inside = sh.h.inside; out[i].prim = (int32_t)sh.gid;
        } else out[i].prim = RT_HIT_MISS;
    }
}
void oracle_light_pdf_rays(const oracle_scene* s, const double* pd, uint32_t n, double* out) {
    Counters c = {0};
    for (uint32_t i = 0; i < n; ++i) out[i] = lights_empty(s) ? 0.0 : light_pdf(s, vld(pd + 6 * i), vld(pd + 6 * i + 3), &c);
}

/* ======================================================================= */
/* KAT hooks                                                                */
/* ======================================================================= */
int oracle_aabb_intersects(const double mn[3], const double mx[3], const double o[3], const double d[3], double* t) {
    AABB a = {vld(mn), vld(mx)};
    return aabb_intersects(&a, vld(o), vld(d), t);
}
int oracle_box_intersection(const double sz[3], const double o[3], const double d[3], double* t, double n[3], int* inside) {
    Hit h;
    if (!box_hit(vld(sz), vld(o), vld(d), &h)) return 0;
    *t = h.t; vst(n, h.ng); *inside = h.inside;
    return 1;
}
int oracle_ellipsoid_intersection(const double r[3], const double o[3], const double d[3], double* t, double n[3], int* inside) {
    Hit h;
    if (!ell_hit(vld(r), vld(o), vld(d), &h)) return 0;
    *t = h.t; vst(n, h.ng); *inside = h.inside;
    return 1;
}
int oracle_plane_intersection(const double nrm[3], const double o[3], const double d[3], double* t, double n[3]) {
    Hit h;
    if (!plane_hit(vld(nrm), vld(o), vld(d), &h)) return 0;
    *t = h.t; vst(n, h.ng);
    return 1;
}
int oracle_triangle_intersection(const double abc[9], const double pos[3], const double rot[4],
                                 const double o[3], const double d[3],
                                 double* t, double ng[3], double ns[3], int* inside) {
    Triangle m = tri_new_geom(vld(abc), vld(abc + 3), vld(abc + 6));
    V3 p = pos ? vld(pos) : v3(0, 0, 0);
    Q q = rot ? qld(rot) : (Q){1.0, {0, 0, 0}};
    V3 a = vadd(qrot(q, m.a), p), b = vadd(qrot(q, vadd(m.ba, m.a)), p), c = vadd(qrot(q, vadd(m.ca, m.a)), p);
    Triangle w = tri_new_smooth(a, b, c, qrot(q, m.na), qrot(q, m.nb), qrot(q, m.nc));
    Hit h;
    if (!tri_hit(&w, vld(o), vld(d), &h)) return 0;
    *t = h.t; vst(ng, h.ng); vst(ns, h.ns); *inside = h.inside;
    return 1;
}
void oracle_cof3(const double m[9], double out[9]) { /* gltf/scene_builder.rs:367-388, m[c*3+r] */
    static const int other[3][2] = {{1, 2}, {0, 2}, {0, 1}};
    for (int col = 0; col < 3; ++col)
        for (int row = 0; row < 3; ++row) {
            int lc = other[col][0], rc = other[col][1], tr = other[row][0], br = other[row][1];
            /* Mat2::new(c0r0, c0r1, c1r0, c1r1).determinant() = c0r0*c1r1 - c1r0*c0r1 */
            double a = m[lc * 3 + tr], b = m[lc * 3 + br], c = m[rc * 3 + tr], d = m[rc * 3 + br];
            double det = a * d - c * b;
            out[col * 3 + row] = ((col + row) & 1) ? -det : det;
        }
}
void oracle_rng_stream_u64(uint64_t seed, uint64_t pixel, uint32_t sample, uint32_t n, uint64_t* out) {
    Rng r; rng_init(&r, seed, pixel, sample);
    for (uint32_t i = 0; i < n; ++i) out[i] = next_u64(&r);
}
void oracle_sampler_draws(uint64_t seed, uint64_t pixel, uint32_t sample, int kind,
                          const double arg[3], uint32_t n, double* out) {
    Rng r; rng_init(&r, seed, pixel, sample);
    for (uint32_t i = 0; i < n; ++i) {
        V3 v = v3(0, 0, 0);
        switch (kind) {
        case 0: v = cosine_sample(vld(arg), &r); break;
        case 1: { uint64_t A = next_u64(&r), B = next_u64(&r), C = next_u64(&r);
                  v = uniform_on_box(vld(arg), A, B, C, &r); } break;
        case 2: v = uniform_on_sphere(&r); break;
        case 3: v.x = (double)gen_range_usize(&r, (uint64_t)arg[0]); break;
        case 4: v.x = (double)gen_bool(&r, arg[0]); break;
        case 5: v.x = gen_range_incl_f64(&r, arg[0], arg[1]); break;
        case 6: v.x = gen_range_f64(&r, arg[0], arg[1]); break;
        case 7: v.x = (double)gen_half(&r); break;
        default: break;
        }
        vst(out + 3 * i, v);
    }
}

/* ======================================================================= */
/* postprocessing.rs, ppm.rs                                                */
/* ======================================================================= */
static double aces1(double x) { /* postprocessing.rs:9-28 */
    const double a = 2.51, b = 0.03, c = 2.43, d = 0.59, e = 0.14;
    double num = (a * x + b) * x;
    double den = (c * x + d) * x + e;
    double v = num / den;
    if (v < 0.0) v = 0.0; /* num_traits::clamp */
    if (v > 1.0) v = 1.0;
    return v;
}
void oracle_tonemap_gamma(const double* in, uint64_t n, double* out) {
    for (uint64_t i = 0; i < 3 * n; ++i) out[i] = pow(aces1(in[i]), 1.0 / 2.2); /* :5-7 */
}
void oracle_ppm_bytes(const double* rgb, uint64_t n, uint8_t* out) { /* ppm.rs:13-15 */
    for (uint64_t i = 0; i < 3 * n; ++i) {
        double v = rgb[i];
        if (v < 0.0) v = 0.0;
        if (v > 1.0) v = 1.0; /* f64::clamp */
        double r = round(v * 255.0);
        out[i] = (uint8_t)(r != r ? 0 : r); /* `as u8` saturates, NaN -> 0 */
    }
}

/* ======================================================================= */
/* extra hooks: raw BVH build, raw intersect_lights                         */
/* ======================================================================= */
uint64_t oracle_bvh_build(const double* boxes, uint64_t n, int64_t* links, double* bounds, uint64_t* order,
                          uint32_t* depth) {
    AABB* bx = (AABB*)malloc(sizeof(AABB) * (n ? n : 1));
    for (uint64_t i = 0; i < n; ++i) { bx[i].min = vld(boxes + 6 * i); bx[i].max = vld(boxes + 6 * i + 3); }
    uint64_t* perm = (uint64_t*)malloc(sizeof(uint64_t) * (n ? n : 1));
    BVH b;
    bvh_build(&b, bx, n, perm);
    if (links) {
        for (uint64_t i = 0; i < b.n_nodes; ++i) {
            const Node* nd = &b.nodes[i];
            links[4 * i + 0] = nd->left; links[4 * i + 1] = nd->right;
            links[4 * i + 2] = (int64_t)nd->start; links[4 * i + 3] = (int64_t)nd->end;
            if (bounds) { vst(bounds + 6 * i, nd->aabb.min); vst(bounds + 6 * i + 3, nd->aabb.max); }
        }
        if (order) for (uint64_t i = 0; i < n; ++i) order[i] = perm[i];
    }
    if (depth) *depth = b.depth;
    uint64_t nn = b.n_nodes;
    free(b.nodes); free(bx); free(perm);
    return nn;
}
void oracle_intersect_lights_rays(const oracle_scene* s, const double* rays, uint32_t n, double* impact,
                                  uint32_t* count) {
    for (uint32_t i = 0; i < n; ++i) {
        Counters c = {0};
        PdfAcc acc = {0.0, vld(rays + 6 * i + 3), &c};
        V3 o = vld(rays + 6 * i), d = vld(rays + 6 * i + 3);
        bvh_all(&s->lboxes, o, d, &acc); /* intersections.rs:87-91 */
        bvh_all(&s->lells, o, d, &acc);
        bvh_all(&s->ltris, o, d, &acc);
        impact[i] = acc.impact;
        if (count) count[i] = (uint32_t)c.lhits;
    }
}
