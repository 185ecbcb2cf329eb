// render.hip — MI355X (gfx950) kernels of the path-tracing hot path.
//
//   path_kernel          generate_image pixel loop (main.rs:94-103) fused with
//                        Camera::fuzzy_ray (camera.rs:48-55) and raytrace /
//                        raytrace_impl (raytrace.rs:8-60) in throughput form.
//                        Persistent 64-lane waves pull (tile, sample chunk,
//                        quadrant) wave-tiles from a queue; inside one, lanes
//                        take (sample, pixel) paths dynamically and commit
//                        radiance per pixel in sample order.
//   reduce_chunks_kernel chunk partial sums -> per-pixel mean
//   intersect_kernel     batch `intersect` (intersections.rs:42-62), one thread per ray
//   trace_kernel         the same, persistent: waves refill finished lanes from a queue
//   light_kernel         batch intersect_lights / Light::pdf
//                        (intersections.rs:87-91, ray_sampler.rs:132-139)
//   unpack_kernel        gathered tiles -> row-major image
//
// BVH traversal keeps the reference's exact visit order (bvh.rs:151-210): the
// far child goes on a per-lane stack (short part in LDS, overflow in a global
// spill area sized from the deepest BVH) with its clamped entry t, and is
// re-checked against the updated best when popped — identical to the
// recursive "visit near, then far if still < best".
#include <hip/hip_runtime.h>

#include <algorithm>

#include "render.h"
#include "rt_device.h"

namespace rt {

constexpr int kBlock = 256;
constexpr int kShort = kMaxBvhDepthShort;
constexpr int kLeafBatch = 16;  // lanes waiting at leaves before the wave tests primitives (bvh_closest)

// ---------------------------------------------------------------- stack ---
// LDS short stack laid out per wave: [wave][slot][lane], so consecutive lanes
// hit consecutive banks for any block size.
constexpr int kWave = 64;

// The pointers are this wave's bases (wave-uniform, so they live in SGPRs);
// each access adds the lane index, recomputed through an opaque mbcnt so the
// compiler cannot hoist it into a long-lived VGPR (which it then spilled to
// scratch and reloaded on every push and pop of the 4-wave path kernel).
RT_D uint32_t stack_lane() {
    uint32_t m = ~0u;
    asm volatile("" : "+s"(m));
    return __builtin_amdgcn_mbcnt_hi(m, __builtin_amdgcn_mbcnt_lo(m, 0u));
}
// OPQ = false keeps the lane index in a register (the 3-wave fused kernel,
// which has room: C2 113.8 vs 115.1 ms with OPQ); OPQ = true recomputes it.
template <bool OPQ, int KS = kShort>  // KS: LDS entries per lane
struct Stack {
    uint32_t* sn;        // LDS node slots of this wave, [slot][lane]
    double* st;          // LDS entry-t slots of this wave, [slot][lane]
    uint32_t* gn;        // global spill of this wave ([slot][stride], lane-indexed) or null
    double* gt;
    uint32_t stride;
    uint32_t ln;         // lane index (OPQ = false)
    int sp;
    RT_D uint32_t lane() const { return OPQ ? stack_lane() : ln; }
    RT_D void push(uint32_t node, double t) {
        const uint32_t l = lane();
        PH_LANE(kPhPushLane);
        if (sp < KS) { sn[sp * kWave + l] = node; st[sp * kWave + l] = t; }
        else {
            PH_LANE(kPhPushGlobal);
            gn[(size_t)(sp - KS) * stride + l] = node; gt[(size_t)(sp - KS) * stride + l] = t;
        }
        ++sp;
    }
    // The spill side reads through volatile pointers: otherwise the compiler
    // merges the two branches into one select-of-pointers + flat load, which
    // puts every pop (LDS in > 99% of cases) on the flat path.
    RT_D void pop(uint32_t& node, double& t) {
        --sp;
        const uint32_t l = lane();
        if (sp < KS) { node = sn[sp * kWave + l]; t = st[sp * kWave + l]; }
        else {
            PH_LANE(kPhPopGlobal);
            node = ((volatile const uint32_t*)gn)[(size_t)(sp - KS) * stride + l];
            t = ((volatile const double*)gt)[(size_t)(sp - KS) * stride + l];
        }
    }
};
// wave_tid = the wave's first thread in the block, wave_gtid = its first
// thread in the grid (both wave-uniform)
template <bool OPQ = false, int KS = kShort>
RT_D Stack<OPQ, KS> make_stack(uint32_t* s_n, double* s_t, uint32_t wave_tid, uint64_t wave_gtid, uint32_t* spill_n,
                               double* spill_t, uint32_t spill_stride) {
    Stack<OPQ, KS> k;
    k.ln = __lane_id();
    const uint32_t base = (wave_tid / kWave) * KS * kWave;
    k.sn = s_n + base; k.st = s_t + base;
    k.gn = spill_n ? spill_n + wave_gtid : nullptr;
    k.gt = spill_t ? spill_t + wave_gtid : nullptr;
    k.stride = spill_stride;
    k.sp = 0;
    return k;
}

// A scene's primitive kinds (host: api.cpp path_kinds): kernel instances for
// one-kind scenes carry no code or state for the other kind.
constexpr int kShapes = 1, kTris = 2;

// Best candidate of one query: materialised into a Hit only for the winner.
struct Cand {
    double t;
    double u, v;       // triangle barycentrics
    uint32_t prim;     // index in its list / BVH order
    uint32_t aux;      // shape face / plane side bits
    uint32_t kind;     // 0 plane, 1 box, 2 ellipsoid, 3 triangle
    bool valid;
};

// Plane::intersection for a kPlaneAxis plane (n = sign * e_K) and a ray_fast
// ray, when o[K] - pos[K] != 0: then model_ray's mo[K] and md[K] are o[K] -
// pos[K] and d[K] bit for bit (finite operands, identity rotation), n.mo =
// sign * x and n.d = sign * d[K] exactly (the zero terms add signed zeros to a
// nonzero value), so t = -(sign x) / (sign d[K]) = -RN(x / d[K]) — by
// dev_quot, exact for x in [2^-449, 2^401] (shape_fast).  Returns -1 when the
// lane must take the generic form (x == 0), else hit (1) / miss (0).
template <int K>
RT_D int plane_axis_t(const DevShape& s, V3 o, V3 d, const Rcp3& rc, double& t, uint32_t& aux) {
    const double x = comp(o, K) - s.pos[K];
    if (x == 0.0) return -1;
    const double dk = comp(d, K);
    const double tt = -dev_quot(x, dk, comp(rc.r, K));
    if (tt < 0.0) return 0;
    t = tt;
    aux = ((s.axis & 4u) ? -dk : dk) <= 0.0 ? 1u : 0u;
    return 1;
}

// box_coef on a generic model-space ray (model_ray; `same`: md == d, whose
// reciprocals rc may serve).  For a kBoxSizes box the dividends +-s - mo are 0
// or in dev_quot's range whenever |mo| <= 2^400 (s and mo are then both 0 or
// at least 2^-420 apart from tiny cases that leave s - mo near s), so when md
// also has every component dir_ok in every lane running this, the wave takes
// the split division (box_coef<true>, with md's own dev_rcp reciprocals): the
// same bits as the quotients of the plain form.
RT_D int box_model(const DevShape& s, V3 mo, V3 md, bool same, const Rcp3& rc, Bpi& en, Bpi& ex) {
#ifndef RT_NO_FASTSHAPE
    if (s.flags & kBoxSizes) {
        const bool ok = dir_ok(md.x) && dir_ok(md.y) && dir_ok(md.z) && fabs(mo.x) <= 0x1p400 &&
                        fabs(mo.y) <= 0x1p400 && fabs(mo.z) <= 0x1p400;
        if (__ballot(!ok) == 0) return box_coef<true>(load3(s.shape), mo, md, same ? rc : make_rcp3(md), en, ex);
    }
#endif
    return box_coef(load3(s.shape), mo, md, rc, en, ex);
}

// closest hit of one shape in model space; t + aux.  rfast: the ray passed
// ray_fast (kShapeFast shapes may then take the exact unguarded division).
template <int KIND>
RT_D bool shape_closest(const DevShape& s, V3 o, V3 d, const Rcp3& rc, bool rfast, double& t, uint32_t& aux) {
    V3 mo, md;
#ifndef RT_NO_FASTSHAPE  // ablation build: the generic form for every shape
    if (KIND == 0 && rfast && (s.flags & (kShapeFast | kPlaneAxis)) == (kShapeFast | kPlaneAxis)) {
        const uint32_t k = s.axis & 3u;  // uniform: one scalar branch
        const int r = k == 0 ? plane_axis_t<0>(s, o, d, rc, t, aux)
                    : (k == 1 ? plane_axis_t<1>(s, o, d, rc, t, aux) : plane_axis_t<2>(s, o, d, rc, t, aux));
        if (r >= 0) return r != 0;
    }
    if (KIND != 0 && shape_fast(s, rfast, o, mo)) {
        if (KIND == 1) {
            Bpi en, ex;
            int k = box_coef<true>(load3(s.shape), mo, d, rc, en, ex);
            if (k == 2) { t = en.t; aux = bpi_aux(en, false); return true; }
            if (k == 1) { t = ex.t; aux = bpi_aux(ex, true); return true; }
            return false;
        }
        double t1, t2;
        int k = ell_coef<true>(load_radii(s), mo, d, t1, t2);
        if (k == 2) { t = t1; aux = 0; return true; }
        if (k == 1) { t = t2; aux = 8; return true; }
        return false;
    }
#endif
    const bool same = model_ray(s, o, d, mo, md);
    if (KIND == 0) return plane_t(load3(s.shape), mo, md, t, aux);
    if (KIND == 1) {
        Bpi en, ex;
        int k = box_model(s, mo, md, same, rc, en, ex);
        if (k == 2) { t = en.t; aux = bpi_aux(en, false); return true; }
        if (k == 1) { t = ex.t; aux = bpi_aux(ex, true); return true; }
        return false;
    }
    double t1, t2;
    int k = ell_coef(load_radii(s), mo, md, t1, t2);
    if (k == 2) { t = t1; aux = 0; return true; }
    if (k == 1) { t = t2; aux = 8; return true; }
    return false;
}

// BVH::intersection (bvh.rs:27-36) + Node::intersection (bvh.rs:151-186) as
// a resumable per-lane state: the path kernel suspends a lane's triangle
// traversal when few lanes of its wave are still traversing,
// lets the finished lanes shade and start their next segments, and resumes.
// Each lane's own sequence of visits, tests, `best` updates and pruning is the
// reference's (bvh.rs:151-210) whatever the suspension points.
struct Trav {
    double best, bu, bv;           // closest candidate so far (best = +inf when none)
    uint32_t prim, aux;
    uint32_t node, cnt, start;     // current node; its primitive range (cnt 0 = internal)
    bool valid, live;
};

// slab test of one box: SLAB 0 = guarded form, 1 = unguarded exact division
// (DevBvh::fast boxes and a ray_fast ray), 2 = per lane (`fast`)
template <int SLAB>
RT_D bool slab(const double* mn, const double* mx, V3 o, V3 d, const Rcp3& rc, bool fast, double& t) {
    if (SLAB == 1 || (SLAB == 2 && fast)) return aabb_hit<true>(load3(mn), load3(mx), o, d, rc, t);
    return aabb_hit<false>(load3(mn), load3(mx), o, d, rc, t);
}
// Both children's boxes of an inner node (bvh.rs:158-159) in one batch of 16-B
// loads.  The asm pins the right box's registers before the left slab test is
// computed, so the compiler cannot sink the right box's loads behind that test:
// one memory round trip per node visit instead of two (C3 -3.3%, C5 -6.3% at
// reduced spp, profiles/r02/variants/variants_preload_*.log).
struct NodeBoxes { V3 lmn, lmx, rmn, rmx; };
RT_D NodeBoxes node_boxes(const DevNode& n) {
    const double2* nw = (const double2*)&n;
    const double2 w0 = nw[0], w1 = nw[1], w2 = nw[2], w3 = nw[3], w4 = nw[4], w5 = nw[5];
    asm volatile("" ::"v"(w3.x), "v"(w3.y), "v"(w4.x), "v"(w4.y), "v"(w5.x), "v"(w5.y));
    return NodeBoxes{v3(w0.x, w0.y, w1.x), v3(w1.y, w2.x, w2.y), v3(w3.x, w3.y, w4.x), v3(w4.y, w5.x, w5.y)};
}
template <int SLAB>
RT_D bool slab_c(float lx, float ly, float lz, float hx, float hy, float hz, V3 o, V3 d, const Rcp3& rc, bool fast,
                 double& t) {
    if (SLAB == 1 || (SLAB == 2 && fast)) return aabb_hit<true>(v3(lx, ly, lz), v3(hx, hy, hz), o, d, rc, t);
    return aabb_hit<false>(v3(lx, ly, lz), v3(hx, hy, hz), o, d, rc, t);
}
template <int SLAB>
RT_D bool slab_v(V3 mn, V3 mx, V3 o, V3 d, const Rcp3& rc, bool fast, double& t) {  // boxes already loaded
    if (SLAB == 1 || (SLAB == 2 && fast)) return aabb_hit<true>(mn, mx, o, d, rc, t);
    return aabb_hit<false>(mn, mx, o, d, rc, t);
}

template <int SLAB, bool ST, class Stk>
RT_D void trav_init(const DevBvh& B, V3 o, V3 d, const Rcp3& rc, bool fast, Stk& S, Cnt<ST>& C, Trav& T) {
    T.valid = false; T.live = false;
    T.best = INFINITY; T.bu = T.bv = 0.0; T.prim = 0; T.aux = 0;
    T.node = 0; T.cnt = 0; T.start = 0;
    S.sp = 0;
    if (B.n_prims == 0) return;
    double t0;
    C.aabb();
    if (!slab<SLAB>(B.root_min, B.root_max, o, d, rc, fast, t0)) return;
    T.cnt = B.nodes[0].count; T.start = B.nodes[0].start;
    T.live = true;
}

// One wave-level step for the live lanes (lv = their ballot).  Deferred
// leaves: a lane that reaches a leaf waits there while the other lanes keep
// stepping through internal nodes; the wave tests leaf primitives once
// >= kLeafBatch lanes wait (or every live lane does), so the primitive loop
// runs with many lanes instead of a few.
// A child / stack word (child_word) -> the lane's current node: a packed leaf's
// range, a big leaf's range from its node (f64 or compact layout), or an
// internal node.
template <bool CMP>
RT_D void trav_enter(const DevBvh& B, Trav& T, uint32_t w) {
    if (w & kPackedLeaf) { T.cnt = (w >> 24) & 127u; T.start = w & 0xFFFFFFu; }
    else if (w & kLeafRef) {
        T.node = w & ~kLeafRef;
        if (CMP) { T.cnt = B.cnodes[T.node].count; T.start = B.cnodes[T.node].start; }
        else { T.cnt = B.nodes[T.node].count; T.start = B.nodes[T.node].start; }
    } else { T.node = w; T.cnt = 0; }
}

// A compact triangle record (rt_layout.h kTriC: a, b, c as f32) in registers:
// ba = b - a and ca = c - a rebuilt in f64, the host's bits (triangle_props).
struct F3 { float x, y, z; };
RT_D F3 ld3(const float* p) { return *(const F3*)p; }
RT_D TriRec load_tri_c(const float* __restrict__ p) {
    const F3 a = ld3(p), b = ld3(p + 3), c = ld3(p + 6);
    asm volatile("" ::"v"(a.x), "v"(a.y), "v"(a.z), "v"(c.x), "v"(c.y), "v"(c.z));
    const V3 A = v3(a.x, a.y, a.z);
    return TriRec{A, v3(b.x, b.y, b.z) - A, v3(c.x, c.y, c.z) - A};
}

#ifndef RT_LEAF_SERIAL  // ablation build: every leaf by the serial loop of trav_step
// Cooperative leaf step (round 6): the records of the waiting lanes' small leaves
// (<= kCoopMax records, every leaf the reference's builder makes below its
// SameNode case, bvh.rs:77) are dealt to consecutive lanes, one record per lane,
// in rounds of <= 64 records; each leaf's lane then folds its records' results in
// record order with the reference's update rule (bvh.rs:213-222).  A record's
// test is a pure function of the ray and the record, so every lane's sequence of
// `best` updates is the serial loop's.  The serial loop runs max(count) trips with
// the waiting lanes still in them (leaf-loop lane use 0.39 on C5); a round runs
// once per 64 records.  With the leaf batch re-tuned for it (render.h): C5 -7.7%,
// C3 -2% at reduced spp, same images and counters (profiles/r06/variants_coop*); full
// frames C3 702.3 -> 677.0 ms, C5 182.8 -> 170.7 ms (profiles/r06/bench_c*_aj.log).
// Reached only from the 64-thread (one-wave) kernels: s_own is per block.
constexpr uint32_t kCoopMax = 4;
RT_D uint32_t lanes_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
template <bool ST>
RT_D void leaf_coop(const DevBvh& B, V3 o, V3 d, Cnt<ST>& C, Trav& T) {
    __shared__ uint8_t s_own[2 * kWave];  // record slot -> the lane whose leaf it is; [64, 128) scratch
    bool mine = T.live && T.cnt != 0 && T.cnt <= kCoopMax;
    uint64_t todo = __ballot(mine);
    while (todo) {
        const uint32_t lane = stack_lane();
        const uint32_t c = mine ? T.cnt : 0u;
        // exclusive prefix of the record counts (c < 8: three bit planes)
        const uint32_t p = lanes_below(__ballot(c & 1u)) + 2u * lanes_below(__ballot(c & 2u)) +
                           4u * lanes_below(__ballot(c & 4u));
        const bool take = mine && p + c <= (uint32_t)kWave;  // a prefix of the waiting lanes
        const uint64_t tk = __ballot(take);
        const uint32_t total = __builtin_amdgcn_readlane(p + c, 63 - __clzll(tk));
        // every lane writes kCoopMax bytes, the ones past its leaf into its own scratch
        // byte: no exec-mask branches (with them, and the fold below as branches, C3 +1.1%
        // and C5 +0.9%: profiles/r06/variants_coopbf_C*.log)
#pragma unroll
        for (uint32_t k = 0; k < kCoopMax; ++k) s_own[(take & (k < c)) ? p + k : kWave + lane] = (uint8_t)lane;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        const bool item = lane < total;
        const uint32_t own = item ? s_own[lane] : lane;
        const uint32_t first = take ? *(const uint32_t*)(B.ctris + (size_t)T.start * kLeafBlock) : 0u;
        const uint32_t po = __shfl(p, own), st = __shfl(T.start, own);
        const V3 oo = v3(__shfl(o.x, own), __shfl(o.y, own), __shfl(o.z, own));
        const V3 od = v3(__shfl(d.x, own), __shfl(d.y, own), __shfl(d.z, own));
        double tt = -1.0, uu = 0.0, vv = 0.0;  // -1: no hit (a hit's t is >= -0 or NaN)
        if (item) {
            PH_COUNT(kPhLeafWave, kPhLeafLane);
            const TriRec r = load_tri_c(B.ctris + (size_t)st * kLeafBlock + 1 + (lane - po) * kTriC);
            double t, u = 0.0, v = 0.0;
            if (tri_uvt_r<true>(r, oo, od, u, v, t, dir_tq(od))) { tt = t; uu = u; vv = v; }
        }
        // the fold: every result fetched first, then the reference's update sequence as
        // selects
        int win = -1;
        double x[kCoopMax];
#pragma unroll
        for (uint32_t k = 0; k < kCoopMax; ++k) x[k] = __shfl(tt, (int)(p + k));
        bool valid = T.valid;
        double best = T.best;
        uint32_t kw = 0;
#pragma unroll
        for (uint32_t k = 0; k < kCoopMax; ++k) {  // update_best_intersection, by selects
            const bool upd = take & (k < c) & !(x[k] < -0.5) & (!valid | (x[k] < best));
            valid = valid | upd;
            best = upd ? x[k] : best;
            win = upd ? (int)(p + k) : win;
            kw = upd ? k : kw;
        }
        const double wu = __shfl(uu, win), wv = __shfl(vv, win);
        if (win >= 0) { T.valid = true; T.best = best; T.prim = first + kw; T.aux = 0; T.bu = wu; T.bv = wv; }
        if (take) { C.tri(c); mine = false; }
        todo = __ballot(mine);
    }
}
#endif

// CMP: the triangle BVH's compact layout (DevBvh::cnodes / ctris, KIND 3 only):
// the same boxes and vertices as exact f32 copies, widened to f64 before the
// same arithmetic — every lane's visits, tests and results are the f64 form's.
// PAIR (with CMP): inner nodes from the pair layout (rt_layout.h kPairFloats), two BVH
// levels per line — see the branch below.
template <int KIND, int SLAB, bool ST, bool CMP = false, bool PAIR = false, class Stk>
RT_D void trav_step(const DevBvh& B, V3 o, V3 d, const Rcp3& rc, bool fast, Stk& S, Cnt<ST>& C, Trav& T,
                    uint64_t lv, int leaf_batch = kLeafBatch) {
    const unsigned long long ph_st = PH_T();
    const uint64_t at_leaf = __ballot(T.live && T.cnt != 0);
    const bool do_leaves = at_leaf == lv || __popcll(at_leaf) >= leaf_batch;
    PH_COUNT(kPhTravWave, kPhTravLane);
    if (T.live) PH_LANE(kPhLiveLane);
    bool next = false;  // this lane finished its current node and pops
    if (do_leaves) {
        const unsigned long long ph_l = PH_T();
#ifndef RT_LEAF_SERIAL
        if constexpr (KIND == 3 && CMP) leaf_coop(B, o, d, C, T);
#endif
        if (T.live && T.cnt != 0) {
            if constexpr (KIND == 3) {
                const uint32_t end = T.start + T.cnt;
                if constexpr (CMP) {
                    // Compact records are loaded when tested: a pipelined form holds the
                    // next record widened (18 VGPRs) through the test, which the 4-wave
                    // kernel pays in spills (a traversal-only kernel needs 105 VGPRs with it,
                    // 84 without): C3 -0.9%, C5 -1.9% at reduced spp
                    // (profiles/r03/variants/variants_leafpipe_C*.log); round 4, with the
                    // spill gone, prefetching only the next record's raw f32 words (9
                    // VGPRs) still loses: 3 -> 18 spilled VGPRs, C3 +1.5%, C5 +1.0%
                    // (profiles/r04/variants_leafpf_C*.log).
                    // the leaf's block (rt_layout.h kLeafBlock): T.start is its index, the
                    // first word its first primitive, then the records in order
                    const float* blk = B.ctris + (size_t)T.start * kLeafBlock;
                    const uint32_t first = *(const uint32_t*)blk;
                    const bool q = dir_tq(d);
#ifndef RT_LEAF_SERIAL
                    const uint32_t n_ser = T.cnt > kCoopMax ? T.cnt : 0u;  // small leaves: leaf_coop
#else
                    const uint32_t n_ser = T.cnt;
#endif
                    for (uint32_t k = 0; k < n_ser; ++k) {
                        PH_COUNT(kPhLeafWave, kPhLeafLane);
                        const TriRec cur = load_tri_c(blk + 1 + k * kTriC);
                        double t, u = 0.0, v = 0.0;
                        C.tri();
                        const bool h = tri_uvt_r<true>(cur, o, d, u, v, t, q);
                        if (h && (!T.valid || t < T.best)) {  // update_best_intersection (bvh.rs:213-222)
                            T.valid = true; T.best = t; T.prim = first + k; T.aux = 0;
                            T.bu = u; T.bv = v;
                        }
                    }
                } else {
                    // Software-pipelined leaf: the next triangle's record loads while this one
                    // is tested (C3 -0.8%, C5 -1.0% at reduced spp, variants_leafpipe_*.log).
                    TriRec cur = load_tri(B.tris[T.start]);
                    const bool q = B.tri_q && dir_tq(d);
                    for (uint32_t i = T.start; i < end; ++i) {
                        PH_COUNT(kPhLeafWave, kPhLeafLane);
                        TriRec nxt = cur;
                        if (i + 1 < end) nxt = load_tri(B.tris[i + 1]);
                        double t, u = 0.0, v = 0.0;
                        C.tri();
                        const bool h = tri_uvt_r<true>(cur, o, d, u, v, t, q);
                        if (h && (!T.valid || t < T.best)) {  // update_best_intersection (bvh.rs:213-222)
                            T.valid = true; T.best = t; T.prim = i; T.aux = 0;
                            T.bu = u; T.bv = v;
                        }
                        cur = nxt;
                    }
                }
            } else {
                for (uint32_t i = T.start; i < T.start + T.cnt; ++i) {
                    PH_COUNT(kPhLeafWave, kPhLeafLane);
                    double t, u = 0.0, v = 0.0;
                    uint32_t aux = 0;
                    C.shape();
                    const bool h = shape_closest<KIND>(B.shapes[i], o, d, rc, fast, t, aux);
                    if (h && (!T.valid || t < T.best)) {  // update_best_intersection (bvh.rs:213-222)
                        T.valid = true; T.best = t; T.bu = u; T.bv = v; T.prim = i; T.aux = aux;
                    }
                }
            }
            next = true;
        }
        PH_ADD(kPhLeafCyc, ph_l);
    } else if (PAIR && T.live && T.cnt == 0) {  // internal node, pair layout: up to two visits
        // Visit c = T.node: its line holds, per child K, the boxes a visit of K tests (K
        // internal; K's own box is their union — exact, build_pairs) or K's box (a leaf).
        // Both children are tested as in the compact branch (bvh.rs:158-185), then, when
        // the near child K is internal, K is visited at once from the same line — what the
        // reference does next (K has no primitives; `best` is unchanged) — so one dependent
        // load serves two levels.  Every visit counts as in the compact form (C.aabb / kids).
        const unsigned long long ph_i = PH_T();
        const float4* nw = (const float4*)(B.pnodes + (size_t)T.node * kPairFloats);
        const float4 a0 = nw[0], a1 = nw[1], a2 = nw[2];
        const uint4 aw = ((const uint4*)nw)[3];
        const float4 b0 = nw[4], b1 = nw[5], b2 = nw[6];
        const uint4 bw = ((const uint4*)nw)[7];
        asm volatile("" ::"v"(b0.x), "v"(b0.y), "v"(b0.z), "v"(b0.w), "v"(b1.x), "v"(b1.y), "v"(b1.z), "v"(b1.w),
                     "v"(b2.x), "v"(b2.y), "v"(b2.z), "v"(b2.w), "v"(bw.z), "v"(bw.w));  // one batch: see node_boxes
        PH_COUNT(kPhInnerWave, kPhInnerLane);
        // half: A = (x0.xyz | x0.w x1.xy), B = (x1.zw x2.x | x2.yzw); a child's box is A u B
        // (a leaf child's half holds its box twice)
        const bool la = aw.w & kPairLeaf, lb = bw.w & kPairLeaf;
        const float lmnx = fminf(a0.x, a1.z), lmny = fminf(a0.y, a1.w), lmnz = fminf(a0.z, a2.x),
                    lmxx = fmaxf(a0.w, a2.y), lmxy = fmaxf(a1.x, a2.z), lmxz = fmaxf(a1.y, a2.w);
        const float rmnx = fminf(b0.x, b1.z), rmny = fminf(b0.y, b1.w), rmnz = fminf(b0.z, b2.x),
                    rmxx = fmaxf(b0.w, b2.y), rmxy = fmaxf(b1.x, b2.z), rmxz = fmaxf(b1.y, b2.w);
        C.aabb(2);
        double lt = 0.0, rt2 = 0.0;
        const bool lh = slab_c<SLAB>(lmnx, lmny, lmnz, lmxx, lmxy, lmxz, o, d, rc, fast, lt);
        const bool rh = slab_c<SLAB>(rmnx, rmny, rmnz, rmxx, rmxy, rmxz, o, d, rc, fast, rt2);
        C.kids(lh, rh);
        double bt = T.best;  // +inf when no hit yet
        double li = lh ? (lt < bt ? lt : bt) : bt;
        double ri = rh ? (rt2 < bt ? rt2 : bt) : bt;
        bool go_left = false, push = false;
        uint32_t pw = 0;
        double pt = 0.0;
        if (li < bt) {
            if (ri < bt) {
                push = true;
                if (li < ri) { pw = bw.z; pt = ri; go_left = true; }
                else { pw = aw.z; pt = li; }
            } else go_left = true;
        } else if (!(ri < bt)) next = true;
        if (push) S.push(pw, pt);
        if (!next) {
            // the near child K: a leaf is entered by its word; an internal one is visited now
            const bool kl = go_left ? la : lb;
            if (kl) {
                trav_enter<true>(B, T, go_left ? aw.z : bw.z);
            } else {
                // K's half by selects (re-reading it from L1 instead: C3 +6%, C5 +4.5%,
                // profiles/r06/variants_pairreload_C*.log)
                const float4 k0 = go_left ? a0 : b0, k1 = go_left ? a1 : b1, k2 = go_left ? a2 : b2;
                const uint32_t kx = go_left ? aw.x : bw.x, ky = go_left ? aw.y : bw.y;
                C.aabb(2);
                const bool lh2 = slab_c<SLAB>(k0.x, k0.y, k0.z, k0.w, k1.x, k1.y, o, d, rc, fast, lt);
                const bool rh2 = slab_c<SLAB>(k1.z, k1.w, k2.x, k2.y, k2.z, k2.w, o, d, rc, fast, rt2);
                C.kids(lh2, rh2);
                li = lh2 ? (lt < bt ? lt : bt) : bt;
                ri = rh2 ? (rt2 < bt ? rt2 : bt) : bt;
                go_left = false;
                push = false;
                if (li < bt) {
                    if (ri < bt) {
                        push = true;
                        if (li < ri) { pw = ky; pt = ri; go_left = true; }
                        else { pw = kx; pt = li; }
                    } else go_left = true;
                } else if (!(ri < bt)) next = true;
                if (push) S.push(pw, pt);
                if (!next) trav_enter<true>(B, T, go_left ? kx : ky);
            }
        }
        PH_ADD(kPhInnerCyc, ph_i);
    } else if (CMP && T.live && T.cnt == 0) {  // internal node, compact layout (64 B)
        // both children's f32 boxes and their two child words (56 of the 64 B: a leaf's
        // own range is read by trav_enter)
        const unsigned long long ph_i = PH_T();
        const float4* nw = (const float4*)(B.cnodes + T.node);
        const float4 w0 = nw[0], w1 = nw[1], w2 = nw[2];
        const uint2 k = ((const uint2*)nw)[6];
        asm volatile("" ::"v"(w1.z), "v"(w1.w), "v"(w2.x), "v"(w2.y), "v"(w2.z), "v"(w2.w));  // see node_boxes
        PH_COUNT(kPhInnerWave, kPhInnerLane);
#ifdef RT_PHASES
        if (__ballot(T.node != (uint32_t)__builtin_amdgcn_readfirstlane(T.node)) == 0 && PH_FIRST())
            atomicAdd(&g_phase[kPhInnerUni], 1ull);
#endif
        C.aabb(2);
        bool go_left = false, push = false;
        uint32_t pw = 0;
        double pt = 0.0;
        double lt = 0.0, rt2 = 0.0;
        const bool lh = slab_c<SLAB>(w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, o, d, rc, fast, lt);
        const bool rh = slab_c<SLAB>(w1.z, w1.w, w2.x, w2.y, w2.z, w2.w, o, d, rc, fast, rt2);
        C.kids(lh, rh);
        const double bt = T.best;  // +inf when no hit yet
        const double li = lh ? (lt < bt ? lt : bt) : bt;
        const double ri = rh ? (rt2 < bt ? rt2 : bt) : bt;
        if (li < bt) {
            if (ri < bt) {
                push = true;
                if (li < ri) { pw = k.y; pt = ri; go_left = true; }
                else { pw = k.x; pt = li; }
            } else go_left = true;
        } else if (!(ri < bt)) next = true;
        if (push) S.push(pw, pt);
        if (!next) trav_enter<true>(B, T, go_left ? k.x : k.y);
        PH_ADD(kPhInnerCyc, ph_i);
    } else if (!CMP && T.live && T.cnt == 0) {  // internal node (count 0 <=> children)
        PH_COUNT(kPhInnerWave, kPhInnerLane);
        const DevNode& n = B.nodes[T.node];
        // the link words and the children's ranges, with the boxes (one 128-B line)
        const uint4 links = *(const uint4*)&n.left, kids = *(const uint4*)&n.lstart;
        double lt = 0.0, rt2 = 0.0;
        C.aabb(2);
        const NodeBoxes nb = node_boxes(n);
        const bool lh = slab_v<SLAB>(nb.lmn, nb.lmx, o, d, rc, fast, lt);
        const bool rh = slab_v<SLAB>(nb.rmn, nb.rmx, o, d, rc, fast, rt2);
        C.kids(lh, rh);
        const double bt = T.best;  // +inf when no hit yet
        const double li = lh ? (lt < bt ? lt : bt) : bt;
        const double ri = rh ? (rt2 < bt ? rt2 : bt) : bt;
        const uint32_t left = links.x, right = links.y;
        bool go_left = false;
        if (li < bt) {
            if (ri < bt) {
                if (li < ri) { S.push(child_word(right, kids.z, kids.w), ri); go_left = true; }
                else S.push(child_word(left, kids.x, kids.y), li);
            } else go_left = true;
        } else if (!(ri < bt)) next = true;
        if (!next) {
            T.node = go_left ? left : right;
            T.cnt = go_left ? kids.y : kids.w;
            T.start = go_left ? kids.x : kids.z;
        }
    }
    if (next) {  // resume from the stack: far children still closer than best
        const unsigned long long ph_p = PH_T();
        bool found = false;
        uint32_t w = 0;
        while (S.sp > 0) {
            double tt;
            S.pop(w, tt);
            if (tt < T.best) { found = true; break; }
        }
        if (!found) T.live = false;
        else trav_enter<CMP>(B, T, w);
        PH_ADD(kPhPopCyc, ph_p);
    }
    PH_ADD(kPhStepCyc, ph_st);
}

// BVH::intersection (bvh.rs:27-36) + Node::intersection (bvh.rs:151-186) run
// to completion, in two code forms with the same steps: TF = false is one
// self-contained loop (the fused kernel: C2 113 ms at 64 spp vs 116 through
// Trav), TF = true runs trav_init/trav_step (the resumable kernel, whose
// register allocation it suits better: C3 364 vs 375 ms).  Only the compiler's
// view differs; every lane's visits, tests and updates are identical.
template <int KIND, bool ST, bool FAST, class Stk>
RT_D bool bvh_closest_tf(const DevBvh& B, V3 o, V3 d, const Rcp3& rc, Stk& S, Cnt<ST>& C, double& bt_out,
                         double& bu, double& bv, uint32_t& bprim, uint32_t& baux) {
    constexpr int SL = FAST ? 1 : 0;
    Trav T;
    trav_init<SL, ST>(B, o, d, rc, FAST, S, C, T);
    for (;;) {
        const uint64_t lv = __ballot(T.live);
        if (lv == 0) break;
        trav_step<KIND, SL, ST>(B, o, d, rc, FAST, S, C, T, lv);
    }
    if (T.valid) { bt_out = T.best; bu = T.bu; bv = T.bv; bprim = T.prim; baux = T.aux; }
    return T.valid;
}

template <int KIND, bool ST, bool FAST, class Stk>
RT_D bool bvh_closest(const DevBvh& B, V3 o, V3 d, const Rcp3& rc, Stk& S, Cnt<ST>& C, double& bt_out,
                      double& bu, double& bv, uint32_t& bprim, uint32_t& baux) {
    if (B.n_prims == 0) return false;
    double t0;
    C.aabb();
    if (!aabb_hit<FAST>(load3(B.root_min), load3(B.root_max), o, d, rc, t0)) return false;
    bool valid = false;
    double best = INFINITY;
    const bool tq = KIND == 3 && B.tri_q && dir_tq(d);  // the split-division triangle solve
    if (B.depth == 1) {  // the root is the only leaf (bvh.rs:77, <= 4 primitives): [0, n_prims) in order
        // uniform index: the records come through the scalar cache
        const uint32_t np = uni_u32(B.n_prims);
        const RT_CAS DevTri* tris = uni(B.tris);
        const RT_CAS DevShape* shapes = uni(B.shapes);
        auto test = [&](uint32_t i) {
            double t, u = 0.0, v = 0.0;
            uint32_t aux = 0;
            bool h;
            if (KIND == 3) { C.tri(); const DevTri tr = tris[i]; h = tri_uvt(tr, o, d, u, v, t, tq); }
            else { C.shape(); const DevShape sh = shapes[i]; h = shape_closest<KIND>(sh, o, d, rc, FAST, t, aux); }
            if (h && (!valid || t < best)) {  // update_best_intersection (bvh.rs:213-222)
                valid = true; best = t; bu = u; bv = v; bprim = i; baux = aux;
            }
        };
        for (uint32_t i = 0; i < np; ++i) test(i);
        if (valid) bt_out = best;
        return valid;
    }
    uint32_t node = 0;
    S.sp = 0;
    // Deferred leaves: a lane that reaches a leaf waits there while the other
    // lanes keep stepping through internal nodes; the wave tests leaf
    // primitives once >= kLeafBatch lanes wait (or every live lane does), so
    // the primitive loop runs with many lanes instead of a few.  Each lane's
    // own sequence of visits, tests, `best` updates and pruning is unchanged
    // (the reference's order, bvh.rs:151-210) — only when it runs moves.
    uint32_t cnt = B.nodes[0].count, start = B.nodes[0].start;  // current node's primitive range
    bool live = true;
    for (;;) {
        const uint64_t lv = __ballot(live);
        if (lv == 0) break;
        const uint64_t at_leaf = __ballot(live && cnt != 0);
        const bool do_leaves = at_leaf == lv || __popcll(at_leaf) >= kLeafBatch;
        PH_COUNT(kPhTravWave, kPhTravLane);
        if (live) PH_LANE(kPhLiveLane);
        bool next = false;  // this lane finished its current node and pops
        if (do_leaves) {
            if (live && cnt != 0) {
                for (uint32_t i = start; i < start + cnt; ++i) {
                    PH_COUNT(kPhLeafWave, kPhLeafLane);
                    double t, u = 0.0, v = 0.0;
                    uint32_t aux = 0;
                    bool h;
                    if (KIND == 3) { C.tri(); h = tri_uvt(B.tris[i], o, d, u, v, t, tq); }
                    else { C.shape(); h = shape_closest<KIND>(B.shapes[i], o, d, rc, FAST, t, aux); }
                    if (h && (!valid || t < best)) {  // update_best_intersection (bvh.rs:213-222)
                        valid = true; best = t; bu = u; bv = v; bprim = i; baux = aux;
                    }
                }
                next = true;
            }
        } else if (live && cnt == 0) {  // internal node (count 0 <=> children)
            PH_COUNT(kPhInnerWave, kPhInnerLane);
            const DevNode& n = B.nodes[node];
            // the link words and the children's ranges, with the boxes (one 128-B line)
            const uint4 links = *(const uint4*)&n.left, kids = *(const uint4*)&n.lstart;
            double lt = 0.0, rt2 = 0.0;
            C.aabb(2);
            bool lh = aabb_hit<FAST>(load3(n.lmin), load3(n.lmax), o, d, rc, lt);
            bool rh = aabb_hit<FAST>(load3(n.rmin), load3(n.rmax), o, d, rc, rt2);
            C.kids(lh, rh);
            const double bt = best;  // +inf when no hit yet
            const double li = lh ? (lt < bt ? lt : bt) : bt;
            const double ri = rh ? (rt2 < bt ? rt2 : bt) : bt;
            const uint32_t left = links.x, right = links.y;
            bool go_left = false;
            if (li < bt) {
                if (ri < bt) {
                    if (li < ri) { S.push(child_word(right, kids.z, kids.w), ri); go_left = true; }
                    else S.push(child_word(left, kids.x, kids.y), li);
                } else go_left = true;
            } else if (!(ri < bt)) next = true;
            if (!next) {
                node = go_left ? left : right;
                cnt = go_left ? kids.y : kids.w;
                start = go_left ? kids.x : kids.z;
            }
        }
        if (next) {  // resume from the stack: far children still closer than best
            bool found = false;
            uint32_t w = 0;
            while (S.sp > 0) {
                double tt;
                S.pop(w, tt);
                if (tt < best) { found = true; break; }
            }
            if (!found) live = false;
            else if (w & kPackedLeaf) { cnt = (w >> 24) & 127u; start = w & 0xFFFFFFu; }
            else if (w & kLeafRef) { node = w & ~kLeafRef; cnt = B.nodes[node].count; start = B.nodes[node].start; }
            else { node = w; cnt = 0; }
        }
    }
    if (valid) bt_out = best;
    return valid;
}

// Slab tests with the unguarded exact division when the BVH's boxes and this
// ray allow it (DevBvh::fast, ray_fast); the guarded form otherwise.
template <int KIND, bool ST, bool TF = false, class Stk>
RT_D bool bvh_closest_sel(const DevBvh& B, bool rfast, V3 o, V3 d, const Rcp3& rc, Stk& S, Cnt<ST>& C,
                          double& bt_out, double& bu, double& bv, uint32_t& bprim, uint32_t& baux) {
    if constexpr (TF) {
        if (B.fast && rfast) return bvh_closest_tf<KIND, ST, true>(B, o, d, rc, S, C, bt_out, bu, bv, bprim, baux);
        return bvh_closest_tf<KIND, ST, false>(B, o, d, rc, S, C, bt_out, bu, bv, bprim, baux);
    }
    if (B.fast && rfast) return bvh_closest<KIND, ST, true>(B, o, d, rc, S, C, bt_out, bu, bv, bprim, baux);
    return bvh_closest<KIND, ST, false>(B, o, d, rc, S, C, bt_out, bu, bv, bprim, baux);
}

// Materialise the winning candidate: model-space normals + their rotation, or
// (world = true) the final world normals.  KM: the scene's primitive kinds
// (kShapes | kTris, below), so a one-kind scene's instance has no code for the
// other kind.
template <int KM = 3>
RT_D Hit materialise(const DevScene& S, const Cand& c, V3 o, V3 d, Quat& rot, uint32_t& mat, int32_t& gid,
                     bool& world) {
    Hit h;
    h.t = c.t;
    world = false;
    if (KM == kTris || (KM & kTris && c.kind == 3)) {  // Triangle::intersection tail (triangle.rs:71-79), DONT_ROTATE
        const DevBvh& B = S.tris;
        const DevTriCold& tc = B.tri_cold[c.prim];
        V3 n = load3(tc.ng), na = load3(tc.na), nb = load3(tc.nb), nc = load3(tc.nc);
        V3 sn = nrm(na + (nb - na) * c.u + (nc - na) * c.v);
        bool inside = dot(d, n) > 0.0;
        h.ng = inside ? -n : n;
        h.ns = inside ? -sn : sn;
        h.inside = inside;
        rot = Quat{1.0, v3(0.0, 0.0, 0.0)};
        mat = B.mat[c.prim];
        gid = B.gid[c.prim];
        return h;
    }
    // Plane sides and box faces have per-primitive constant normals: their
    // with_rotated_normal result (rotate by rot, normalize) is a host-computed
    // table (DevScene::plane_nrm / box_nrm), so `world` skips rotated().
    if (c.kind == 0) {  // n * (aux bit0 ? 1 : -1)
        mat = S.plane_mat[c.prim]; gid = S.plane_gid[c.prim];
        const V3 n = load3(S.plane_nrm + ((size_t)c.prim * 2 + (c.aux & 1u)) * 3);
        h.ng = n; h.ns = n; h.inside = false;
        world = true;
        return h;
    }
    if (c.kind == 1) {  // aux_box_normal(aux)
        mat = S.boxes.mat[c.prim]; gid = S.boxes.gid[c.prim];
        const V3 n = load3(S.box_nrm + ((size_t)c.prim * 8 + (c.aux & 7u)) * 3);
        h.ng = n; h.ns = n; h.inside = (c.aux & 8u) != 0;
        world = true;
        return h;
    }
    const DevBvh& B = S.ells;
    mat = B.mat[c.prim]; gid = B.gid[c.prim];
    const DevShape s = B.shapes[c.prim];
    rot = load_quat(s.rot);
    {
        V3 mo, md;
        model_ray(s, o, d, mo, md);
        V3 n = ell_normal(load_radii(s), mo, md, c.t);
        bool inside = (c.aux & 8u) != 0;
        if (inside) n = -n;
        // both normals are this n, so with_rotated_normal's two rotate + normalize
        // results are the same bits: computed once here (world = true)
        n = nrm(rotate_fast(rot, is_identity(rot), n));
        h.ng = n; h.ns = n; h.inside = inside;
        world = true;
    }
    return h;
}

// One box of a single-leaf box BVH: box_coef on the model-space ray, exactly
// as shape_closest<1> (closest hit) and leaf_all<1> (light pdf) compute it —
// the fast and generic forms give the same bits.
RT_D int box_test(const DevShape& s, V3 o, V3 d, const Rcp3& rc, bool rfast, Bpi& en, Bpi& ex) {
    V3 mo, md;
#ifndef RT_NO_FASTSHAPE
    if (shape_fast(s, rfast, o, mo)) return box_coef<true>(load3(s.shape), mo, d, rc, en, ex);
#endif
    const bool same = model_ray(s, o, d, mo, md);
    return box_model(s, mo, md, same, rc, en, ex);
}
// The Light::pdf callback terms of one light box crossing (leaf_all<1>:
// intersection_probability.rs:15-23, ray_sampler.rs:132-139,172-174)
template <bool ST>
RT_D void box_light_terms(const DevShape& s, int k, const Bpi& en, const Bpi& ex, V3 d, Cnt<ST>& C,
                          double& impact) {
    const double pb = s.aux[0];
    const Quat q = load_quat(s.rot);
    const bool qid = is_identity(q);
    if (k == 2) {
        const double dn = qid ? fabs(comp(d, bpi_dim(en))) : fabs(dot(d, nrm(rotate(q, bpi_normal(en)))));
        impact += pb * (en.t * en.t / dn);
        C.lhit();
    }
    if (k >= 1) {
        const double dn = qid ? fabs(comp(d, bpi_dim(ex))) : fabs(dot(d, nrm(rotate(q, bpi_normal(ex)))));
        impact += pb * (ex.t * ex.t / dn);
        C.lhit();
    }
}

// Shared light tests (DevScene::slt_mask): the box part of `intersect` for a
// single-leaf box BVH, which also yields the Light::pdf sum of the previous
// diffuse bounce for lanes whose pdf is pending (`pend`).  That bounce's light
// query ray (pos + dir * eps, dir) IS this segment's ray, and every light is a
// box whose record equals scene box i of the mask, so each light crossing comes
// from the box_coef this query computes anyway.  Per lane, the steps and
// counters are those of bvh_closest (bvh.rs:27-36) followed by intersect_lights
// (intersections.rs:87-91 over lboxes; lells and ltris are empty), including
// both root AABB tests: a light box is tested for the pdf exactly when the
// light BVH's root is hit, whatever the scene BVH's root test said.
template <bool ST>
RT_D void boxes_slt(const DevScene& S, V3 o, V3 d, const Rcp3& rc, bool rfast, bool pend, Cnt<ST>& C, bool& valid,
                    double& bt, uint32_t& bp, uint32_t& baux, double& impact) {
    const DevBvh& B = S.boxes;
    const DevBvh& L = S.lboxes;
    valid = false;
    double t0;
    C.aabb();
    const bool sroot = (B.fast && rfast) ? aabb_hit<true>(load3(B.root_min), load3(B.root_max), o, d, rc, t0)
                                         : aabb_hit<false>(load3(B.root_min), load3(B.root_max), o, d, rc, t0);
    bool lroot = false;
    if (pend) {
        C.lq();
        C.aabb();
        lroot = slab<2>(L.root_min, L.root_max, o, d, rc, L.fast && rfast, t0);
    }
    const uint32_t np = uni_u32(B.n_prims), mask = uni_u32(S.slt_mask);
    const RT_CAS DevShape* shapes = uni(B.shapes);
    double best = INFINITY;
    auto test = [&](uint32_t i) {
        const bool lt = ((mask >> i) & 1u) && lroot;
        if (!(sroot || lt)) return;
        const DevShape sh = shapes[i];
        Bpi en, ex;
        const int k = box_test(sh, o, d, rc, rfast, en, ex);
        if (sroot) {
            C.shape();
            if (k > 0) {
                const double t = k == 2 ? en.t : ex.t;
                if (!valid || t < best) {  // update_best_intersection (bvh.rs:213-222)
                    valid = true; best = t; bp = i; baux = k == 2 ? bpi_aux(en, false) : bpi_aux(ex, true);
                }
            }
        }
        if (lt) {
            C.shape();
            box_light_terms<ST>(sh, k, en, ex, d, C, impact);
        }
    };
    // the first two boxes unrolled (a uniform early exit): C2 -1.3%
#pragma unroll
    for (uint32_t i = 0; i < 2; ++i) {
        if (i >= np) break;
        test(i);
    }
    for (uint32_t i = 2; i < np; ++i) test(i);
    if (valid) bt = best;
}

// intersect(ray, &scene.primitives, +inf) (intersections.rs:42-62) in three
// parts, so the path kernel can traverse the triangle BVH resumably:
// shapes_closest (planes, boxes, ellipsoids: :45-55), take_tri (triangles
// last, strict <: :55), intersect_tail (:56-61).
// SLT: the fused path kernel's form, with the shared light tests of boxes_slt.
template <bool ST, bool TF, class Stk, bool SLT = false>
RT_D void shapes_closest(const DevScene& S, V3 o, V3 d, const Rcp3& rc, bool rfast, Stk& stk, Cnt<ST>& C,
                         Cand& best, bool pend = false, double* impact = nullptr) {
    best.valid = false; best.t = 0.0; best.u = best.v = 0.0; best.prim = 0; best.aux = 0; best.kind = 0;
    unsigned long long ph = PH_T();
    const uint32_t np = uni_u32(S.n_planes);
    const RT_CAS DevShape* planes = uni(S.planes);
    // the first 8 planes unrolled (a uniform early exit): their records' scalar
    // loads issue together instead of one loop trip at a time (C2 -1.9%)
#pragma unroll
    for (uint32_t i = 0; i < 8; ++i) {
        if (i >= np) break;
        double t; uint32_t aux;
        C.shape();
        const DevShape sh = planes[i];
        if (!shape_closest<0>(sh, o, d, rc, rfast, t, aux)) continue;
        if (!best.valid || t < best.t) { best.valid = true; best.t = t; best.prim = i; best.aux = aux; best.kind = 0; }
    }
    for (uint32_t i = 8; i < np; ++i) {  // :45-49
        double t; uint32_t aux;
        C.shape();
        const DevShape sh = planes[i];
        if (!shape_closest<0>(sh, o, d, rc, rfast, t, aux)) continue;
        if (!best.valid || t < best.t) { best.valid = true; best.t = t; best.prim = i; best.aux = aux; best.kind = 0; }
    }
    PH_ADD(kPhPlanes, ph);
    ph = PH_T();
    if (SLT && uni_u32(S.slt_mask)) {
        bool bv; double t = 0.0; uint32_t p = 0, aux = 0;
        boxes_slt<ST>(S, o, d, rc, rfast, pend, C, bv, t, p, aux, *impact);
        if (bv && (!best.valid || t < best.t)) {
            best.valid = true; best.t = t; best.prim = p; best.aux = aux; best.kind = 1;
        }
    } else {
        double t, u, v; uint32_t p, aux = 0;
        if (bvh_closest_sel<1, ST, TF>(S.boxes, rfast, o, d, rc, stk, C, t, u, v, p, aux) && (!best.valid || t < best.t)) {
            best.valid = true; best.t = t; best.prim = p; best.aux = aux; best.kind = 1;
        }
    }
    PH_ADD(kPhBoxes, ph);
    ph = PH_T();
    {
        double t, u, v; uint32_t p, aux = 0;
        if (bvh_closest_sel<2, ST, TF>(S.ells, rfast, o, d, rc, stk, C, t, u, v, p, aux) && (!best.valid || t < best.t)) {
            best.valid = true; best.t = t; best.prim = p; best.aux = aux; best.kind = 2;
        }
    }
    PH_ADD(kPhElls, ph);
}
RT_D void take_tri(Cand& best, bool valid, double t, double u, double v, uint32_t p) {
    if (valid && (!best.valid || t < best.t)) {
        best.valid = true; best.t = t; best.prim = p; best.u = u; best.v = v; best.aux = 0; best.kind = 3;
    }
}
template <bool ST, int KM = 3>
RT_D bool intersect_tail(const DevScene& S, const Cand& best, V3 o, V3 d, Cnt<ST>& C, Hit& out, uint32_t& mat,
                         int32_t& gid) {
    if (!best.valid) return false;
    // :56, t * d.magnitude() <= +inf, i.e. the product is not NaN.  With dd = d.d
    // (>= 0 or NaN), sqrt(dd) is NaN / 0 / inf exactly when dd is, so the product
    // is NaN iff t or dd is NaN, or t is inf and dd 0, or t is 0 and dd inf: the
    // same outcome without the square root.
    const double dd = dot(d, d);
    if (isnan(best.t) || isnan(dd) || (isinf(best.t) && dd == 0.0) || (best.t == 0.0 && isinf(dd))) return false;
    const unsigned long long ph = PH_T();
    Quat rot;
    bool world;
    Hit h = materialise<KM>(S, best, o, d, rot, mat, gid, world);
    out = world ? h : rotated(h, rot);
    PH_ADD(kPhMaterialise, ph);
    C.shaded();
    return true;
}
template <bool ST, class Stk, bool SLT = false, int KM = 3>
RT_D bool scene_intersect(const DevScene& S, V3 o, V3 d, Stk& stk, Cnt<ST>& C, Hit& out, uint32_t& mat,
                          int32_t& gid, bool pend = false, double* impact = nullptr) {
    const Rcp3 rc = make_rcp3(d);
    const bool rfast = ray_fast(o, rc);
    Cand best;
    shapes_closest<ST, false, Stk, SLT>(S, o, d, rc, rfast, stk, C, best, pend, impact);
    if (KM & kTris) {
        const unsigned long long ph = PH_T();
        double t, u = 0.0, v = 0.0; uint32_t p = 0, aux = 0;
        const bool th = bvh_closest_sel<3, ST>(S.tris, rfast, o, d, rc, stk, C, t, u, v, p, aux);
        take_tri(best, th, t, u, v, p);
        PH_ADD(kPhTris, ph);
    }
    return intersect_tail<ST, KM>(S, best, o, d, C, out, mat, gid);
}

// ---------------------------------------------------------- light pdf ----
// intersection_probability.rs:9-35 + to_direction_probability (ray_sampler.rs:172-174)
// (the box's 1/sum/8 is a per-primitive constant precomputed on the host: DevShape::aux[0])
RT_D double prob_ell(V3 r, V3 ng) {
    V3 coef = mul(v3(r.y * r.z, r.x * r.z, r.x * r.y), ng);
    return 1.0 / (4.0 * kPi * sqrt(dot(coef, coef)));
}

// the Light::pdf callback over the primitives [start, start + cnt) of a leaf
// (bvh.rs:194-198 -> intersection_probability.rs:9-35)
// UNI: [start, start + cnt) is the same for every lane (the single-leaf BVH),
// so the shape records come through the scalar cache (uni)
template <int KIND, bool ST, bool UNI = false>
RT_D void leaf_all(const DevBvh& B, uint32_t start, uint32_t cnt, V3 o, V3 d, const Rcp3& rc, bool rfast,
                   Cnt<ST>& C, double& impact, uint32_t& nhits) {
    constexpr bool kUni = UNI;
    if (kUni) cnt = uni_u32(cnt);
    for (uint32_t i = start; i < start + cnt; ++i) {
        if (KIND == 3) {
            C.tri();
            double u, v, t;
            DevTri tr;
            if (kUni) tr = uni(B.tris)[i];
            else tr = B.tris[i];
            if (tri_uvt(tr, o, d, u, v, t, B.tri_q && dir_tq(d))) {
                V3 ng = load3(B.tri_cold[i].ng);  // sign flip (triangle.rs:76) cancels in |d.n|
                impact += B.tri_inv_area[i] * (t * t / fabs(dot(d, ng)));
                C.lhit(); nhits++;
            }
        } else {
            C.shape();
            DevShape s;
            if (kUni) s = uni(B.shapes)[i];
            else s = B.shapes[i];
            V3 mo, md;
#ifndef RT_NO_FASTSHAPE
            const bool fs = shape_fast(s, rfast, o, mo);  // then model_ray gives (o - pos, d)
#else
            const bool fs = false;
#endif
            bool same = true;
            if (fs) md = d;
            else same = model_ray(s, o, d, mo, md);
            Quat q = load_quat(s.rot);
            const bool qid = is_identity(q);
            V3 sz = load3(s.shape);
            if (KIND == 1) {
                Bpi en, ex;
                int k = fs ? box_coef<true>(sz, mo, md, rc, en, ex) : box_model(s, mo, md, same, rc, en, ex);
                const double pb = s.aux[0];
                // |d . normalize(rotate(q, n))| for a face normal n = sign * e_dim.  With an
                // identity q, rotate returns n up to the signs of its zero components and
                // normalize leaves a unit axis vector unchanged, so the dot is +-d[dim] up to
                // signed zeros, which fabs discards: exactly |d[dim]|.
                if (k == 2) {
                    const double dn = qid ? fabs(comp(d, bpi_dim(en))) : fabs(dot(d, nrm(rotate(q, bpi_normal(en)))));
                    impact += pb * (en.t * en.t / dn);
                    C.lhit(); nhits++;
                }
                if (k >= 1) {
                    const double dn = qid ? fabs(comp(d, bpi_dim(ex))) : fabs(dot(d, nrm(rotate(q, bpi_normal(ex)))));
                    impact += pb * (ex.t * ex.t / dn);
                    C.lhit(); nhits++;
                }
            } else {
                double t1, t2;
                const Radii R = load_radii(s);
                int k = fs ? ell_coef<true>(R, mo, md, t1, t2) : ell_coef(R, mo, md, t1, t2);
                if (k == 2) {
                    V3 ng = nrm(rotate_fast(q, qid, ell_normal(R, mo, md, t1)));
                    impact += prob_ell(sz, ng) * (t1 * t1 / fabs(dot(d, ng)));
                    C.lhit(); nhits++;
                }
                if (k >= 1) {
                    V3 ng = nrm(rotate_fast(q, qid, -ell_normal(R, mo, md, t2)));
                    impact += prob_ell(sz, ng) * (t2 * t2 / fabs(dot(d, ng)));
                    C.lhit(); nhits++;
                }
            }
        }
    }
}

// Node::intersections (bvh.rs:188-210) accumulating the Light::pdf callback
template <int KIND, bool ST, class Stk>
RT_D void bvh_all(const DevBvh& B, V3 o, V3 d, const Rcp3& rc, bool rfast, Stk& S, Cnt<ST>& C, double& impact,
                  uint32_t& nhits) {
    if (B.n_prims == 0) return;
    double t0;
    C.aabb();
    const bool fast = B.fast && rfast;  // unguarded exact slab division (aabb_hit_fast)
    if (!slab<2>(B.root_min, B.root_max, o, d, rc, fast, t0)) return;
    if (B.depth == 1) {  // the root is the only leaf: [0, n_prims), no stack
        leaf_all<KIND, ST, true>(B, 0u, B.n_prims, o, d, rc, rfast, C, impact, nhits);
        return;
    }
    uint32_t node = 0;
    S.sp = 0;
    for (;;) {
        const DevNode& n = B.nodes[node];
        const uint32_t cnt = n.count, start = n.start;
        leaf_all<KIND, ST>(B, start, cnt, o, d, rc, rfast, C, impact, nhits);
        const int32_t left = n.left;
        if (left >= 0) {
            double lt, rt2;
            C.aabb(2);
            bool lh = slab<2>(n.lmin, n.lmax, o, d, rc, fast, lt);
            bool rh = slab<2>(n.rmin, n.rmax, o, d, rc, fast, rt2);
            if (lh) {
                if (rh) S.push((uint32_t)n.right, 0.0);
                node = (uint32_t)left;
                continue;
            }
            if (rh) { node = (uint32_t)n.right; continue; }
        }
        if (S.sp == 0) break;
        double tt;
        S.pop(node, tt);
    }
}

// intersect_lights (intersections.rs:87-91): boxes, ellipsoids, triangles (KM:
// the scene's primitive kinds; the light BVHs of an absent kind are empty)
template <bool ST, class Stk, int KM = 3>
RT_D double lights_impact(const DevScene& S, V3 o, V3 d, Stk& stk, Cnt<ST>& C, uint32_t& nhits) {
    double impact = 0.0;
    const Rcp3 rc = make_rcp3(d);
    const bool rfast = ray_fast(o, rc);
    if (KM & kShapes) {
        bvh_all<1, ST>(S.lboxes, o, d, rc, rfast, stk, C, impact, nhits);
        bvh_all<2, ST>(S.lells, o, d, rc, rfast, stk, C, impact, nhits);
    }
    if (KM & kTris) bvh_all<3, ST>(S.ltris, o, d, rc, rfast, stk, C, impact, nhits);
    return impact;
}
// the same query from its origin q = pos + dir * kEpsilon, already computed
template <bool ST, class Stk, int KM = 3>
RT_D double light_pdf_at(const DevScene& S, V3 q, V3 dir, Stk& stk, Cnt<ST>& C) {
    C.lq();
    uint32_t nh = 0;
    double impact = lights_impact<ST, Stk, KM>(S, q, dir, stk, C, nh);
    const uint32_t nl = S.n_lights;  // x / 1 == x exactly: skip the division sequence for one light
    return nl == 1u ? impact : impact / (double)nl;
}
template <bool ST, class Stk, int KM = 3>
RT_D double light_pdf(const DevScene& S, V3 pos, V3 dir, Stk& stk, Cnt<ST>& C) {  // ray_sampler.rs:132-139
    C.lq();
    uint32_t nh = 0;
    double impact = lights_impact<ST, Stk, KM>(S, pos + dir * kEpsilon, dir, stk, C, nh);
    const uint32_t nl = S.n_lights;  // x / 1 == x exactly: skip the division sequence for one light
    return nl == 1u ? impact : impact / (double)nl;
}

// ------------------------------------------------------------ samplers ----
// The diffuse sampler's draws (Mix::sample, ray_sampler.rs:87-93).  After the
// Mix coin both branches take the same three u64 draws A, B, C of the stream
// and differ only in how they map them, so the draws (and their Philox
// refills) run once for the wave instead of once per branch.  The layout
// (oracle.c diffuse_sample does the same) keeps every distribution:
//   cosine (ray_sampler.rs:69-76, uniform_on_sphere :159-170): gen_f64 of A, B, C;
//   box light (uniform_on_box :142-157): choice = gen_range of A, sign = the
//     lowest bit of A (value0_1 uses only A's top 52 bits, so the two are
//     independent), u1 / u2 = the inclusive [-1, 1] draws of B / C;
//   ellipsoid light: uniform_on_sphere of A, B, C; triangle light: u, v of A, B;
//   the light index (more than one light) is drawn after C.
RT_D double f64_of(uint64_t u) { return (double)(u >> 11) * (1.0 / 9007199254740992.0); }  // Standard f64
RT_D double unit_of(uint64_t u) {  // value0_1 (UniformFloat's [0, 1) form)
    return __longlong_as_double((long long)((u >> 12) | 0x3FF0000000000000ull)) - 1.0;
}
RT_D V3 cube_point(uint64_t A, uint64_t B, uint64_t C) {  // uniform_on_sphere before its normalize
    return v3(f64_of(A) * 2.0 - 1.0, f64_of(B) * 2.0 - 1.0, f64_of(C) * 2.0 - 1.0);
}
struct Scales { double s01, s11; };  // new_inclusive scales for [0,1] and [-1,1]
RT_D V3 uniform_on_box(V3 s, uint64_t A, uint64_t B, uint64_t C, Rng& r, const Scales& sc) {  // :142-157
    double w4x = s.y * s.z, w4y = s.x * s.z, w4z = s.x * s.y;
    const double high = (w4x + w4y) + w4z, scale = high - 0.0;
    double choice;
    for (;;) {  // gen_range(0.0, high) (UniformFloat::sample_single): never rejects, kept for form
        choice = unit_of(A) * scale + 0.0;
        if (choice < high) break;
        A = next_u64(r);
    }
    const double sign = (A & 1u) ? 1.0 : -1.0;
    const double u1 = unit_of(B) * sc.s11 + -1.0, u2 = unit_of(C) * sc.s11 + -1.0;  // gen_range(-1.0..=1.0)
    V3 p;
    if (choice < w4x) p = v3(sign, u1, u2);
    else if (choice < w4x + w4y) p = v3(u1, sign, u2);
    else p = v3(u1, u2, sign);
    return mul(p, s);
}
template <int KM = 3>
RT_D V3 light_point(const DevScene& S, uint64_t A, uint64_t B, uint64_t C, Rng& r,
                    const Scales& sc) {  // ray_sampler.rs:101-129
    // a one-element range needs no draw (the result is 0 either way; oracle.c gen_range_usize)
    const uint32_t nl = uni_u32(S.n_lights);
    uint64_t index = 0;
    if (nl != 1u) {
        rng_top_up(r);
        index = gen_index(r, nl, S.light_zone);
    }
    constexpr bool TO = KM == kTris;
    const uint32_t nb = TO ? 0u : S.lboxes.n_prims, ne = TO ? 0u : S.lells.n_prims;
    V3 world;
    if (!TO && index < nb) {
        const DevShape l = S.lboxes.shapes[index];
        const Quat q = load_quat(l.rot);
        world = rotate_fast(q, is_identity(q), uniform_on_box(load3(l.shape), A, B, C, r, sc)) + load3(l.pos);
    } else if (!TO && (KM == kShapes || index < (uint64_t)nb + ne)) {
        const DevShape l = S.lells.shapes[index - nb];
        const Quat q = load_quat(l.rot);
        world = rotate_fast(q, is_identity(q), mul(nrm(cube_point(A, B, C)), load3(l.shape))) + load3(l.pos);
    } else {
        const DevTri t = S.ltris.tris[index - nb - ne];
        double u = unit_of(A) * sc.s01 + 0.0;  // gen_range(0.0..=1.0)
        double v = unit_of(B) * sc.s01 + 0.0;
        if (u + v > 1.0) { u = 1.0 - u; v = 1.0 - v; }
        world = (load3(t.ba) * u + load3(t.ca) * v) + load3(t.a);
    }
    return world;
}
// The last-bounce light query may be skipped: its origin q lies outside every
// light's grown world box (DevScene::lq_boxes; zero when the scene does not qualify)
RT_D bool lq_skippable(const DevScene& S, V3 q) {
    const uint32_t n = uni_u32(S.lq_boxes);
    if (n == 0) return false;
    bool inside = false;
    for (uint32_t i = 0; i < n; ++i) {
        const double* b = S.lq_box[i];
        inside = inside || (q.x >= b[0] && q.y >= b[1] && q.z >= b[2] && q.x <= b[3] && q.y <= b[4] && q.z <= b[5]);
    }
    return !inside && q.x == q.x && q.y == q.y && q.z == q.z;
}
RT_D double cosine_pdf(V3 n, V3 d) {  // ray_sampler.rs:78-83
    if (dot(n, d) <= 0.0) return 0.0;
    return dot(n, d) / kPi;
}

// --------------------------------------------------------- integrator ----
RT_D double powi5(double x) { double x2 = x * x; return x * (x2 * x2); }

// Throughput weight of a diffuse bounce, col * cos / pi / pdf (raytrace.rs:26-33),
// as col * (cosine_pdf / pdf): cosine_pdf is cos / pi exactly as computed for the
// Mix pdf (cos > 0 here), so one division replaces the six of the per-channel
// form.  The weight only scales radiance — no random decision reads it — so hit
// ids stay bit-exact and radiance moves by an ulp-level reassociation (oracle.c
// raytrace_iter does the same; the recursive form is within rtol 1e-12).
RT_D V3 diffuse_weight(V3 col, double cp, double pdf) {
    const double f = cp / pdf;
    return v3(col.x * f, col.y * f, col.z * f);
}

struct PathState {
    V3 o, d;       // current ray
    V3 T;          // throughput
    V3 L;          // radiance of this path so far
    // a diffuse bounce whose light pdf comes with this segment's box tests
    // (boxes_slt): its cos(dir, n), cosine pdf and material; T is updated once
    // the pdf is known, before anything reads it
    bool pend;
    double pcos;
    uint32_t pmat;
};

// The closest-hit query of one segment, held across path-loop trips while the
// lane's triangle traversal is suspended (path_kernel): the ray's reciprocals,
// the best plane/box/ellipsoid candidate and the triangle-BVH traversal state.
struct SegQuery {
    Rcp3 rc;
    Cand best;
    Trav T;
    bool fast;  // unguarded slab division for the triangle BVH (DevBvh::fast && ray_fast)
};

// raytrace_impl's `intersect` call (raytrace.rs:13), first part: planes,
// boxes and ellipsoids to completion, then the triangle traversal is set up.
// KM == kTris (a triangle-only scene): no shapes to test, and the candidate is
// the triangle traversal's alone (q.best is not carried across the loop)
template <bool ST, int KM = 3, class Stk>
RT_D void segment_begin(const DevScene& S, const PathState& ps, Stk& stk, Cnt<ST>& C, SegQuery& q) {
    C.segment();
    q.rc = make_rcp3(ps.d);
    const bool rfast = ray_fast(ps.o, q.rc);
    if (KM != kTris) shapes_closest<ST, true>(S, ps.o, ps.d, q.rc, rfast, stk, C, q.best);
    q.fast = S.tris.fast && rfast;
    trav_init<2, ST>(S.tris, ps.o, ps.d, q.rc, q.fast, stk, C, q.T);
}

// A lane's throughput T and radiance L in the wave's LDS block, [component][lane]
// (the 4-wave resumable kernel).  The lane index is re-derived (stack_lane), so
// it is not held in a register across the traversal either.  The shading step
// updates them in place (tl_add_L, tl_mul_T) where the reference does, so they
// occupy no registers while the light query and the samplers run (round 4).
RT_D void tl_store(double* s_tl, V3 T, V3 L) {
    const uint32_t l = stack_lane();
    s_tl[l] = T.x; s_tl[kWave + l] = T.y; s_tl[2 * kWave + l] = T.z;
    s_tl[3 * kWave + l] = L.x; s_tl[4 * kWave + l] = L.y; s_tl[5 * kWave + l] = L.z;
}
RT_D V3 tl_L(const double* s_tl) {
    const uint32_t l = stack_lane();
    return v3(s_tl[3 * kWave + l], s_tl[4 * kWave + l], s_tl[5 * kWave + l]);
}

RT_D void tl_add_L(double* s_tl, V3 e) {  // L = L + T (x) e
    const uint32_t l = stack_lane();
    const V3 T = v3(s_tl[l], s_tl[kWave + l], s_tl[2 * kWave + l]);
    s_tl[3 * kWave + l] = s_tl[3 * kWave + l] + T.x * e.x;
    s_tl[4 * kWave + l] = s_tl[4 * kWave + l] + T.y * e.y;
    s_tl[5 * kWave + l] = s_tl[5 * kWave + l] + T.z * e.z;
}
RT_D void tl_mul_T(double* s_tl, V3 w) {  // T = T (x) w
    const uint32_t l = stack_lane();
    s_tl[l] = s_tl[l] * w.x; s_tl[kWave + l] = s_tl[kWave + l] * w.y; s_tl[2 * kWave + l] = s_tl[2 * kWave + l] * w.z;
}
RT_D void tl_nan_L(double* s_tl) {
    const uint32_t l = stack_lane();
    s_tl[3 * kWave + l] = NAN; s_tl[4 * kWave + l] = NAN; s_tl[5 * kWave + l] = NAN;
}

// One segment of raytrace_impl (raytrace.rs:12-60) in throughput form, from
// the closest-hit result on.  Returns true when the path continues with the
// updated ray.  `last`: this is the path's last segment (raytrace_impl with
// left == 1).
// LT: the path's T and L live in the wave's LDS (s_tl; the 4-wave resumable
// kernel), updated in place; ps.T / ps.L are not used.
template <bool ST, class Stk, bool SLT = false, int KM = 3, bool LT = false>
RT_D bool segment_shade(const DevScene& S, const KParams& P, const Scales& sc, PathState& ps, Rng& rng,
                        Stk& stk, Cnt<ST>& C, bool hit, const Hit& h, uint32_t mat, int32_t gid,
                        int32_t& hit_gid, bool more, bool last, double* s_tl = nullptr) {
    if (!hit) {
        hit_gid = RT_HIT_MISS;
        if (LT) tl_add_L(s_tl, load3(P.bg));
        else ps.L = ps.L + mul(ps.T, load3(P.bg));
        return false;
    }
    hit_gid = gid;
    const DevMaterial& m = S.mats[mat];
    const V3 col = load3(m.color);
    if (LT) tl_add_L(s_tl, load3(m.emission));
    else ps.L = ps.L + mul(ps.T, load3(m.emission));
    // The last segment shades like every other: its direction and pdf decide
    // whether raytrace_impl's last level is NaN (below).  (Stopping after the
    // emission, round 2, was 2.6% faster on C2 but misses that NaN.)
    rng_align(rng);   // shading draws start on a block boundary (oracle.c rng_align)
    rng_top_up(rng);  // every hit lane here: a coherent refill point
    const V3 o = ps.o, d = ps.d;
    if (m.kind == RT_MAT_DIFFUSE) {  // :16-34
        V3 pos = o + d * h.t;
        const bool empty = S.n_lights == 0;
        V3 dir;
        // Mix::sample (ray_sampler.rs:87-93): the coin (when there are lights), then the
        // three draws both samplers share (see "samplers")
        bool by_cosine;
        uint64_t ua, ub, uc;
        diffuse_draws(rng, !empty, by_cosine, ua, ub, uc);
        // both samplers end in normalize(w): one call after the branches join
        V3 sw;
        bool degen = false;
        if (by_cosine) {
            sw = nrm(cube_point(ua, ub, uc)) + h.ns;  // cosine_sample (ray_sampler.rs:69-76)
            const double eps = kEpsilon * 16.0;
            degen = fabs(sw.x) <= eps && fabs(sw.y) <= eps && fabs(sw.z) <= eps;
        } else {
            const unsigned long long ph1 = PH_T();
            sw = light_point<KM>(S, ua, ub, uc, rng, sc) - pos;
            PH_ADDW(kPhLightSample, ph1);
        }
        dir = degen ? h.ns : nrm(sw);
        const double cs = dot(dir, h.ns);
        if (cs <= 0.0) return false;
        if (SLT && more && uni_u32(S.slt_mask)) {
            // the light query's ray is the next segment's: defer the pdf to its box
            // tests.  cosine_pdf = cs / pi here (cs > 0); above 2^-1000 the Mix pdf
            // (cos + light) / 2 cannot be 0, so the path surely continues.
            const double cp = cosine_pdf(h.ns, dir);
            if (cp > 0x1p-1000) {
                ps.pend = true; ps.pcos = cp; ps.pmat = mat;
                ps.o = pos + dir * kEpsilon;
                ps.d = dir;
                return true;
            }
        }
        if (LT) {
            // The light query's ray (pos + dir * eps, dir; ray_sampler.rs:132-139) IS the
            // next segment's: set it first, so the old ray, the hit and the colour are dead
            // while the query runs (the colour is re-read for the weight).
            const double cp = cosine_pdf(h.ns, dir);
            ps.o = pos + dir * kEpsilon;
            ps.d = dir;
            double lp = 0.0;
            bool query = !empty;
            if (KM != kTris && last && query && lq_skippable(S, ps.o)) {  // box lights only
                C.lqskip();
                query = ST;
            }
            if (query) {
                const unsigned long long ph2 = PH_T();
                lp = light_pdf_at<ST, Stk, KM>(S, ps.o, ps.d, stk, C);
                PH_ADDW(kPhLightPdf, ph2);
            }
            const double pdf = empty ? cp : (cp + lp) / 2.0;  // Mix::pdf
            if (pdf == 0.0) return false;
            tl_mul_T(s_tl, diffuse_weight(load3(S.mats[mat].color), cp, pdf));
            if (last && (isnan(cs) || isnan(pdf))) tl_nan_L(s_tl);  // see below
            return true;
        }
        double lp = 0.0;
        // On the path's last bounce only the pdf's NaN-ness is observable (below), and
        // a query whose origin is outside every light's grown world box cannot give
        // NaN (DevScene::lq_boxes): the timed kernel skips it.  The stats instance
        // runs every query, so its counters stay the oracle's, and counts the skips.
        bool query = !empty;
        if (KM != kTris && last && query && lq_skippable(S, pos + dir * kEpsilon)) {  // box lights only
            C.lqskip();
            query = ST;
        }
        if (query) {
            const unsigned long long ph2 = PH_T();
            lp = light_pdf<ST, Stk, KM>(S, pos, dir, stk, C);
            PH_ADDW(kPhLightPdf, ph2);
        }
        const double cp = cosine_pdf(h.ns, dir);
        double pdf = empty ? cp : (cp + lp) / 2.0;  // Mix::pdf
        if (pdf == 0.0) return false;
        ps.T = mul(ps.T, diffuse_weight(col, cp, pdf));
        // The last bounce: raytrace_impl still adds dot * col (x) raytrace_impl(.., 0) / pi
        // / pdf (raytrace.rs:13,32-33), NaN exactly when the direction or the pdf is NaN
        // (a NaN light pdf is reachable: oracle.c raytrace_iter); it reaches the pixel
        // through every enclosing level.  T is not read again, so the rule is explicit.
        if (last && (isnan(cs) || isnan(pdf))) ps.L = v3(NAN, NAN, NAN);
        ps.o = pos + dir * kEpsilon;
        ps.d = dir;
        return true;
    }
    // reflected_ray (raytrace.rs:67-73)
    const V3 rdir = d - (h.ns * 2.0) * dot(h.ns, d);
    const V3 hp = o + d * h.t;
    if (m.kind == RT_MAT_DIELECTRIC) {  // :36-54
        // n1 / n2 and r0 are per-material constants (DevMaterial::k_out, r0)
        const double k = h.inside ? m.ior : m.k_out;
        // refracted_ray (raytrace.rs:75-88)
        const double cos1 = -dot(h.ns, d);
        const double sin2 = k * dev_sqrt(1.0 - cos1 * cos1);
        bool reflect = true;
        if (!(sin2 > 1.0)) {
            const double r0 = m.r0;  // ((n1 - n2) / (n1 + n2)).powi(2)
            const double power = r0 + (1.0 - r0) * powi5(1.0 + dot(d, h.ns));   // reflection_power
            double p = power;
            if (p < 0.0) p = 0.0;
            if (p > 1.0) p = 1.0;
            reflect = gen_bool(rng, p);
            if (!reflect) {
                const double cos2 = dev_sqrt(1.0 - sin2 * sin2);
                const V3 tdir = d * k + h.ns * (k * cos1 - cos2);
                ps.o = hp + tdir * kEpsilon;
                ps.d = tdir;
                if (!h.inside) {
                    if (LT) tl_mul_T(s_tl, col);
                    else ps.T = mul(ps.T, col);
                }
            }
        }
        if (reflect) { ps.o = hp + rdir * kEpsilon; ps.d = rdir; }
        return true;
    }
    // Metallic (:56-58)
    ps.o = hp + rdir * kEpsilon;
    ps.d = rdir;
    if (LT) tl_mul_T(s_tl, col);
    else ps.T = mul(ps.T, col);
    return true;
}

// the resumable form's end of a segment: finish `intersect`, then shade
template <bool ST, int KM = 3, bool CMP = false, bool LT = false, class Stk>
RT_D bool segment_end(const DevScene& S, const KParams& P, const Scales& sc, PathState& ps, Rng& rng,
                      Stk& stk, Cnt<ST>& C, SegQuery& q, int32_t& hit_gid, bool last, double* s_tl) {
    Hit h; uint32_t mat = 0; int32_t gid = 0;
    if (KM == kTris) {  // the candidate is the triangle traversal's (take_tri on an empty best)
        q.best.valid = false; q.best.t = 0.0; q.best.u = q.best.v = 0.0; q.best.prim = 0; q.best.aux = 0;
        q.best.kind = 0;
    }
    take_tri(q.best, q.T.valid, q.T.best, q.T.bu, q.T.bv, q.T.prim);
    const bool hit = intersect_tail<ST, KM>(S, q.best, ps.o, ps.d, C, h, mat, gid);
    return segment_shade<ST, Stk, false, KM, LT>(S, P, sc, ps, rng, stk, C, hit, h, mat, gid, hit_gid, false, last,
                                                 s_tl);
}

// the fused form: one whole segment (scene_intersect to completion, then shade);
// LT as segment_shade's
template <bool ST, int KM = 3, bool LT = false, class Stk>
RT_D bool segment(const DevScene& S, const KParams& P, const Scales& sc, PathState& ps, Rng& rng, Stk& stk,
                  Cnt<ST>& C, int32_t& hit_gid, bool more, double* s_tl = nullptr) {
    Hit h; uint32_t mat; int32_t gid;
    C.segment();
    const unsigned long long ph0 = PH_T();
    double impact = 0.0;
    const bool hit = scene_intersect<ST, Stk, true, KM>(S, ps.o, ps.d, stk, C, h, mat, gid, ps.pend, &impact);
    if (ps.pend) {  // the previous bounce's Mix pdf and weight (raytrace.rs:26-33, ray_sampler.rs:95-97)
        const uint32_t nl = S.n_lights;
        const double lp = nl == 1u ? impact : impact / (double)nl;
        const double pdf = (ps.pcos + lp) / 2.0;
        const V3 w = diffuse_weight(load3(S.mats[ps.pmat].color), ps.pcos, pdf);
        if (LT) tl_mul_T(s_tl, w);
        else ps.T = mul(ps.T, w);
        ps.pend = false;
    }
    PH_ADDW(kPhIntersect, ph0);
    return segment_shade<ST, Stk, true, KM, LT>(S, P, sc, ps, rng, stk, C, hit, h, mat, gid, hit_gid, more, !more,
                                                s_tl);
}

template <bool ST>
RT_D void wave_flush(const Cnt<ST>& C, unsigned long long* stats, uint32_t wave_iters) {
    if (!ST) return;
    uint32_t v[12] = {C.c.paths, C.c.segments, C.c.aabb, C.c.tri, C.c.shape, C.c.shaded, C.c.lq, C.c.lhits,
                      C.c.lq_skip, C.c.kids[0], C.c.kids[1], C.c.kids[2]};
#pragma unroll
    for (int k = 0; k < 12; ++k) {
        const int w = k < 8 ? k : kStatLqSkip + (k - 8);
        unsigned long long x = v[k];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
        if ((threadIdx.x & 63) == 0 && x) atomicAdd(&stats[w], x);
    }
    // lane utilisation: path steps summed over lanes vs 64 x the wave's loop iterations
    unsigned long long s = C.c.steps;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    if ((threadIdx.x & 63) == 0 && wave_iters) {
        atomicAdd(&stats[8], s);
        atomicAdd(&stats[9], 64ull * wave_iters);
    }
}

// Camera::fuzzy_ray + raytrace's normalize (camera.rs:48-55, raytrace.rs:9) for
// a fresh stream: draws exactly the two gen_range(0, 1) of block 0 (value0_1 < 1
// never rejects), so afterwards r is {blk 1, nothing buffered}.
RT_D V3 camera_dir(const KParams& P, uint32_t px, uint32_t py, Rng& r) {
    rng_top_up(r);
    const double fx = (double)px + gen_range(r, 0.0, 1.0);
    const double fy = (double)py + gen_range(r, 0.0, 1.0);
    const double x = (2.0 * fx / P.fw - 1.0) * P.tan_x;
    const double y = -(2.0 * fy / P.fh - 1.0) * P.tan_y;
    const V3 dir = (load3(P.cam_right) * x + load3(P.cam_up) * y) + load3(P.cam_fwd) * 1.0;
    return nrm(dir);
}

// ------------------------------------------------------------ kernels ----
// path_kernel — persistent waves (one 64-lane wave per workgroup, as many as
// fit on the chip) pull wave-tiles from a global queue.  A wave-tile is
// (tile slot, sample chunk, 8x8 quadrant): 64 pixels x chunk_spp samples.
// Inside it the lanes take (sample row, pixel) paths dynamically in row-major
// order — a lane whose path ends starts the next one at once, so lanes do not
// idle while the wave's longest path finishes (rt_stats lane/wave steps).  A
// finished path's radiance goes to a per-wave ring of kRing sample rows; a row
// is committed once all 64 of its paths are done, each lane adding its OWN
// pixel's value — so every pixel is still summed in sample order
// (main.rs:94-104; bit-identical to the sequential sum when chunks == 1).
constexpr int kRing = (int)kRingRows;
constexpr uint32_t kCamSlots = 128;  // precomputed camera rays per wave (two sample rows)

// WAVES = minimum waves per SIMD the register budget must allow (3: 168 VGPRs,
// 4: 128 VGPRs + spill); RES = the resumable segment form (segment_begin /
// suspendable trav_step / segment_end) instead of the fused `segment`; both
// chosen per scene by the host.
//
// The scene and frame constants come by pointer (device memory), and each loop
// trip re-derives the pointers through opaque(): their fields are then
// scalar-loaded where used instead of being hoisted into SGPRs for the whole
// kernel, which (with ~1 KB of them) spilled hundreds of SGPRs into VGPR lanes.
//
// The pointer goes through the asm in the constant address space (the scene
// and frame records are device memory no kernel writes), so the fields are
// s_load'ed through the scalar cache; as a generic pointer they were per-lane
// flat loads, each a full vector-memory round trip.
template <class T>
RT_D const T* opaque(const T* p) {
    const RT_CAS T* q = (const RT_CAS T*)p;
    asm volatile("" : "+s"(q));
    return (const T*)q;
}

// A wave-tile (tile slot, sample chunk, 8x8 quadrant) in frame coordinates.
struct UnitGeo {
    uint32_t qx0, qy0, s0, nrows, oslot;  // quadrant origin, first sample, sample rows, output slot
    uint32_t quad;
    bool tile_ok;
};
RT_D UnitGeo unit_geo(const KParams& P, uint32_t unit) {
    UnitGeo g;
    g.quad = unit & 3u;
    const uint32_t sci = unit >> 2;  // slot * chunks + chunk
    const uint32_t slot = sci / P.chunks, chunk = sci % P.chunks;
    const uint64_t tile = (uint64_t)P.rank + (uint64_t)slot * P.world;
    g.tile_ok = tile < P.n_tiles;
    g.qx0 = (uint32_t)(tile % P.tiles_x) * RT_TILE + (g.quad & 1u) * 8u;
    g.qy0 = (uint32_t)(tile / P.tiles_x) * RT_TILE + (g.quad >> 1) * 8u;
    g.s0 = chunk * P.chunk_spp;
    g.nrows = min(P.spp, g.s0 + P.chunk_spp) - g.s0;
    g.oslot = P.chunks == 1 ? slot : sci;  // out[slot] (means) or part[sci] (chunk sums)
    return g;
}
// The queue's tail (round 5, DESIGN.md §5 "per-launch tail"): the last P.n_tail
// wave-tiles are handed out as P.tail_split parts of consecutive rows each, so the
// waves that take the queue's last entries hold a fraction of a wave-tile when it
// empties.  A part's rows go to the row buffer P.rows ([tail unit][row][lane][3]),
// and tail_combine_kernel sums every tail wave-tile's rows in sample order after the
// launch: the same additions in the same order as one wave's commit, so the frame
// is bit-identical whatever the split (and for any rank count).  Queue entry q:
// q < n_units - n_tail a whole wave-tile, else part (q - first) % split of tail
// wave-tile (q - first) / split.  Returns false for an empty part.
RT_D bool queue_entry(const KParams& P, uint32_t n_units, uint32_t q, UnitGeo& g, uint32_t& tail, uint32_t& roff) {
    const uint32_t first = n_units - P.n_tail;
    if (q < first) { g = unit_geo(P, q); tail = ~0u; roff = 0; return true; }
    const uint32_t j = q - first, t = j / P.tail_split, part = j % P.tail_split;
    g = unit_geo(P, first + t);
    const uint32_t r0 = g.nrows * part / P.tail_split, r1 = g.nrows * (part + 1) / P.tail_split;
    g.s0 += r0;
    g.nrows = r1 - r0;
    tail = t;
    roff = r0;
    return g.nrows > 0;
}
// an open wave-tile's LDS entry: first stream row, qx0 | qy0 << 16, first
// sample, rows, output slot (a tail part: its tail unit), tile_ok | quad << 1
// (| 8 | row offset in its wave-tile << 16 for a tail part)
// Open wave-tiles a wave may hold (s_uq).  A split-tail part may hold a single row,
// so kUQ of them can cover fewer rows than the commit window (kRing); the resumable
// kernel's suspend test therefore counts the queue as able to feed idle lanes only
// while another wave-tile can be opened (can_take) — without that condition an
// RT_RING_ROWS=16 build with kUQ = 8 spun without progress on C5 (round 5).
// 16 entries: 384 B of LDS (the 64-row window with 64 entries pushed the 4-wave
// kernel past 16 waves a CU); 16 whole wave-tiles of >= 8 rows cover the window.
#ifndef RT_OPEN_UNITS
#define RT_OPEN_UNITS 16
#endif
constexpr uint32_t kUQ = RT_OPEN_UNITS, kUW = 6;
constexpr uint32_t kUnitTail = 8u;
RT_D void store_unit(uint32_t* e, uint32_t first, const UnitGeo& g, uint32_t tail = ~0u, uint32_t roff = 0) {
    e[0] = first; e[1] = g.qx0 | (g.qy0 << 16); e[2] = g.s0; e[3] = g.nrows;
    e[4] = tail == ~0u ? g.oslot : tail;
    e[5] = (g.tile_ok ? 1u : 0u) | (g.quad << 1) | (tail == ~0u ? 0u : kUnitTail | (roff << 16));
}
// entry index of the open wave-tile holding stream row `row` (wave-uniform)
RT_D uint32_t unit_of_row(const uint32_t* uq, uint32_t uq_back, uint32_t row) {
    uint32_t i = uq_back - 1u;
    while (uq[(i % kUQ) * kUW] > row) --i;
    return i % kUQ;
}


template <bool ST, bool HIT, int WAVES, bool RES, int KM = 3, bool CMP = false, bool PAIR = false>
__global__ __launch_bounds__(kWave, WAVES) void path_kernel(DevScene Sv, KParams Pv,
                                                     const DevScene* __restrict__ Sg,
                                                     const KParams* __restrict__ Pg, double* __restrict__ out,
                                                     double* __restrict__ part, int32_t* __restrict__ hit_ids,
                                                     unsigned long long* __restrict__ stats, uint32_t* spill_n,
                                                     double* spill_t, uint32_t* __restrict__ queue,
                                                     double* __restrict__ ring_all) {
    // the 4-wave resumable kernel: a shorter LDS stack, and the path's throughput and
    // radiance in LDS (kTL) — they are read only while a lane shades, so they do not
    // occupy registers (or scratch, where the 128-VGPR budget put them) across the
    // triangle traversal
    // (the fused kernel of shape-only scenes at 4-5 waves: T/L in LDS too, and no LDS
    // stack — the shapes' BVH walks push to the global spill stack)
    constexpr bool kW4S = !RES && WAVES >= 4 && KM == kShapes;
    constexpr int kS = (RES && WAVES >= 4) ? kShortRes : (kW4S ? 0 : kShort);
    constexpr bool kTL = (RES && WAVES >= 4) || kW4S;
    __shared__ uint32_t s_n[kS ? kS * kWave : 1];
    __shared__ double s_t[kS ? kS * kWave : 1];
    __shared__ double s_tl[kTL ? 6 * kWave : 1];  // [T.x T.y T.z L.x L.y L.z][lane]
    __shared__ uint32_t s_cnt[kRing];  // finished paths per ring row
    // camera rays of the next kCamSlots paths, [component][slot] (fused kernel only)
    __shared__ double s_cam[RES ? 1 : 3 * kCamSlots];
    __shared__ uint32_t s_uq[kUQ * kUW];  // open wave-tiles (store_unit)
    const uint32_t lane = threadIdx.x;
    auto stk = make_stack<RES, kS>(s_n, s_t, 0u, (uint64_t)blockIdx.x * kWave, spill_n, spill_t,
                                   gridDim.x * kWave);
    double* ring = ring_all + (uint64_t)blockIdx.x * kRing * kWave * 3;
    const KParams& Pt = WAVES == 3 ? *Pg : Pv;  // per-wave-tile constants
    const uint32_t depth = Pt.ray_depth;
    const uint32_t n_units = Pt.n_slots * Pt.chunks * 4u;
    const uint32_t n_queue = n_units + Pt.n_tail * (Pt.tail_split - 1u);  // tail wave-tiles in parts
    Cnt<ST> C;
    C.zero();
#ifdef RT_PHASES
    if (lane < kPhN) g_phase[lane] = 0;
    __syncthreads();
#endif
    // The wave's work is one stream of sample rows: wave-tiles pulled from the
    // queue append their rows to it (s_uq holds the open ones), idle lanes take
    // the next (row, pixel) paths across wave-tile boundaries, and rows commit
    // in stream order, each lane adding its own pixel's radiance; the last row
    // of the oldest open wave-tile writes that tile's sums.  Lanes never wait
    // for a wave-tile's longest path before starting the next one.
    const unsigned long long ph_tile = PH_T();
    // stats instance: the wave's timeline (s_memrealtime, 100 MHz) — start, the trip
    // that found the wave-tile queue drained, exit (raw stats words 52..59, tools/timeline.py)
    const uint64_t tl_start = ST ? wall_clock64() : 0;
    uint64_t tl_drain = 0;
    if (lane < kRing) s_cnt[lane] = 0;
    __syncthreads();
    V3 sum = v3(0.0, 0.0, 0.0);
    uint32_t base = 0, next = 0, witers = 0;  // wave-uniform: next row to commit, next path to hand out
    uint32_t open_end = 0;                    // rows of the wave-tiles pulled so far
    uint32_t uq_front = 0, uq_back = 0;       // open wave-tiles: s_uq entries [uq_front, uq_back)
    bool drained = false;                     // the queue is empty
    uint32_t cam_end = 0;  // camera rays of paths [cam_end - kCamSlots, cam_end) are in s_cam
    bool busy = false;
    uint32_t cur = 0, s = 0, b = 0;
    uint64_t pixel = 0;
    PathState ps;
    Rng rng;
    SegQuery q;
    q.T.live = false;
    bool inq = false;  // this lane's segment query is under way
    uint32_t stall = 0;  // stats instance: consecutive trips without progress (kStatStall)
    for (;;) {
        // fields s_load'ed where used (see opaque), for both register budgets
        // (C3 at 64 spp: 315.6 vs 325.9 ms with the by-value kernel
        // arguments of the 4-wave kernel, whose loads were hoisted into
        // SGPRs and spilled)
        const DevScene& S = *opaque(Sg);
        const KParams& P = *opaque(Pg);
        const Scales sc{P.scale01, P.scale11};
        const uint64_t idle = __ballot(!busy);
        const unsigned long long ph_a = PH_T();
        const uint32_t prog0 = next + base + uq_back + (drained ? 1u : 0u);  // ST: the progress guard
        bool worked = false;  // ST: a traversal step or a shaded segment in this trip
        // pull wave-tiles until the rows the idle lanes could take exist (inside the
        // commit window of kRing rows, at most kUQ open)
        const uint32_t window = (base + kRing) * kWave;
        const uint32_t want = min(window, next + (uint32_t)__popcll(idle));
        while (!drained && open_end * kWave < want && uq_back - uq_front < kUQ) {
            uint32_t u = 0;
            if (lane == 0) u = atomicAdd(queue, 1u);
            const uint32_t unit = __builtin_amdgcn_readfirstlane(u);
            if (unit >= n_queue) {
                drained = true;
                if (ST) tl_drain = wall_clock64();
                break;
            }
            UnitGeo g;
            uint32_t tail, roff;
            if (!queue_entry(Pt, n_units, unit, g, tail, roff)) continue;  // an empty tail part
            if (lane == 0) store_unit(s_uq + (uq_back % kUQ) * kUW, open_end, g, tail, roff);
            open_end += g.nrows;
            ++uq_back;
            __syncthreads();
        }
        const uint32_t limit = min(window, open_end * kWave);
        if (next < limit && idle) {
            if constexpr (!RES) {
                // Camera rays for the paths this trip may hand out, one sample row
                // (64 paths, lane = pixel) at a time with every lane active, instead
                // of per path start with only the idle lanes.  Rows
                // [cam_end - 128, cam_end - 64) are overwritten only once consumed.
                const uint32_t need = min(limit, next + (uint32_t)__popcll(idle));
                while (cam_end < need) {
                    const uint32_t row = cam_end / kWave;
                    const uint32_t* e = s_uq + unit_of_row(s_uq, uq_back, row) * kUW;
                    const uint32_t qxy = e[1];
                    const uint32_t px = (qxy & 0xFFFFu) + (lane & 7u), py = (qxy >> 16) + (lane >> 3);
                    V3 dir = v3(0.0, 0.0, 0.0);
                    if ((e[5] & 1u) && px < P.width && py < P.height) {
                        Rng cr;
                        rng_init(cr, P.seed, (uint64_t)py * P.width + px, e[2] + (row - e[0]));
                        dir = camera_dir(P, px, py, cr);
                    }
                    const uint32_t slot = (cam_end + lane) % kCamSlots;
                    s_cam[slot] = dir.x; s_cam[kCamSlots + slot] = dir.y; s_cam[2 * kCamSlots + slot] = dir.z;
                    cam_end += kWave;
                }
                __syncthreads();
            }
            // idle lanes below this one (v_mbcnt: no lane mask held across the loop)
            const uint32_t k = __builtin_amdgcn_mbcnt_hi((uint32_t)(idle >> 32),
                                                         __builtin_amdgcn_mbcnt_lo((uint32_t)idle, 0u));
            if (!busy && next + k < limit) {
                cur = next + k;
                const uint32_t row = cur / kWave, col = cur % kWave;
                // the row is in the newest open wave-tile or the one before it (a trip
                // hands out at most 64 consecutive paths: two rows)
                const uint32_t eb = (uq_back - 1u) % kUQ;
                const uint32_t* e = s_uq + (row >= s_uq[eb * kUW] ? eb : (uq_back - 2u) % kUQ) * kUW;
                const uint32_t qxy = e[1];
                const uint32_t px = (qxy & 0xFFFFu) + (col & 7u), py = (qxy >> 16) + (col >> 3);
                s = e[2] + (row - e[0]);
                if ((e[5] & 1u) && px < P.width && py < P.height) {
                    // Camera::fuzzy_ray + raytrace (camera.rs:48-55, raytrace.rs:8-10)
                    pixel = (uint64_t)py * P.width + px;
                    rng_init(rng, P.seed, pixel, s);
                    ps.o = load3(P.cam_pos);
                    if constexpr (!RES) {  // precomputed above: block 0 consumed
                        const uint32_t slot = cur % kCamSlots;
                        ps.d = v3(s_cam[slot], s_cam[kCamSlots + slot], s_cam[2 * kCamSlots + slot]);
                        rng.blk = 1;
                    } else {
                        ps.d = camera_dir(P, px, py, rng);
                    }
                    if constexpr (kTL) {
                        tl_store(s_tl, v3(1.0, 1.0, 1.0), v3(0.0, 0.0, 0.0));
                    } else {
                        ps.T = v3(1.0, 1.0, 1.0);
                        ps.L = v3(0.0, 0.0, 0.0);
                    }
                    ps.pend = false;
                    b = 0;
                    busy = true;
                    C.path();
                } else {
                    atomicAdd(&s_cnt[row % kRing], 1u);  // no pixel: done at once, never read
                }
            }
            next = min(limit, next + (uint32_t)__popcll(idle));
        }
        PH_ADD(kPhAssign, ph_a);
#ifdef RT_PHASES
        if (!busy) {  // why this lane has no path this trip
            if (drained && next >= open_end * kWave) PH_LANE(kPhIdleDrain);
            else PH_LANE(kPhIdleWin);
        }
#endif
        bool ends = false;  // this lane's path ends in this trip
        if constexpr (RES) {
            // lanes between segments (new paths, continued paths) start their query
            const unsigned long long ph_b = PH_T();
            if (busy && !inq && b < depth) {
                segment_begin<ST, KM>(S, ps, stk, C, q);
                inq = true;
            }
            PH_ADDW(kPhIntersect, ph_b);
            // Triangle traversal, resumable: step while enough lanes are live; once
            // fewer than P.suspend are, and other lanes wait to shade or to take a new
            // path, suspend the live ones (their stacks and Trav stay put) so the
            // waiting lanes run now and rejoin the traversal with their next rays.
            const unsigned long long ph_t = PH_T();
            for (;;) {
                const uint64_t lv = __ballot(q.T.live);
                if (lv == 0) break;
                if (__popcll(lv) < (int)P.suspend) {
                    const uint32_t win = (base + kRing) * kWave;
                    const bool can_take = next < min(win, open_end * kWave) ||
                                          (!drained && next < win && uq_back - uq_front < kUQ);
                    if (__ballot((busy && !q.T.live) || (!busy && can_take))) break;
                }
                trav_step<3, 2, ST, CMP, PAIR>(S.tris, ps.o, ps.d, q.rc, q.fast, stk, C, q.T, lv, (int)P.leaf_batch);
                if (ST) worked = true;
            }
            PH_ADD(kPhTris, ph_t);
            // lanes whose query finished shade and end (or continue) their segment
            if (busy && !q.T.live) {
                C.step();
                if (ST) worked = true;
                bool cont = false;
                if (inq) {
                    int32_t g;
                    const unsigned long long ph_s = PH_T();
                    if constexpr (kTL) rng_rekey(rng, P.seed);
                    cont = segment_end<ST, KM, CMP, kTL>(S, P, sc, ps, rng, stk, C, q, g, b + 1 >= depth, s_tl);
                    if constexpr (kTL) rng_park(rng);
                    PH_ADDW(kPhSegment, ph_s);
                    if (HIT) hit_ids[(pixel * P.spp + s) * depth + b] = g;
                    ++b;
                    inq = false;
                }
                ends = !cont || b >= depth;
            }
        } else if (busy) {  // fused: one whole segment of every live path
            C.step();
            if (ST) worked = true;
            bool cont = false;
            if (b < depth) {
                int32_t g;
                const unsigned long long ph_s = PH_T();
                if constexpr (kTL) rng_rekey(rng, P.seed);
                cont = segment<ST, KM, kTL>(S, P, sc, ps, rng, stk, C, g, b + 1 < depth, s_tl);
                if constexpr (kTL) rng_park(rng);
                PH_ADDW(kPhSegment, ph_s);
                if (HIT) hit_ids[(pixel * P.spp + s) * depth + b] = g;
                ++b;
            }
            ends = !cont || b >= depth;
        }
        if (ends) {
            if (HIT) for (uint32_t k = b; k < depth; ++k) hit_ids[(pixel * P.spp + s) * depth + k] = RT_HIT_NONE;
            const uint32_t r = (cur / kWave) % kRing;
            double* rp = ring + ((uint64_t)r * kWave + cur % kWave) * 3;
            if constexpr (kTL) ps.L = tl_L(s_tl);
            rp[0] = ps.L.x; rp[1] = ps.L.y; rp[2] = ps.L.z;
            atomicAdd(&s_cnt[r], 1u);
            busy = false;
        }
        ++witers;
        // commit complete rows in stream order (ring stores visible to the wave);
        // the last row of the oldest open wave-tile writes its per-pixel sums
        const unsigned long long ph_c = PH_T();
        __syncthreads();
        while (base < open_end && s_cnt[base % kRing] == (uint32_t)kWave) {
            const double* rp = ring + ((uint64_t)(base % kRing) * kWave + lane) * 3;
            const uint32_t* e = s_uq + (uq_front % kUQ) * kUW;
            if (e[5] & kUnitTail) {  // a tail part: the row to the row buffer (tail_combine_kernel sums)
                double* w = Pt.rows + (((uint64_t)e[4] * Pt.chunk_spp + (e[5] >> 16) + (base - e[0])) * kWave + lane) * 3;
                w[0] = rp[0]; w[1] = rp[1]; w[2] = rp[2];
            } else {
                sum = sum + v3(rp[0], rp[1], rp[2]);
            }
            __syncthreads();
            if (lane == 0) s_cnt[base % kRing] = 0;
            __syncthreads();
            if (base + 1u == e[0] + e[3] && (e[5] & kUnitTail)) {
                ++uq_front;
            } else if (base + 1u == e[0] + e[3]) {  // main.rs:104 for this wave-tile's pixels
                const uint32_t qxy = e[1], quad = e[5] >> 1;
                const uint32_t lx = (quad & 1u) * 8u + (lane & 7u), ly = (quad >> 1) * 8u + (lane >> 3);
                const bool own = (e[5] & 1u) && (qxy & 0xFFFFu) + (lane & 7u) < Pt.width &&
                                 (qxy >> 16) + (lane >> 3) < Pt.height;
                const V3 res = own ? (Pt.chunks == 1 ? sum / (double)Pt.spp : sum) : v3(0.0, 0.0, 0.0);
                double* o = (Pt.chunks == 1 ? out : part) + ((uint64_t)e[4] * kBlock + ly * RT_TILE + lx) * 3;
                o[0] = res.x; o[1] = res.y; o[2] = res.z;
                sum = v3(0.0, 0.0, 0.0);
                ++uq_front;
            }
            ++base;
        }
        PH_ADD(kPhCommit, ph_c);
        if (drained && uq_front == uq_back) break;  // every pulled wave-tile written
        if constexpr (ST) {
            // Progress guard (render.h kStatStall): a trip that pulls, hands out, steps,
            // shades or commits nothing can only repeat itself — flag the wave and exit.
            const bool moved = __ballot(worked) != 0 || next + base + uq_back + (drained ? 1u : 0u) != prog0;
            stall = moved ? 0u : stall + 1u;
            if (stall >= kStallTrips) {
                if (lane == 0) atomicAdd(&stats[kStatStall], 1ull);
                break;
            }
        }
    }
    wave_flush<ST>(C, stats, witers);
    if (ST && lane == 0) {
        const uint64_t te = wall_clock64(), td = tl_drain ? tl_drain : te;
        atomicMax(&stats[kTimeline + 0], ~(unsigned long long)tl_start);  // ~ : earliest start
        atomicMax(&stats[kTimeline + 1], (unsigned long long)te);         // last exit
        atomicMax(&stats[kTimeline + 2], ~(unsigned long long)td);        // earliest drain
        atomicMax(&stats[kTimeline + 3], (unsigned long long)td);         // last drain
        atomicAdd(&stats[kTimeline + 4], (unsigned long long)(te - td));  // sum of drain-to-exit
        atomicMax(&stats[kTimeline + 5], (unsigned long long)(te - td));
        atomicAdd(&stats[kTimeline + 6], (unsigned long long)(te - tl_start));
        atomicAdd(&stats[kTimeline + 7], 1ull);
    }
    PH_ADD(kPhTile, ph_tile);
#ifdef RT_PHASES
    if (ST && lane < kPhN) atomicAdd(&stats[kPhaseWord0 + lane], g_phase[lane]);
#endif
}

// trace_kernel — batch `intersect` (intersections.rs:42-62) as a persistent
// traversal: each wave keeps its lanes busy by fetching the next rays from a
// global counter as soon as enough lanes have finished (kRefill), so a wave
// never waits for its slowest ray.  Per ray the steps are those of
// scene_intersect (shapes to completion, then the resumable triangle traversal
// in the reference order), so the hits are identical to intersect_kernel's.
constexpr int kRefill = 16;
RT_D void write_hit(rt_hit* __restrict__ out, uint32_t i, bool ok, const Hit& h, int32_t gid) {
    rt_hit r;
    if (ok) {
        r.t = h.t; store3(r.geometry_normal, h.ng); store3(r.shading_normal, h.ns);
        r.inside = h.inside ? 1 : 0; r.prim = gid;
    } else {
        r.t = 0.0; store3(r.geometry_normal, v3(0, 0, 0)); store3(r.shading_normal, v3(0, 0, 0));
        r.inside = 0; r.prim = RT_HIT_MISS;
    }
    out[i] = r;
}

// CMP: the triangle BVH's compact layout, PAIR: its pair lines (trav_step)
template <int WAVES, bool CMP = false, bool PAIR = false>
__global__ __launch_bounds__(kWave, WAVES) void trace_kernel(DevScene S, const double* __restrict__ rays,
                                                             uint32_t n, rt_hit* __restrict__ out,
                                                             uint32_t* __restrict__ queue, uint32_t* spill_n,
                                                             double* spill_t) {
    __shared__ uint32_t s_n[kShort * kWave];
    __shared__ double s_t[kShort * kWave];
    auto stk = make_stack<true>(s_n, s_t, 0u, (uint64_t)blockIdx.x * kWave, spill_n, spill_t, gridDim.x * kWave);
    Cnt<false> C;
    const uint64_t below = (1ull << threadIdx.x) - 1ull;
    bool has = false, drained = false;  // drained: wave-uniform
    uint32_t idx = 0;
    PathState ps;
    SegQuery q;
    q.T.live = false;
    for (;;) {
        const uint64_t idle = __ballot(!has);
        const uint64_t lv = __ballot(q.T.live);
        if (!drained && idle && (__popcll(idle) >= kRefill || lv == 0)) {
            uint32_t b = 0;
            if (threadIdx.x == 0) b = atomicAdd(queue, (uint32_t)__popcll(idle));
            const uint32_t base = __builtin_amdgcn_readfirstlane(b);
            if ((uint64_t)base + (uint64_t)__popcll(idle) >= n) drained = true;
            if (!has) {
                const uint32_t k = base + (uint32_t)__popcll(idle & below);
                if (k < n) {
                    idx = k;
                    ps.o = load3(rays + 6 * (size_t)k);
                    ps.d = load3(rays + 6 * (size_t)k + 3);
                    segment_begin<false>(S, ps, stk, C, q);
                    has = true;
                }
            }
        }
        const uint64_t lv2 = __ballot(q.T.live);
        if (lv2) trav_step<3, 2, false, CMP, PAIR>(S.tris, ps.o, ps.d, q.rc, q.fast, stk, C, q.T, lv2);
        if (has && !q.T.live) {
            Hit h; uint32_t mat = 0; int32_t gid = 0;
            take_tri(q.best, q.T.valid, q.T.best, q.T.bu, q.T.bv, q.T.prim);
            const bool ok = intersect_tail<false>(S, q.best, ps.o, ps.d, C, h, mat, gid);
            write_hit(out, idx, ok, h, gid);
            has = false;
        }
        if (drained && !__ballot(has)) break;
    }
}

__global__ __launch_bounds__(kBlock) void intersect_kernel(DevScene S, const double* __restrict__ rays, uint32_t n,
                                                           rt_hit* __restrict__ out, uint32_t* spill_n,
                                                           double* spill_t) {
    __shared__ uint32_t s_n[kShort * kBlock];
    __shared__ double s_t[kShort * kBlock];
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const uint32_t wtid = __builtin_amdgcn_readfirstlane(threadIdx.x) & ~(uint32_t)(kWave - 1);
    auto stk = make_stack(s_n, s_t, wtid, (uint64_t)blockIdx.x * kBlock + wtid, spill_n, spill_t, gridDim.x * kBlock);
    Cnt<false> C;
    Hit h; uint32_t mat; int32_t gid;
    V3 o = load3(rays + 6 * (size_t)i), d = load3(rays + 6 * (size_t)i + 3);
    rt_hit r;
    if (scene_intersect<false>(S, o, d, stk, C, h, mat, gid)) {
        r.t = h.t; store3(r.geometry_normal, h.ng); store3(r.shading_normal, h.ns);
        r.inside = h.inside ? 1 : 0; r.prim = gid;
    } else {
        r.t = 0.0; store3(r.geometry_normal, v3(0, 0, 0)); store3(r.shading_normal, v3(0, 0, 0));
        r.inside = 0; r.prim = RT_HIT_MISS;
    }
    out[i] = r;
}

// mode 0: raw intersect_lights impact sum + hit count; mode 1: Light::pdf
__global__ __launch_bounds__(kBlock) void light_kernel(DevScene S, const double* __restrict__ rays, uint32_t n,
                                                       int mode, double* __restrict__ out, uint32_t* __restrict__ cnt,
                                                       uint32_t* spill_n, double* spill_t) {
    __shared__ uint32_t s_n[kShort * kBlock];
    __shared__ double s_t[kShort * kBlock];
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const uint32_t wtid = __builtin_amdgcn_readfirstlane(threadIdx.x) & ~(uint32_t)(kWave - 1);
    auto stk = make_stack(s_n, s_t, wtid, (uint64_t)blockIdx.x * kBlock + wtid, spill_n, spill_t, gridDim.x * kBlock);
    Cnt<false> C;
    V3 o = load3(rays + 6 * (size_t)i), d = load3(rays + 6 * (size_t)i + 3);
    uint32_t nh = 0;
    double v;
    if (mode == 0) v = lights_impact<false>(S, o, d, stk, C, nh);
    else v = S.n_lights == 0 ? 0.0 : light_pdf<false>(S, o, d, stk, C);
    out[i] = v;
    if (cnt) cnt[i] = nh;
}

__global__ void unpack_kernel(const double* __restrict__ g, double* __restrict__ img, uint32_t W, uint32_t H,
                              uint32_t tiles_x, uint32_t world, uint32_t per_rank) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (uint64_t)W * H) return;
    const uint32_t x = (uint32_t)(i % W), y = (uint32_t)(i / W);
    const uint64_t tile = (uint64_t)(y / RT_TILE) * tiles_x + x / RT_TILE;
    const uint64_t rank = tile % world, slot = tile / world;
    const double* src = g + (((rank * per_rank + slot) * kBlock) + (y % RT_TILE) * RT_TILE + (x % RT_TILE)) * 3;
    img[3 * i] = src[0]; img[3 * i + 1] = src[1]; img[3 * i + 2] = src[2];
}

__global__ void ell_rcp_kernel(DevShape* __restrict__ s, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    for (int k = 0; k < 3; ++k) s[i].aux[k] = dev_rcp(s[i].shape[k]);
}
hipError_t launch_ell_rcp(DevShape* shapes, uint32_t n, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(ell_rcp_kernel, dim3((n + 255) / 256), dim3(256), 0, st, shapes, n);
    return hipGetLastError();
}

__global__ void fp64_probe_kernel(const double* a, const double* b, double* out, uint32_t n, int op) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[i] = op == 0 ? sqrt(a[i])
           : op == 1 ? a[i] / b[i]
           : op == 2 ? dev_quot(a[i], b[i], dev_rcp(b[i]))
           : op == 3 ? dev_sqrt(a[i])
           : op == 4 ? dev_inv_len(a[i]) : dev_quotf(a[i], b[i], dev_rcp(b[i]));
}

// ------------------------------------------------------------- launch ----
// Persistent grid: the number of path-kernel waves resident on the device at
// once (occupancy x CUs), capped by the number of wave-tiles.  Extra waves
// would only find the queue drained.
namespace {
using PathFn = void (*)(DevScene, KParams, const DevScene*, const KParams*, double*, double*, int32_t*,
                        unsigned long long*, uint32_t*, double*, uint32_t*, double*);
// kinds (kShapes | kTris): one-kind instances of the two kernels the host picks
// by default — the 4-wave resumable kernel for triangle-only scenes (every glTF
// scene) and the 3-wave fused kernel for shape-only scenes (the Cornell box)
template <bool ST, bool HIT>
PathFn path_fn_r(uint32_t waves, bool resume, int kinds) {
#ifdef RT_ONLY_C2  // experiment builds (tools/variants.py): only the C2 instances, 4x faster to compile
    (void)waves; (void)resume;
#ifdef RT_C2_W  // experiment: the shape-only fused kernel at RT_C2_W waves/SIMD
    return kinds == kShapes ? path_kernel<ST, HIT, RT_C2_W, false, kShapes> : path_kernel<ST, HIT, 3, false>;
#else
    return kinds == kShapes ? path_kernel<ST, HIT, 3, false, kShapes> : path_kernel<ST, HIT, 3, false>;
#endif
#elif defined(RT_ONLY_C3)  // ... only the C3 instances
    (void)waves; (void)resume;
#ifdef RT_C3_W  // experiment: the compact triangle-only kernel at RT_C3_W waves/SIMD
    if (kinds == kKindsCompact) return path_kernel<ST, HIT, RT_C3_W, true, kTris, true>;
#else
    if (kinds == kKindsCompact) return path_kernel<ST, HIT, 4, true, kTris, true>;
#endif
    if (kinds == kKindsPair) return path_kernel<ST, HIT, 4, true, kTris, true, true>;
    return kinds == kTris ? path_kernel<ST, HIT, 4, true, kTris> : path_kernel<ST, HIT, 4, true>;
#else
    if (waves == 4 && resume) {
        if (kinds == kKindsCompact) return path_kernel<ST, HIT, 4, true, kTris, true>;  // compact triangle layout
        if (kinds == kKindsPair) return path_kernel<ST, HIT, 4, true, kTris, true, true>;  // + pair layout
        return kinds == kTris ? path_kernel<ST, HIT, 4, true, kTris> : path_kernel<ST, HIT, 4, true>;
    }
    kinds &= 3;  // the compact layout has only the triangle-only resumable instance (host: path_kinds)
    if (waves == 5 && !resume && kinds == kShapes) return path_kernel<ST, HIT, 5, false, kShapes>;  // api.cpp path_waves
    if (waves == 4) return kinds == kShapes ? path_kernel<ST, HIT, 4, false, kShapes> : path_kernel<ST, HIT, 4, false>;
    if (resume) return path_kernel<ST, HIT, 3, true>;
    return kinds == kShapes ? path_kernel<ST, HIT, 3, false, kShapes> : path_kernel<ST, HIT, 3, false>;
#endif
}
PathFn path_fn(bool stats, bool hits, uint32_t waves, bool resume, int kinds) {
    if (stats) return hits ? path_fn_r<true, true>(waves, resume, kinds) : path_fn_r<true, false>(waves, resume, kinds);
    return hits ? path_fn_r<false, true>(waves, resume, kinds) : path_fn_r<false, false>(waves, resume, kinds);
}
}  // namespace

hipError_t path_grid(bool stats, bool hits, uint32_t waves, bool resume, int kinds, uint32_t n_units,
                     uint32_t* grid) {
    int dev = 0, cus = 0, per_cu = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (e != hipSuccess) return e;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)path_fn(stats, hits, waves, resume, kinds),
                                                     kWave, 0);
    if (e != hipSuccess) return e;
    const uint64_t g = (uint64_t)std::max(per_cu, 1) * (uint64_t)std::max(cus, 1);
    *grid = (uint32_t)std::min<uint64_t>(g, std::max<uint32_t>(n_units, 1u));
    return hipSuccess;
}

__global__ void stage_params_kernel(KParams* dst, KParams P) { *dst = P; }
__global__ void tail_combine_kernel(KParams P, uint32_t n_units, double* __restrict__ out, double* __restrict__ part);

hipError_t launch_path(const DevScene& S, const KParams& P, const PathWork& W, double* out, int32_t* hit_ids,
                       unsigned long long* stats, hipStream_t st) {
    if (P.chunks == 0 || (P.chunks > 1 && !W.part) || !W.queue || !W.ring || W.grid == 0) return hipErrorInvalidValue;
    if (W.waves < 3 || W.waves > 5 || (W.waves == 5 && (W.resume || W.kinds != kShapes))) return hipErrorInvalidValue;
    hipError_t e = hipMemsetAsync(W.queue, 0, kQueueWords * sizeof(uint32_t), st);
    if (e != hipSuccess) return e;
    // the stats instance's wave timeline (words kTimeline..+7) describes ONE launch: it
    // is cleared here, while the counters accumulate until rt_read_stats resets them
    if (stats && (e = hipMemsetAsync(stats + kTimeline, 0, 8 * sizeof(unsigned long long), st)) != hipSuccess)
        return e;
    // the frame constants travel by pointer (see opaque): stage them in the scene's
    // slot, stream-ordered (the by-value argument is captured at launch)
    hipLaunchKernelGGL(stage_params_kernel, dim3(1), dim3(1), 0, st, W.d_params, P);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(path_fn(stats != nullptr, hit_ids != nullptr, W.waves, W.resume, W.kinds), dim3(W.grid),
                       dim3(kWave), 0, st,
                       S, P, W.d_scene, W.d_params, out, W.part, hit_ids, stats, W.spill_n, W.spill_t, W.queue, W.ring);
    e = hipGetLastError();
    if (e == hipSuccess && P.n_tail) {
        hipLaunchKernelGGL(tail_combine_kernel, dim3((P.n_tail + 3) / 4), dim3(4 * kWave), 0, st, P,
                           P.n_slots * P.chunks * 4u, out, W.part);
        e = hipGetLastError();
    }
    if (e != hipSuccess || P.chunks == 1) return e;
    return launch_reduce_chunks(W.part, out, P, st);
}

// Content checksum of a device array (rt_scene_checksum; multi.cpp checks every
// replica against devices[0]'s after the fill): word i (8 B, little-endian, the last
// one zero-padded) contributes splitmix64(w + i * golden) to a 64-bit sum — order-free,
// so the atomics keep it deterministic, and a word moved, changed or missing shows.
RT_D uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
__global__ void checksum_kernel(const uint8_t* __restrict__ p, uint64_t bytes, unsigned long long* __restrict__ out) {
    const uint64_t words = (bytes + 7) / 8, full = bytes / 8;
    const uint64_t* w = (const uint64_t*)p;
    uint64_t h = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t v = 0;
        if (i < full) v = w[i];
        else for (uint64_t b = 8 * i; b < bytes; ++b) v |= (uint64_t)p[b] << (8 * (b - 8 * i));
        h += mix64(v + i * 0x9e3779b97f4a7c15ull);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) h += __shfl_xor(h, off, 64);
    if ((threadIdx.x & 63) == 0 && h) atomicAdd(out, (unsigned long long)h);
}
hipError_t launch_checksum(const void* p, uint64_t bytes, unsigned long long* d_out, hipStream_t st) {
    hipError_t e = hipMemsetAsync(d_out, 0, sizeof(*d_out), st);
    if (e != hipSuccess || bytes == 0) return e;
    const uint64_t words = (bytes + 7) / 8;
    const uint32_t blocks = (uint32_t)std::min<uint64_t>(2048, (words + kBlock - 1) / kBlock);
    hipLaunchKernelGGL(checksum_kernel, dim3(blocks), dim3(kBlock), 0, st, (const uint8_t*)p, bytes, d_out);
    return hipGetLastError();
}

// The queue's tail wave-tiles (queue_entry): each pixel's rows summed in sample order
// from v3(0) — path_kernel's commit, addition for addition — and written where that
// commit writes (means when chunks == 1, else the chunk partial).
__global__ void tail_combine_kernel(KParams P, uint32_t n_units, double* __restrict__ out, double* __restrict__ part) {
    const uint32_t lane = threadIdx.x & (kWave - 1), t = blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave;
    if (t >= P.n_tail) return;
    const UnitGeo g = unit_geo(P, n_units - P.n_tail + t);
    const double* r = P.rows + ((uint64_t)t * P.chunk_spp * kWave + lane) * 3;
    V3 sum = v3(0.0, 0.0, 0.0);
    for (uint32_t k = 0; k < g.nrows; ++k) sum = sum + v3(r[(uint64_t)k * kWave * 3], r[(uint64_t)k * kWave * 3 + 1],
                                                          r[(uint64_t)k * kWave * 3 + 2]);
    const uint32_t lx = (g.quad & 1u) * 8u + (lane & 7u), ly = (g.quad >> 1) * 8u + (lane >> 3);
    const bool own = g.tile_ok && g.qx0 + (lane & 7u) < P.width && g.qy0 + (lane >> 3) < P.height;
    const V3 res = own ? (P.chunks == 1 ? sum / (double)P.spp : sum) : v3(0.0, 0.0, 0.0);
    double* o = (P.chunks == 1 ? out : part) + ((uint64_t)g.oslot * kBlock + ly * RT_TILE + lx) * 3;
    o[0] = res.x; o[1] = res.y; o[2] = res.z;
}

// Chunk partial sums -> per-pixel mean: ((p0 + p1) + ... + pK-1) / spp, in
// chunk order (the oracle's chunked iterative form sums identically).
__global__ void reduce_chunks_kernel(const double* __restrict__ part, double* __restrict__ out, uint32_t n_slots,
                                     uint32_t chunks, double spp) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;  // (slot, pixel-in-tile, channel)
    if (i >= (uint64_t)n_slots * kBlock * 3) return;
    const uint64_t slot = i / (kBlock * 3), rem = i % (kBlock * 3);
    const double* p = part + slot * chunks * (kBlock * 3) + rem;
    double s = p[0];
    for (uint32_t k = 1; k < chunks; ++k) s = s + p[(uint64_t)k * kBlock * 3];
    out[i] = s / spp;
}

hipError_t launch_reduce_chunks(const double* part, double* out, const KParams& P, hipStream_t st) {
    const uint64_t n = (uint64_t)P.n_slots * kBlock * 3;
    hipLaunchKernelGGL(reduce_chunks_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, part, out,
                       P.n_slots, P.chunks, (double)P.spp);
    return hipGetLastError();
}
hipError_t launch_intersect(const DevScene& S, const double* rays, uint32_t n, rt_hit* out, uint32_t* spill_n,
                            double* spill_t, hipStream_t st) {
    uint32_t blocks = (n + kBlock - 1) / kBlock;
    hipLaunchKernelGGL(intersect_kernel, dim3(blocks), dim3(kBlock), 0, st, S, rays, n, out, spill_n, spill_t);
    return hipGetLastError();
}
// persistent batch intersect (trace_kernel): grid = resident waves, capped by the rays
hipError_t launch_trace(const DevScene& S, const double* rays, uint32_t n, rt_hit* out, uint32_t* queue,
                        uint32_t* spill_n, double* spill_t, uint32_t grid, int compact, hipStream_t st) {
    hipError_t e = hipMemsetAsync(queue, 0, kQueueWords * sizeof(uint32_t), st);
    if (e != hipSuccess) return e;
    if (compact == 2 && S.tris.pnodes)
        hipLaunchKernelGGL((trace_kernel<4, true, true>), dim3(grid), dim3(kWave), 0, st, S, rays, n, out, queue,
                           spill_n, spill_t);
    else if (compact && S.tris.cnodes)
        hipLaunchKernelGGL((trace_kernel<4, true>), dim3(grid), dim3(kWave), 0, st, S, rays, n, out, queue, spill_n,
                           spill_t);
    else
        hipLaunchKernelGGL(trace_kernel<4>, dim3(grid), dim3(kWave), 0, st, S, rays, n, out, queue, spill_n, spill_t);
    return hipGetLastError();
}
#ifdef RT_WF_PROBE
// Experiment (variant builds only): a traversal-only persistent kernel for a
// triangle-only scene on the compact layout — the trace half of a wavefront form.
// It carries only the ray, its reciprocals and the traversal state, so it may run
// more waves per SIMD (kWfWaves) with a KS-entry LDS stack.  Writes t and the
// global id of the closest triangle (rt_hit.t / .prim; the normals are not filled).
constexpr int kWfWaves = 6;
constexpr int kWfKS = 8;
template <int WAVES, int KS>
__global__ __launch_bounds__(kWave, WAVES) void trace_tri_kernel(DevScene S, const double* __restrict__ rays,
                                                                 uint32_t n, rt_hit* __restrict__ out,
                                                                 uint32_t* __restrict__ queue, uint32_t* spill_n,
                                                                 double* spill_t) {
    __shared__ uint32_t s_n[KS * kWave];
    __shared__ double s_t[KS * kWave];
    auto stk = make_stack<true, KS>(s_n, s_t, 0u, (uint64_t)blockIdx.x * kWave, spill_n, spill_t, gridDim.x * kWave);
    Cnt<false> C;
    const uint64_t below = (1ull << threadIdx.x) - 1ull;
    bool has = false, drained = false;
    uint32_t idx = 0;
    V3 o = v3(0, 0, 0), d = v3(0, 0, 0);
    Rcp3 rc;
    bool fast = false;
    Trav T;
    T.live = false;
    for (;;) {
        const uint64_t idle = __ballot(!has);
        const uint64_t lv = __ballot(T.live);
        if (!drained && idle && (__popcll(idle) >= kRefill || lv == 0)) {
            uint32_t b = 0;
            if (threadIdx.x == 0) b = atomicAdd(queue, (uint32_t)__popcll(idle));
            const uint32_t base = __builtin_amdgcn_readfirstlane(b);
            if ((uint64_t)base + (uint64_t)__popcll(idle) >= n) drained = true;
            if (!has) {
                const uint32_t k = base + (uint32_t)__popcll(idle & below);
                if (k < n) {
                    idx = k;
                    o = load3(rays + 6 * (size_t)k);
                    d = load3(rays + 6 * (size_t)k + 3);
                    rc = make_rcp3(d);
                    fast = S.tris.fast && ray_fast(o, rc);
                    trav_init<2, false>(S.tris, o, d, rc, fast, stk, C, T);
                    has = true;
                }
            }
        }
        const uint64_t lv2 = __ballot(T.live);
        if (lv2) trav_step<3, 2, false, true>(S.tris, o, d, rc, fast, stk, C, T, lv2, 32);
        if (has && !T.live) {
            rt_hit* r = out + idx;
            r->t = T.valid ? T.best : 0.0;
            r->prim = T.valid ? S.tris.gid[T.prim] : RT_HIT_MISS;
            has = false;
        }
        if (drained && !__ballot(has)) break;
    }
}
hipError_t launch_trace_tri(const DevScene& S, const double* rays, uint32_t n, rt_hit* out, uint32_t* queue,
                            uint32_t* spill_n, double* spill_t, uint32_t grid, hipStream_t st) {
    hipError_t e = hipMemsetAsync(queue, 0, kQueueWords * sizeof(uint32_t), st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((trace_tri_kernel<kWfWaves, kWfKS>), dim3(grid), dim3(kWave), 0, st, S, rays, n, out, queue,
                       spill_n, spill_t);
    return hipGetLastError();
}
hipError_t trace_tri_grid(uint32_t n, uint32_t* grid) {
    int dev = 0, cus = 0, per_cu = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (e == hipSuccess)
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)trace_tri_kernel<kWfWaves, kWfKS>,
                                                         kWave, 0);
    if (e != hipSuccess) return e;
    const uint64_t g = (uint64_t)std::max(per_cu, 1) * (uint64_t)std::max(cus, 1);
    *grid = (uint32_t)std::min<uint64_t>(g, std::max<uint64_t>(((uint64_t)n + kWave - 1) / kWave, 1));
    return hipSuccess;
}
#endif
hipError_t trace_grid(uint32_t n, uint32_t* grid) {
    int dev = 0, cus = 0, per_cu = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (e == hipSuccess) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)trace_kernel<4>, kWave, 0);
    if (e != hipSuccess) return e;
    const uint64_t g = (uint64_t)std::max(per_cu, 1) * (uint64_t)std::max(cus, 1);
    *grid = (uint32_t)std::min<uint64_t>(g, std::max<uint64_t>(((uint64_t)n + kWave - 1) / kWave, 1));
    return hipSuccess;
}
hipError_t launch_light(const DevScene& S, const double* rays, uint32_t n, int mode, double* out, uint32_t* cnt,
                        uint32_t* spill_n, double* spill_t, hipStream_t st) {
    uint32_t blocks = (n + kBlock - 1) / kBlock;
    hipLaunchKernelGGL(light_kernel, dim3(blocks), dim3(kBlock), 0, st, S, rays, n, mode, out, cnt, spill_n, spill_t);
    return hipGetLastError();
}
hipError_t launch_unpack(const double* g, double* img, uint32_t W, uint32_t H, uint32_t tiles_x, uint32_t world,
                         uint32_t per_rank, hipStream_t st) {
    uint64_t n = (uint64_t)W * H;
    hipLaunchKernelGGL(unpack_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, g, img, W, H, tiles_x,
                       world, per_rank);
    return hipGetLastError();
}
hipError_t launch_fp64_probe(const double* a, const double* b, double* out, uint32_t n, int op, hipStream_t st) {
    hipLaunchKernelGGL(fp64_probe_kernel, dim3((n + 255) / 256), dim3(256), 0, st, a, b, out, n, op);
    return hipGetLastError();
}

}  // namespace rt
