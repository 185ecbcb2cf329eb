// rt_device.h — device-side building blocks of the path tracer (gfx950).
//
// Everything here restates the reference's per-ray arithmetic in f64 with the
// reference's operation order so that, on the same Philox stream, the device
// produces bit-identical hit ids and radiance to the oracle's iterative form
// (oracle/oracle.c raytrace_iter).  Cited reference lines are in
// /root/reference/src.
#pragma once
#include <hip/hip_runtime.h>

#include "phases.h"
#include "rt_layout.h"
#include "rt_math.h"

namespace rt {

#define RT_D __device__ __forceinline__

// Wave-uniform scene data in the scalar path.  The scene's fields reach the
// kernels through generic pointers, so the compiler reads them with per-lane
// flat loads (a flat load may hit scratch, so its result counts as divergent)
// and every dependent access waits a full vector-memory round trip.  A POINTER
// VALUE read from the scene (device global memory no kernel writes) is made
// uniform with readfirstlane and viewed in the constant address space: loads
// through it with a uniform index become s_load through the scalar cache.
// Only for values every active lane holds (scene pointers and counts).
#ifdef __HIP_DEVICE_COMPILE__  // the host pass of a .hip file only parses these
#define RT_CAS __attribute__((address_space(4)))
#else
#define RT_CAS
#endif
template <class T>
RT_D const RT_CAS T* uni(const T* p) {
    const uint64_t v = (uint64_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return (const RT_CAS T*)(((uint64_t)hi << 32) | lo);
}
RT_D uint32_t uni_u32(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// ------------------------------------------------------------------ RNG ----
// Counter-based Philox4x32-10 per (pixel, sample) replaces ThreadRng
// (main.rs:95); ctr = {block, sample, pixel_lo, pixel_hi}, key = seed.
// Words are consumed in order; next_u64 = lo word | hi word << 32 (rand
// BlockRng order).  The 4-word block lives in two u64 "queues" so no
// dynamically indexed register array (which would go to scratch).
//
// Refills are where divergence bites: lanes sit at different offsets of their
// block, so a refill inside every draw would run Philox at nearly every call
// site for a handful of lanes.  So the NEXT block is generated ahead at a few
// coherent points (rng_top_up: path start, each hit, before the diffuse
// sampler) and a draw that empties the current block only swaps it in.  The
// word stream is unchanged — blocks are still produced and consumed in counter
// order; only when they are computed moves.  At each hit the rest of the
// current block is skipped (rng_align), so the blocks of one shading step line
// up across lanes.
struct Rng {
    uint32_t sample, pix_lo, pix_hi, k0, k1;
    uint32_t blk;       // counter of the next block to generate
    uint32_t avail;     // words left in q0/q1 (current block)
    uint32_t nready;    // n0/n1 holds block blk-1, not yet current
    uint64_t q0, q1;    // current block
    uint64_t n0, n1;    // next block
};

// a ^ b ^ k in one gfx950 v_bitop3_b32 (truth table 0x96): the compiler emits two
// v_xor_b32 for the chain, so a Philox round is 4 VALU instead of 6 (C2 -2.8%, C3
// -0.5% at reduced spp, same digests; profiles/r04/variants_xor3_C*.log).  k is the
// round key — the frame seed plus a round constant — and MUST be wave-uniform: it is
// the instruction's SGPR operand.  The readfirstlane states that (a per-lane key
// would otherwise be read from the first active lane without notice); every key
// comes from the frame's seed (rng_init / rng_rekey from KParams::seed), so it is
// the value every lane holds, and the "s" constraint needs the same readfirstlane.
RT_D uint32_t xor3(uint32_t a, uint32_t b, uint32_t k) {
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "s"(__builtin_amdgcn_readfirstlane(k)));
    return r;
}
RT_D void philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1,
                 uint64_t& q0, uint64_t& q1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
        // one 32x32->64 product per multiplier (v_mad_u64_u32) instead of mul_hi + mul_lo
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        uint32_t n0 = xor3(hi1, c1, k0), n2 = xor3(hi0, c3, k1);
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    }
    q0 = (uint64_t)c0 | ((uint64_t)c1 << 32);
    q1 = (uint64_t)c2 | ((uint64_t)c3 << 32);
}
RT_D void rng_init(Rng& r, uint64_t seed, uint64_t pixel, uint32_t sample) {
    r.sample = sample; r.pix_lo = (uint32_t)pixel; r.pix_hi = (uint32_t)(pixel >> 32);
    r.k0 = (uint32_t)seed; r.k1 = (uint32_t)(seed >> 32);
    r.blk = 0; r.avail = 0; r.nready = 0; r.q0 = r.q1 = r.n0 = r.n1 = 0;
}
// Fallback for the rare draw that finds no next block ready.
RT_D void philox_next(Rng& r) {
    PH_COUNT(kPhRngWave, kPhRngLane);
    philox(r.blk, r.sample, r.pix_lo, r.pix_hi, r.k0, r.k1, r.n0, r.n1);
    r.blk++;
    r.nready = 1;
}
RT_D void rng_top_up(Rng& r) {  // coherent refill point (see Rng)
    if (!r.nready) {
        PH_COUNT(kPhRngWave, kPhRngLane);
        philox(r.blk, r.sample, r.pix_lo, r.pix_hi, r.k0, r.k1, r.n0, r.n1);
        r.blk++;
        r.nready = 1;
    }
}
// Skip the rest of the current block: the next draw starts a fresh one.  At
// every hit (oracle.c rng_align), so all lanes start their shading draws on a
// block boundary and lanes in the same branch refill at the same points.
RT_D void rng_align(Rng& r) { r.avail = 0; }
// Between two shading steps of the resumable path kernel a stream needs only its
// counter: the next shading step starts with rng_align, so the buffered words
// are never read (avail = 0), and a next block computed ahead (nready) is
// dropped and recomputed later from the same counter (blk - 1) — the same words.
// The key is re-read from the frame constants (rng_rekey) before the next step.
// Then nothing of the stream but blk (and its pixel / sample) stays live in
// registers across the triangle traversal.
RT_D void rng_park(Rng& r) {
    if (r.nready) { r.blk--; r.nready = 0; }
    r.avail = 0;
}
RT_D void rng_rekey(Rng& r, uint64_t seed) { r.k0 = (uint32_t)seed; r.k1 = (uint32_t)(seed >> 32); }
RT_D uint32_t next_u32(Rng& r) {
    if (r.avail == 0) {
        if (!r.nready) philox_next(r);
        r.q0 = r.n0; r.q1 = r.n1;
        r.nready = 0;
        r.avail = 4;
    }
    uint32_t w = (uint32_t)r.q0;
    r.q0 = (r.q0 >> 32) | (r.q1 << 32);
    r.q1 >>= 32;
    r.avail--;
    return w;
}
RT_D uint64_t next_u64(Rng& r) {
    uint64_t lo = next_u32(r);
    uint64_t hi = next_u32(r);
    return lo | (hi << 32);
}
// The draws of a diffuse shading step (render.hip segment_shade: the Mix coin
// word when `coin_draw`, then three u64) read straight from the block words.
// Precondition: rng_align + rng_top_up just ran, so nothing is buffered and the
// next block b sits in n0/n1 (nready) — true at every hit.  The words are those
// next_u32 / next_u64 would return (block b, then block b + 1, generated here
// as rng_top_up would), and the state afterwards is theirs too, without the
// per-word queue bookkeeping.
RT_D void diffuse_draws(Rng& r, bool coin_draw, bool& coin, uint64_t& A, uint64_t& B, uint64_t& C) {
    const uint64_t b0 = r.n0, b1 = r.n1;  // w0 | w1 << 32, w2 | w3 << 32 of block b
    uint64_t m0, m1;                      // block b + 1
    PH_COUNT(kPhRngWave, kPhRngLane);
    philox(r.blk, r.sample, r.pix_lo, r.pix_hi, r.k0, r.k1, m0, m1);
    r.blk++;
    r.nready = 0;
    r.q1 = 0;
    if (coin_draw) {
        coin = (uint32_t)b0 < 0x80000000u;  // gen_half: word w0
        A = (b0 >> 32) | (b1 << 32);        // w1, w2
        B = (b1 >> 32) | (m0 << 32);        // w3, block b + 1 w0
        C = (m0 >> 32) | (m1 << 32);        // w1, w2 of block b + 1
        r.q0 = m1 >> 32;                    // w3 of block b + 1 left
        r.avail = 1;
    } else {
        coin = true;
        A = b0; B = b1; C = m0;
        r.q0 = m1;
        r.avail = 2;
    }
}

// rand 0.8.5 transforms (see oracle.c header for the full list)
RT_D double gen_f64(Rng& r) { return (double)(next_u64(r) >> 11) * (1.0 / 9007199254740992.0); }
RT_D double value0_1(Rng& r) {
    return __longlong_as_double((long long)((next_u64(r) >> 12) | 0x3FF0000000000000ull)) - 1.0;
}
RT_D double gen_range(Rng& r, double low, double high) {  // UniformFloat::sample_single
    double scale = high - low;
    for (;;) {
        double res = value0_1(r) * scale + low;
        if (res < high) return res;
    }
}
RT_HD double inclusive_scale(double low, double high) {  // UniformFloat::new_inclusive
    const double max_rand = 1.0 - 2.220446049250313080847263336181640625e-16;  // (u64::MAX>>12 | 1.0) - 1
    double scale = (high - low) / max_rand;
    while (scale * max_rand + low > high) {
        uint64_t b;
        __builtin_memcpy(&b, &scale, 8);
        b -= 1;
        __builtin_memcpy(&scale, &b, 8);
    }
    return scale;
}
RT_D double gen_range_incl(Rng& r, double low, double scale) { return value0_1(r) * scale + low; }
// UniformInt<usize>::sample_single(0..range) with the exact acceptance zone
// (host-precomputed: DevScene::light_zone; oracle.c usize_zone)
RT_D uint64_t gen_index(Rng& r, uint64_t range, uint64_t zone) {
    for (;;) {
        uint64_t v = next_u64(r);
        uint64_t lo = v * range, hi = __umul64hi(v, range);
        if (lo <= zone) return hi;
    }
}
// Bernoulli(0.5) from one word: P(w < 2^31) = 1/2 exactly (oracle.c gen_half)
RT_D bool gen_half(Rng& r) { return next_u32(r) < 0x80000000u; }
RT_D bool gen_bool(Rng& r, double p) {  // Bernoulli
    if (p == 1.0) return true;  // ALWAYS_TRUE, no draw
    uint64_t p_int = (p >= 0.0 && p < 1.0) ? (uint64_t)(p * 18446744073709551616.0) : 0ull;
    return next_u64(r) < p_int;
}

// ------------------------------------------------------------- counters ---
struct Counters {
    uint32_t segments, aabb, tri, shape, shaded, lq, lhits, paths, steps;
    uint32_t lq_skip;  // last-bounce light queries the timed kernel skips (DevScene::lq_boxes)
    uint32_t kids[3];  // inner-node visits of closest-hit traversals by child boxes hit: none, one, both
};
template <bool ON>
struct Cnt {
    Counters c;
    RT_D void zero() { if (ON) { c = Counters{0, 0, 0, 0, 0, 0, 0, 0, 0, 0, {0, 0, 0}}; } }
    RT_D void kids(bool l, bool r) { if (ON) c.kids[(l ? 1 : 0) + (r ? 1 : 0)]++; }
    RT_D void lqskip() { if (ON) c.lq_skip++; }
    RT_D void segment() { if (ON) c.segments++; }
    RT_D void aabb(uint32_t n = 1) { if (ON) c.aabb += n; }
    RT_D void tri(uint32_t n = 1) { if (ON) c.tri += n; }
    RT_D void shape() { if (ON) c.shape++; }
    RT_D void shaded() { if (ON) c.shaded++; }
    RT_D void lq() { if (ON) c.lq++; }
    RT_D void lhit() { if (ON) c.lhits++; }
    RT_D void path() { if (ON) c.paths++; }
    RT_D void step() { if (ON) c.steps++; }
};

// ------------------------------------------------------ exact division ----
// The device's own division, split.  x / y compiles on gfx950 to
//   d = v_div_scale(y), r = v_rcp(d), two Newton steps r += r * (1 - d*r),
//   n = v_div_scale(x), q = n*r, rem = fma(-d, q, n),
//   v_div_fmas(rem, r, q), v_div_fixup
// (render.hip ISA).  When neither operand needs div_scale's rescaling,
// div_scale returns its operand, div_fmas is fma(rem, r, q) and div_fixup
// passes a finite normal quotient through — so the sequence splits into a
// per-divisor reciprocal part (dev_rcp: rcp + 4 FMAs) and a per-dividend
// quotient part (dev_quot: mul + 2 FMAs) with the SAME bits as x / y.  No
// rescaling happens for |y| in [2^-360, 2^360] (dir_ok) and |x| in
// [2^-500, 2^402]: the exponent gap stays below 768, the quotient is
// normal and the dividend's exponent far above the tiny-numerator case.
// A ray's 3 reciprocals then serve every slab and shape quotient of the
// ray at 3 ops each (instead of ~11 for x / y); an ellipsoid's reciprocals
// are computed once, by the device, into its record.
// Checked bit for bit against the host's x / y on random and adversarial
// pairs of the range (tests/test_gpu_parity.py test_dev_quot_matches_host).

// |d| in [2^-360, 2^360]: a ray direction component whose quotients may take dev_quot
RT_D bool dir_ok(double v) {
    return (((uint32_t)((uint64_t)__double_as_longlong(v) >> 52) & 0x7ffu) - 663u) < 721u;
}
RT_D double dev_rcp(double y) {
    double r = __builtin_amdgcn_rcp(y);
    double e = fma(-y, r, 1.0);
    r = fma(r, e, r);
    e = fma(-y, r, 1.0);
    return fma(r, e, r);
}
RT_D double dev_quot(double x, double y, double r) {
    const double q = x * r;
    const double rem = fma(-y, q, x);
    return fma(rem, r, q);
}
// dev_quot that also returns x / y's signed zero for x == +-0 (x * r has the
// sign sign(x) ^ sign(y), as x / y does)
RT_D double dev_quotz(double x, double y, double r) {
    const double q = dev_quot(x, y, r);
    return x == 0.0 ? x * r : q;
}

// dev_quot finished with the division's own last step, v_div_fixup: it passes a
// finite normal quotient through and returns x / y's signed zero for x == +-0
// (dev_quot's last FMA gives +0 for x == -0, y > 0).  x / y's bits over
// dev_quot's range and for x == +-0 in 4 ops (dev_quotz's compare-and-select
// takes 6); checked against the host (test_dev_quot_matches_host, op 5).
RT_D double dev_quotf(double x, double y, double r) {
    return __builtin_amdgcn_div_fixup(dev_quot(x, y, r), y, x);
}

// sqrt(x) as the device computes it (render.hip ISA): for x < 2^-767 the compiler
// pre-scales by 2^256, and 0 / +inf pass through a class test; for x in
// [2^-767, +inf) both steps are identities and the result is this core — rsq,
// two products and six FMAs — bit for bit.  Other x take the library sqrt (a
// divergent branch that whole waves skip).  dev_inv_len(dd) = 1 / sqrt(dd) of
// normalize (cgmath normalize_to(1)) with the split division where the length
// is in dir_ok's range.  Checked against the host (test_dev_sqrt_matches_host).
RT_D double sqrt_core(double x) {
    double r = __builtin_amdgcn_rsq(x);
    double g = x * r, h = r * 0.5;
    const double e = fma(-h, g, 0.5);
    g = fma(g, e, g);
    h = fma(h, e, h);
    double d = fma(-g, g, x);
    g = fma(d, h, g);
    d = fma(-g, g, x);
    return fma(d, h, g);
}
RT_D double dev_sqrt(double x) {
    if (x >= 0x1p-767 && x < INFINITY) return sqrt_core(x);
    return sqrt(x);
}
RT_D double dev_inv_len(double dd) {
    if (dd >= 0x1p-700 && dd <= 0x1p700) {  // length in [2^-350, 2^350]
        const double m = sqrt_core(dd);
        return dev_quot(1.0, m, dev_rcp(m));
    }
    return 1.0 / sqrt(dd);
}
RT_D V3 nrm(V3 v) { return v * dev_inv_len(dot(v, v)); }  // normalize (rt_math.h), device form

// per-axis reciprocals of a ray direction (shared by every slab test of a ray):
// dev_rcp(d) for dev_quot; ok bit i <=> dir_ok(d[i])
struct Rcp3 {
    V3 r;
    uint32_t ok;
};
RT_D Rcp3 make_rcp3(V3 d) {
    return Rcp3{v3(dev_rcp(d.x), dev_rcp(d.y), dev_rcp(d.z)),
                (dir_ok(d.x) ? 1u : 0u) | (dir_ok(d.y) ? 2u : 0u) | (dir_ok(d.z) ? 4u : 0u)};
}
// a ray whose slab and shape quotients may take dev_quot (given DevBvh::fast
// boxes / kShapeFast shapes): coordinates 0 or in [2^-397, 2^400], so every
// dividend min - o is 0 or in [2^-449, 2^401]
RT_D bool ray_fast(V3 o, const Rcp3& rc) {
    return rc.ok == 7u && coord_fast(o.x) && coord_fast(o.y) && coord_fast(o.z);
}

// ------------------------------------------------------------ geometry ----
// AABB::intersects (aabb.rs:51-108)
RT_D double safe_min(double a, double b) {
    if (!isfinite(a)) return b;
    if (!isfinite(b)) return a;
    return rmin(a, b);
}
RT_D double safe_max(double a, double b) {
    if (!isfinite(a)) return b;
    if (!isfinite(b)) return a;
    return rmax(a, b);
}
// FAST: the ray passed ray_fast() and the BVH's boxes DevBvh::fast — every
// slab quotient takes the unguarded exact division (no d == 0 axis either).
//
// In FAST mode the test reduces, exactly, to six quotients and plain min/max:
//   * no d == 0 axis and every quotient finite (operands in range), so the
//     safe_min/safe_max guards never fire;
//   * no NaN, so rmin/rmax equal v_min/v_max up to the sign of a zero result,
//     which no comparison observes;
//   * the inside test folds into max(t_near, 0): inside => t_near <= 0 <= t_far
//     (every axis has min - o <= 0 <= max - o); not inside => some axis has both
//     quotients of one sign, nonzero (|min - o| >= 2^-449), so either
//     t_near > 0 or t_far < 0 (a miss);
//   * so hit <=> t_near <= t_far && 0 <= t_far, and t = max(t_near, 0).
// (The host sets DevBvh::fast only when every box has min <= max per axis.)
RT_D bool aabb_hit_fast(V3 mn, V3 mx, V3 o, const Rcp3& rc, V3 d, double& t) {
    const double ax = dev_quot(mn.x - o.x, d.x, rc.r.x), bx = dev_quot(mx.x - o.x, d.x, rc.r.x);
    const double ay = dev_quot(mn.y - o.y, d.y, rc.r.y), by = dev_quot(mx.y - o.y, d.y, rc.r.y);
    const double az = dev_quot(mn.z - o.z, d.z, rc.r.z), bz = dev_quot(mx.z - o.z, d.z, rc.r.z);
    const double tn = __builtin_fmax(__builtin_fmax(__builtin_fmin(ax, bx), __builtin_fmin(ay, by)),
                                     __builtin_fmin(az, bz));
    const double tf = __builtin_fmin(__builtin_fmin(__builtin_fmax(ax, bx), __builtin_fmax(ay, by)),
                                     __builtin_fmax(az, bz));
    t = __builtin_fmax(tn, 0.0);
    return tn <= tf && 0.0 <= tf;
}
template <bool FAST = false>
RT_D bool aabb_hit(V3 mn, V3 mx, V3 o, V3 d, const Rcp3& rc, double& t) {
    if (FAST) return aabb_hit_fast(mn, mx, o, rc, d, t);
    if (!FAST && ((d.x == 0.0 && (o.x < mn.x || mx.x < o.x)) || (d.y == 0.0 && (o.y < mn.y || mx.y < o.y)) ||
                  (d.z == 0.0 && (o.z < mn.z || mx.z < o.z))))
        return false;
    if (!(o.x < mn.x || mx.x < o.x || o.y < mn.y || mx.y < o.y || o.z < mn.z || mx.z < o.z)) {
        t = 0.0;  // inside (aabb.rs:58-60)
        return true;
    }
    V3 tmin, tmax;
    if (FAST) {
        tmin = v3(dev_quot(mn.x - o.x, d.x, rc.r.x), dev_quot(mn.y - o.y, d.y, rc.r.y),
                  dev_quot(mn.z - o.z, d.z, rc.r.z));
        tmax = v3(dev_quot(mx.x - o.x, d.x, rc.r.x), dev_quot(mx.y - o.y, d.y, rc.r.y),
                  dev_quot(mx.z - o.z, d.z, rc.r.z));
    } else {
        tmin = div(mn - o, d);
        tmax = div(mx - o, d);
    }
    double t1x = safe_min(tmin.x, tmax.x), t1y = safe_min(tmin.y, tmax.y), t1z = safe_min(tmin.z, tmax.z);
    double t2x = safe_max(tmin.x, tmax.x), t2y = safe_max(tmin.y, tmax.y), t2z = safe_max(tmin.z, tmax.z);
    double tn = safe_max(safe_max(t1x, t1y), t1z);
    double tf = safe_min(safe_min(t2x, t2y), t2z);
    if (tn > tf) return false;
    if (0.0 <= tn) { t = tn; return true; }
    if (0.0 <= tf) { t = tf; return true; }
    return false;
}

// Quaternion::rotate_vector with an identity quaternion (s == 1, v == ±0):
// every cross product term is a signed zero, so each NONZERO finite component
// comes back bit-for-bit unchanged (x + ±0 == x).  Only a zero component can
// change (its sign depends on the others), so vectors with a zero or
// non-finite component take the generic formula.  Bit-exact either way.
RT_D bool is_identity(const Quat& q) {
    return q.s == 1.0 && q.v.x == 0.0 && q.v.y == 0.0 && q.v.z == 0.0;
}
RT_D bool all_nonzero_finite(V3 v) {
    return v.x != 0.0 && v.y != 0.0 && v.z != 0.0 && isfinite(v.x) && isfinite(v.y) && isfinite(v.z);
}
RT_D V3 rotate_fast(const Quat& q, bool ident, V3 v) {
    if (ident && all_nonzero_finite(v)) return v;
    return rotate(q, v);
}

// model_space_ray (intersections.rs:93-99).  Returns true when md == d bit for
// bit (identity rotation, d without zero components): the caller may then
// reuse the world ray's direction reciprocals.
RT_D bool model_ray(const DevShape& s, V3 o, V3 d, V3& mo, V3& md) {
    Quat r = conjugate(load_quat(s.rot));
    const bool ident = is_identity(r);
    mo = rotate_fast(r, ident, o - load3(s.pos));
    const bool same = ident && all_nonzero_finite(d);
    md = same ? d : rotate(r, d);
    return same;
}

// Model-space origin of a ray_fast ray for a kShapeFast shape (identity
// rotation, rt_layout.h) when it equals model_ray's bit for bit: o - pos and d
// without zero components, which rotate_fast returns unchanged (md = d).  Then
// o, pos and the shape's sizes are 0 or multiples of 2^-449 below 2^401, so
// every quotient of the box/ellipsoid test has a dividend that is 0 or in
// [2^-449, 2^402] and takes dev_quot(z) exactly.
RT_D bool shape_fast(const DevShape& s, bool rfast, V3 o, V3& mo) {
    if (!rfast || !(s.flags & kShapeFast)) return false;
    mo = o - load3(s.pos);
    return mo.x != 0.0 && mo.y != 0.0 && mo.z != 0.0;
}

// Plane::intersection (plane.rs:11-21); aux bit0 = (nd <= 0)
RT_D bool plane_t(V3 n, V3 o, V3 d, double& t, uint32_t& aux) {
    double nd = dot(n, d);
    double tt = -dot(n, o) / nd;
    if (tt < 0.0) return false;
    t = tt;
    aux = nd <= 0.0 ? 1u : 0u;
    return true;
}

// intersect_box_coef (box.rs:75-115). Entry/exit as (t, face): face = dim | 4 when
// the plane's normal sign is +1 (one 32-bit word, so each max/min update of the
// three axes selects three registers instead of five)
struct Bpi { double t; uint32_t face; };
// FD: shape_fast holds (d has no zero component; every quotient exact by dev_quotf)
template <bool FD = false>
RT_D int box_coef(V3 s, V3 o, V3 d, const Rcp3& rc, Bpi& en, Bpi& ex) {
    bool have = false;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        double di = comp(d, i), oi = comp(o, i), si = comp(s, i);
        if (!FD && di == 0.0 && si < fabs(oi)) return 0;
        if (!FD && di == 0.0) continue;
        const double ri = comp(rc.r, i);
        double t1 = FD ? dev_quotf(si - oi, di, ri) : (si - oi) / di;
        double t2 = FD ? dev_quotf(-si - oi, di, ri) : (-si - oi) / di;
        double a, b;
        uint32_t f;
        if (t1 < t2) { a = t1; b = t2; f = (uint32_t)i | 4u; } else { a = t2; b = t1; f = (uint32_t)i; }
        if (!have) { en = Bpi{a, f}; ex = Bpi{b, f}; have = true; }
        else {
            if (!(a < en.t)) en = Bpi{a, f};   // BoxPlaneIntersection::max (box.rs:57-59)
            if (b < ex.t) ex = Bpi{b, f};      // BoxPlaneIntersection::min (box.rs:60-62)
        }
    }
    if (!have) return 0;
    if (ex.t < en.t) return 0;
    if (0.0 <= en.t) return 2;
    if (0.0 <= ex.t) return 1;
    return 0;
}
RT_D V3 bpi_normal(const Bpi& p) {  // box.rs:64-72
    const double sign = (p.face & 4u) ? 1.0 : -1.0;
    const uint32_t dim = p.face & 3u;
    if (dim == 0) return v3(sign, 0.0, 0.0);
    if (dim == 1) return v3(0.0, sign, 0.0);
    return v3(0.0, 0.0, sign);
}
RT_D int bpi_dim(const Bpi& p) { return (int)(p.face & 3u); }
// aux encodes the returned face: bits0-1 dim, bit2 sign(+1), bit3 inside
RT_D uint32_t bpi_aux(const Bpi& p, bool inside) { return p.face | (inside ? 8u : 0u); }
RT_D V3 aux_box_normal(uint32_t aux) {
    double s = (aux & 4u) ? 1.0 : -1.0;
    uint32_t dim = aux & 3u;
    if (dim == 0) return v3(s, 0.0, 0.0);
    if (dim == 1) return v3(0.0, s, 0.0);
    return v3(0.0, 0.0, s);
}

// Ellipsoid radii with their device-computed reciprocals dev_rcp(r) (DevShape::aux).
struct Radii {
    V3 r, inv;
};
RT_D Radii load_radii(const DevShape& s) { return Radii{load3(s.shape), load3(s.aux)}; }
RT_D V3 div_radii(V3 v, const Radii& R) {  // v.div_element_wise(r)
    return div(v, R.r);
}

// intersect_ellipsoid_coef (ellipsoid.rs:49-76).  FD: shape_fast holds (o
// and d without zero components, radii dir_ok: o / r and d / r by dev_quot)
template <bool FD = false>
RT_D int ell_coef(const Radii& R, V3 o, V3 d, double& t1o, double& t2o) {
    V3 oo, dd;
    if (FD) {
        oo = v3(dev_quot(o.x, R.r.x, R.inv.x), dev_quot(o.y, R.r.y, R.inv.y), dev_quot(o.z, R.r.z, R.inv.z));
        dd = v3(dev_quot(d.x, R.r.x, R.inv.x), dev_quot(d.y, R.r.y, R.inv.y), dev_quot(d.z, R.r.z, R.inv.z));
    } else {
        oo = div_radii(o, R); dd = div_radii(d, R);
    }
    double c = dot(oo, oo), b = dot(oo, dd), a = dot(dd, dd);
    double disc = b * b - a * (c - 1.0);
    if (disc < 0.0) return 0;
    double ds = dev_sqrt(disc);
    double t1 = (-b + ds) / a, t2 = (-b - ds) / a;
    if (t2 < t1) { double tmp = t1; t1 = t2; t2 = tmp; }
    t1o = t1; t2o = t2;
    if (0.0 <= t1) return 2;
    if (0.0 <= t2) return 1;
    return 0;
}
RT_D V3 ell_normal(const Radii& R, V3 o, V3 d, double t) {  // ellipsoid.rs:26,29
    V3 p = o + d * t;
    return nrm(div_radii(div_radii(p, R), R));
}

// Triangle::intersection (triangle.rs:49-80) up to (u, v, t); normals later.
// TriRec: the hot record in registers (a, ba, ca).
struct TriRec { V3 a, ba, ca; };
RT_D TriRec load_tri(const DevTri& tr) {  // one batch of 16-B loads
    const double2* tw = (const double2*)&tr;
    const double2 w0 = tw[0], w1 = tw[1], w2 = tw[2], w3 = tw[3], w4 = tw[4];
    return TriRec{v3(w0.x, w0.y, w1.x), v3(w1.y, w2.x, w2.y), v3(w3.x, w3.y, w4.x)};
}
// A direction whose triangle quotients may take the split division against a
// compact record (Q below): every component 0 or |d_i| in [2^-240, 2^60).
RT_D bool tq_ok(double v) {
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    return (b << 1) == 0 || (((uint32_t)(b >> 52) & 0x7ffu) - 783u) < 300u;
}
RT_D bool dir_tq(V3 d) { return tq_ok(d.x) && tq_ok(d.y) && tq_ok(d.z); }
// Q && q: the record's edges are 0 or in [2^-149, 2^129) (differences of f32
// vertices, the compact layout; DevBvh::tri_q otherwise) and dir_tq(d) holds.  Every product of two edge or edge and
// direction components is then 0 or in [2^-389, 2^258], each cross-product
// component (a difference of two such products: 0 or a multiple of the smaller
// one's ulp) 0 or in [2^-441, 2^259], and |det| in [1e-11, 2^322] once the
// degenerate test passed: the nine quotients c / det are in dev_quot's range
// (or have a zero dividend), so one dev_rcp(det) and dev_quotf give x / y's bits
// at 4 ops each instead of the full division's 11.
template <bool Q = false>
RT_D bool tri_uvt_r(const TriRec& r, V3 o, V3 d, double& u, double& v, double& t, bool q = false) {
    V3 m0 = r.ba, m1 = r.ca, m2 = -d;
    double det = m0.x * (m1.y * m2.z - m2.y * m1.z) - m1.x * (m0.y * m2.z - m2.y * m0.z) +
                 m2.x * (m0.y * m1.z - m1.y * m0.z);
    if (fabs(det) < 1e-11) return false;
    const V3 c0 = cross(m1, m2), c1 = cross(m2, m0), c2 = cross(m0, m1);
    V3 x0, x1, x2;
    if (Q && q) {
        const double rr = dev_rcp(det);
        x0 = v3(dev_quotf(c0.x, det, rr), dev_quotf(c0.y, det, rr), dev_quotf(c0.z, det, rr));
        x1 = v3(dev_quotf(c1.x, det, rr), dev_quotf(c1.y, det, rr), dev_quotf(c1.z, det, rr));
        x2 = v3(dev_quotf(c2.x, det, rr), dev_quotf(c2.y, det, rr), dev_quotf(c2.z, det, rr));
    } else {
        x0 = c0 / det; x1 = c1 / det; x2 = c2 / det;
    }
    V3 w = o - r.a;
    double uu = dot(x0, w), vv = dot(x1, w), tt = dot(x2, w);
    if (uu < 0.0 || vv < 0.0 || 1.0 < uu + vv || tt < 0.0) return false;
    u = uu; v = vv; t = tt;
    return true;
}
RT_D bool tri_uvt(const DevTri& tr, V3 o, V3 d, double& u, double& v, double& t, bool q = false) {
    // The whole record in one batch of 16-B loads; the asm keeps `a` from being
    // loaded only after the determinant and its early exit, which exposed a second
    // memory round trip per test (C3 -1.3%, C5 -1.4% at reduced spp,
    // profiles/r02/variants/variants_tripre_*.log).
    const TriRec r = load_tri(tr);
    asm volatile("" ::"v"(r.a.x), "v"(r.a.y), "v"(r.a.z));
    return tri_uvt_r<true>(r, o, d, u, v, t, q);
}

// Intersection (intersections.rs:10-16)
struct Hit { double t; V3 ng, ns; bool inside; };

RT_D Hit rotated(const Hit& h, Quat q) {  // with_rotated_normal (intersections.rs:32-39)
    const bool ident = is_identity(q);
    return Hit{h.t, nrm(rotate_fast(q, ident, h.ng)), nrm(rotate_fast(q, ident, h.ns)), h.inside};
}

}  // namespace rt
