// rt_math.h — f64 vector/quaternion/AABB arithmetic with cgmath 0.18's exact
// operation order (host scene build + device kernels share it).
//
// Every operation below is a plain IEEE binary64 op; the whole product is
// compiled with -ffp-contract=off so no a*b+c becomes an FMA (the Rust
// reference never contracts).  Op-order conventions:
//   dot(a,b)      = (a.x*b.x + a.y*b.y) + a.z*b.z        (cgmath InnerSpace::dot)
//   normalize(v)  = v * (1 / sqrt(dot(v,v)))             (normalize_to(1))
//   q.rotate(v)   = t = q.v x v + v*q.s;  q.v x t * 2 + v  (Quaternion * Vector3)
//   conjugate(q)  = (q.s, -q.v)
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#define RT_HD __host__ __device__ __forceinline__

namespace rt {

constexpr double kPi = 3.14159265358979323846264338327950288;   // types.rs:13
constexpr double kEpsilon = 2.220446049250313080847263336181640625e-16 * 512.0;  // types.rs:14

struct V3 { double x, y, z; };
struct Quat { double s; V3 v; };     // cgmath Quaternion { s, v }
struct Box3 { V3 min, max; };        // aabb.rs:6-9

RT_HD V3 v3(double x, double y, double z) { return V3{x, y, z}; }
RT_HD V3 operator+(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
RT_HD V3 operator-(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
RT_HD V3 operator-(V3 a) { return v3(-a.x, -a.y, -a.z); }
RT_HD V3 operator*(V3 a, double s) { return v3(a.x * s, a.y * s, a.z * s); }
RT_HD V3 operator/(V3 a, double s) { return v3(a.x / s, a.y / s, a.z / s); }
// Coordinate range of the unguarded exact slab division (rt_device.h dev_quot):
// 0, or 2^-397 <= |v| <= 2^400.
RT_HD bool coord_fast(double v) {
    const double a = v < 0.0 ? -v : v;
    return a == 0.0 || (a >= 0x1p-397 && a <= 0x1p400);
}
RT_HD V3 mul(V3 a, V3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }   // mul_element_wise
RT_HD V3 div(V3 a, V3 b) { return v3(a.x / b.x, a.y / b.y, a.z / b.z); }   // div_element_wise
RT_HD double dot(V3 a, V3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
RT_HD V3 cross(V3 a, V3 b) {
    return v3((a.y * b.z) - (a.z * b.y), (a.z * b.x) - (a.x * b.z), (a.x * b.y) - (a.y * b.x));
}
RT_HD double magnitude(V3 a) { return sqrt(dot(a, a)); }
RT_HD V3 normalize(V3 a) { return a * (1.0 / magnitude(a)); }
RT_HD double comp(V3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }
RT_HD V3 load3(const double* p) { return v3(p[0], p[1], p[2]); }
RT_HD void store3(double* p, V3 a) { p[0] = a.x; p[1] = a.y; p[2] = a.z; }

RT_HD Quat conjugate(Quat q) { return Quat{q.s, -q.v}; }
RT_HD V3 rotate(Quat q, V3 v) {
    V3 tmp = cross(q.v, v) + v * q.s;
    return cross(q.v, tmp) * 2.0 + v;
}
RT_HD Quat load_quat(const double* p) { return Quat{p[0], v3(p[1], p[2], p[3])}; }

// aabb.rs:34-40 — NaN-asymmetric min/max
RT_HD double rmin(double a, double b) { return a < b ? a : b; }
RT_HD double rmax(double a, double b) { return b < a ? a : b; }
RT_HD Box3 box_empty() {  // aabb.rs:16-21
    return Box3{v3(INFINITY, INFINITY, INFINITY), v3(-INFINITY, -INFINITY, -INFINITY)};
}
RT_HD void box_extend(Box3& b, V3 v) {  // aabb.rs:23-26
    b.min = v3(rmin(b.min.x, v.x), rmin(b.min.y, v.y), rmin(b.min.z, v.z));
    b.max = v3(rmax(b.max.x, v.x), rmax(b.max.y, v.y), rmax(b.max.z, v.z));
}
RT_HD void box_extend(Box3& b, const Box3& o) {  // aabb.rs:28-31
    b.min = v3(rmin(b.min.x, o.min.x), rmin(b.min.y, o.min.y), rmin(b.min.z, o.min.z));
    b.max = v3(rmax(b.max.x, o.max.x), rmax(b.max.y, o.max.y), rmax(b.max.z, o.max.z));
}

}  // namespace rt
