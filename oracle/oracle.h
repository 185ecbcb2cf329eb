/*
 * oracle.h — CPU restatement of uncerso/cpu-raytracing-rt's hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (cpu-raytracing-rt_amd/)
 * links, loads or calls this; only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py do, and only as the checker / CPU baseline.
 *
 * Parity status:
 *  - pinned by the reference's own 13 known-answer tests (tests/golden/kats.json:
 *    aabb.rs:118-151, primitives/box.rs:129-171, primitives/triangle.rs:98-144,
 *    gltf/scene_builder.rs:408-426) — checked by tests/test_oracle_kats.py;
 *  - Philox4x32-10 pinned by the Random123 known-answer vectors;
 *  - everything else (cgmath op order, rand 0.8 transforms, image-level
 *    estimator) is "parity unpinned": the Rust reference cannot be built here
 *    (no cargo/rustc, no crates) and has no golden images; the restatement
 *    follows the cited file:line of the reference operation by operation.
 */
#ifndef RT_ORACLE_H
#define RT_ORACLE_H

#include <stdint.h>
#include "../include/rt_api.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_scene oracle_scene;

/* Scene::new / make_scenes (scene.rs:180-223) incl. the six BVH builds. */
oracle_scene* oracle_scene_create(const rt_scene_desc* desc);
void oracle_scene_destroy(oracle_scene* s);
/* node counts / depths of the six BVHs, same order as rt_scene_info.bvh_nodes */
void oracle_scene_bvh_info(const oracle_scene* s, uint64_t nodes[6], uint32_t depth[6]);
/* Flattened pre-order node dump of BVH k (0..5) for structure comparison:
   per node: left, right, start, end (int64, -1 for none), then min[3], max[3]. */
uint64_t oracle_scene_bvh_dump(const oracle_scene* s, int k, int64_t* links, double* bounds);
/* Global primitive id of the i-th primitive of BVH k, in BVH order. */
int64_t oracle_scene_bvh_prim(const oracle_scene* s, int k, uint64_t i);

/* generate_image (main.rs:85-114) without tonemapping: mean radiance.
   mode 0 = recursive raytrace_impl (raytrace.rs:12-60, faithful form),
   mode 1 = iterative throughput form (the device algorithm, bit-identical to it),
   mode 2 = recursive raytrace_impl drawing the reference's own rand 0.8.5 call
            sequence (ray_sampler.rs:87-157, raytrace.rs:46: gen_bool(0.5) coin,
            per-branch draws, an index draw even for one light, rand's conservative
            UniformInt zones, no block alignment) on the same Philox word stream —
            the statistical pin of the build's stream layout (modes 0/1).
   row_begin/row_end restrict the rendered rows (CPU-baseline sub-window);
   threads <= 0 => OpenMP default.  Returns 0 or negative on error. */
int oracle_render(const oracle_scene* s, const rt_render_params* p, int mode,
                  int threads, uint32_t row_begin, uint32_t row_end,
                  double* out_mean_rgb, int32_t* opt_hit_ids, rt_stats* opt_stats);

/* As oracle_render, with the device's chunked sample summation: a pixel's
   samples are summed in runs of chunk_spp (each run from 0), the run sums are
   added in order and the total divided by spp (render.hip reduce_chunks_kernel).
   chunk_spp >= spp (or 0) is the plain sequential sum of main.rs:94-104. */
int oracle_render_chunked(const oracle_scene* s, const rt_render_params* p, int mode,
                          int threads, uint32_t row_begin, uint32_t row_end, uint32_t chunk_spp,
                          double* out_mean_rgb, int32_t* opt_hit_ids, rt_stats* opt_stats);

/* As oracle_render (sequential sum), plus the per-pixel second moment
   out_sq = sum over samples of L*L / spp per channel (the sample variance of the
   estimator is out_sq - mean^2). */
int oracle_render_moments(const oracle_scene* s, const rt_render_params* p, int mode,
                          int threads, uint32_t row_begin, uint32_t row_end,
                          double* out_mean_rgb, double* out_sq, rt_stats* opt_stats);

/* intersect(ray, primitives, +inf) for a batch (intersections.rs:42-62). */
void oracle_intersect_rays(const oracle_scene* s, const double* rays, uint32_t n, rt_hit* out);
/* Light::pdf for a batch of (pos, dir) (ray_sampler.rs:132-139). */
void oracle_light_pdf_rays(const oracle_scene* s, const double* pos_dir, uint32_t n, double* out);

/* ---- known-answer-test hooks ------------------------------------------- */
/* AABB::intersects (aabb.rs:51-78); returns 1 and *t if Some. */
int oracle_aabb_intersects(const double mn[3], const double mx[3], const double o[3], const double d[3], double* t);
/* Box::intersection (box.rs:21-33): returns 1 if Some; t, geometry normal, inside. */
int oracle_box_intersection(const double sizes[3], const double o[3], const double d[3],
                            double* t, double n[3], int* inside);
/* Ellipsoid::intersection (ellipsoid.rs:21-32). */
int oracle_ellipsoid_intersection(const double r[3], const double o[3], const double d[3],
                                  double* t, double n[3], int* inside);
/* Plane::intersection (plane.rs:11-21). */
int oracle_plane_intersection(const double nrm[3], const double o[3], const double d[3],
                              double* t, double n[3]);
/* TrianglePrimitive::new(Triangle::new_with_geometry_normals(a,b,c), pos, rot) then
   intersection (triangle.rs:19-80, scene.rs:139-165). rot = (s,x,y,z). */
int oracle_triangle_intersection(const double abc[9], const double pos[3], const double rot[4],
                                 const double o[3], const double d[3],
                                 double* t, double ng[3], double ns[3], int* inside);
/* cof() of gltf/scene_builder.rs:367-388, column-major m[c][r]. */
void oracle_cof3(const double m[9], double out[9]);
/* Philox4x32-10 block (Random123 convention). */
void oracle_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
/* First n u64 of the per-(pixel,sample) stream, and rand-0.8 transforms. */
void oracle_rng_stream_u64(uint64_t seed, uint64_t pixel, uint32_t sample, uint32_t n, uint64_t* out);
/* Samplers on a stream: kind 0 = Cosine::sample(normal), kind 1 = uniform_on_box(sizes),
   kind 2 = uniform_on_sphere, kind 3 = gen_range(0..n) (n in arg[0]), 4 = gen_bool(arg[0]).
   Writes 3 doubles per draw (unused slots 0). */
void oracle_sampler_draws(uint64_t seed, uint64_t pixel, uint32_t sample, int kind,
                          const double arg[3], uint32_t n, double* out);

/* BVH::new over raw boxes [n][6]; returns node count (call with links NULL first). */
uint64_t oracle_bvh_build(const double* boxes, uint64_t n, int64_t* links, double* bounds, uint64_t* order,
                          uint32_t* depth);
/* intersect_lights accumulation without offset/normalisation + callback count. */
void oracle_intersect_lights_rays(const oracle_scene* s, const double* rays, uint32_t n, double* impact,
                                  uint32_t* count);

/* ---- host output surface restated (postprocessing.rs, ppm.rs) ----------- */
void oracle_tonemap_gamma(const double* in, uint64_t n_pixels, double* out);
void oracle_ppm_bytes(const double* rgb, uint64_t n_pixels, uint8_t* out);

#ifdef __cplusplus
}
#endif
#endif
