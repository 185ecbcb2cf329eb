/*
 * rt_api.h — C ABI of the MI355X-native path-tracing hot path.
 *
 * Drop-in boundary for uncerso/cpu-raytracing-rt (Rust, CPU).  The reference
 * has no FFI: its only seam is `generate_image(&Scene) -> Image`
 * (src/main.rs:85-114), called once per frame by `main` (src/main.rs:73).
 * Every entry point below names the reference item it replaces.  All
 * signatures are plain C (PODs, pointers, sizes) so a Rust host can bind them
 * with `extern "C"` + `#[repr(C)]`, or Python via ctypes.
 *
 * Conventions
 *  - Return value: 0 (RT_OK) on success, a negative rt_error otherwise.  Nothing
 *    unwinds or aborts across the ABI (the reference panics instead:
 *    src/gltf/scene_builder.rs:58,210,212, src/scene.rs:188).  The message of the
 *    last failure on the calling thread is available from rt_last_error().
 *  - Ownership: the caller owns every host buffer; arrays in descriptors are
 *    BORROWED for the duration of the call.  The library owns device memory
 *    behind opaque handles.
 *  - Numerics: f64 everywhere, like the reference (src/types.rs:5).
 *  - Threading: one host thread per handle (a handle is not re-entrant), as
 *    the reference calls its pixel loop once from the main thread.
 *  - Devices: a scene lives on the device that was current at rt_scene_create.
 *    Every call taking a scene switches to that device for its duration and
 *    restores the caller's current device before returning.
 *  - Streams: launches that use a scene's shared workspace (queue, sample ring,
 *    chunk partials, stack spill) are ordered by the library: each waits for
 *    the previous one on that scene through an event, whatever stream either
 *    was issued on.  Calls on different streams therefore never overlap on one
 *    scene (they serialise); use one scene per stream for concurrency.
 */
#ifndef RT_API_H
#define RT_API_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_API_VERSION 6

typedef enum rt_error {
    RT_OK = 0,
    RT_ERR_INVALID = -1,     /* bad argument / inconsistent descriptor            */
    RT_ERR_DEVICE = -2,      /* HIP runtime error (no device, launch failure ...) */
    RT_ERR_NOMEM = -3,       /* host or device allocation failed                  */
    RT_ERR_PARSE = -4,       /* scene text / glTF JSON could not be parsed        */
    RT_ERR_IO = -5,          /* file could not be read or written                 */
    RT_ERR_UNSUPPORTED = -6  /* input the reference also rejects (e.g. glTF mode!=4) */
} rt_error;

/* ---- materials: src/scene.rs:6-18 (Material, Metadata) ------------------- */
enum { RT_MAT_DIFFUSE = 0, RT_MAT_METALLIC = 1, RT_MAT_DIELECTRIC = 2 };

typedef struct rt_material {
    uint32_t kind;        /* RT_MAT_*                                         */
    uint32_t _pad;
    double ior;           /* Material::Dielectric(ior); ignored otherwise      */
    double color[3];      /* Metadata::color    (default 0, scene.rs:102)      */
    double emission[3];   /* Metadata::emission (!= 0 => light, scene.rs:225)  */
} rt_material;

/* ---- analytic shapes: src/primitives/{plane,box,ellipsoid}.rs ------------ */
enum { RT_SHAPE_PLANE = 0, RT_SHAPE_BOX = 1, RT_SHAPE_ELLIPSOID = 2 };

typedef struct rt_shape {
    uint32_t type;        /* RT_SHAPE_*                                        */
    uint32_t material;    /* index into rt_scene_desc.materials                */
    double shape[3];      /* plane normal | box half-sizes | ellipsoid radii   */
    double position[3];   /* Primitive::position (default 0, scene.rs:110)     */
    double rotation[4];   /* Primitive::rotation as (s, x, y, z); NOT normalised,
                             exactly as parsed (scene_parser.rs:51-57)         */
} rt_shape;

/* ---- triangles ------------------------------------------------------------ */
enum {
    /* custom-format TRIANGLE: Triangle::new_with_geometry_normals then
       TrianglePrimitive::new (rotate+translate, props recomputed)
       (scene_parser.rs:71-73, scene.rs:139-165)                                */
    RT_TRI_CUSTOM = 0,
    /* glTF: world-space vertices+normals, Triangle::new_with_smooth_normal then
       `instantiate` (AABB of a, a+ba, a+ca) (gltf/scene_builder.rs:42-55,329-356) */
    RT_TRI_GLTF = 1
};

/*
 * Scene description = the reference's parsed scene (parsed_scene.rs:4-75 for
 * the custom format; the flattened triangle list of gltf/scene_builder.rs for
 * glTF).  Shapes and triangles are each in INPUT order; the library splits them
 * per kind preserving relative order and builds the six BVHs exactly as
 * make_scenes does (scene.rs:194-223).  Global primitive id (used by hit-id
 * dumps): shape i -> i, triangle j -> n_shapes + j.
 */
typedef struct rt_scene_desc {
    uint32_t n_materials;
    uint32_t n_shapes;
    uint64_t n_triangles;
    const rt_material* materials;
    const rt_shape* shapes;
    uint32_t tri_mode;              /* RT_TRI_CUSTOM | RT_TRI_GLTF            */
    uint32_t _pad;
    const double* tri_vertices;     /* [n][3][3]: a, b, c                     */
    const double* tri_normals;      /* [n][3][3]: na, nb, nc (GLTF only)      */
    const double* tri_position;     /* [n][3] (CUSTOM only; NULL => 0)        */
    const double* tri_rotation;     /* [n][4] (s,x,y,z) (CUSTOM; NULL => id)  */
    const uint32_t* tri_material;   /* [n]                                    */
} rt_scene_desc;

/* ---- camera: src/scene.rs:36-49 (Fov, CameraParams), src/camera.rs ------- */
enum { RT_FOV_X = 0, RT_FOV_Y = 1 };

/* flags */
#define RT_FLAG_STATS        0x1u  /* fill rt_stats work counters (separate untimed pass) */
#define RT_FLAG_HIT_IDS      0x2u  /* dump (pixel, sample, bounce) -> global primitive id */

typedef struct rt_render_params {
    uint32_t width, height;        /* Scene::dimensions                        */
    uint32_t spp;                  /* Scene::samples                           */
    uint32_t ray_depth;            /* Scene::ray_depth (u8 in the reference)   */
    double bg_color[3];            /* Scene::bg_color                          */
    double cam_position[3];        /* CameraParams (already normalised for the
                                      custom format, scene.rs:169-175)         */
    double cam_right[3], cam_up[3], cam_forward[3];
    uint32_t fov_axis;             /* RT_FOV_X | RT_FOV_Y                      */
    uint32_t flags;                /* RT_FLAG_*                                */
    double fov;                    /* radians                                  */
    uint64_t seed;                 /* counter-based RNG key (replaces the
                                      OS-seeded thread_rng, main.rs:95)        */
} rt_render_params;

/* Work counters of one render (canonical byte model: DESIGN.md §4). */
typedef struct rt_stats {
    uint64_t paths;            /* camera paths = W*H*spp                         */
    uint64_t segments;         /* closest-hit queries (raytrace.rs:14) = samples */
    uint64_t aabb_tests;       /* AABB::intersects calls (aabb.rs:51)            */
    uint64_t tri_tests;        /* Triangle::intersection calls                   */
    uint64_t shape_tests;      /* plane/box/ellipsoid intersection calls         */
    uint64_t shaded_hits;      /* closest hits returned to the integrator        */
    uint64_t light_queries;    /* Light::pdf all-hits queries                    */
    uint64_t light_hits;       /* callbacks of intersect_lights                  */
    double   kernel_ms;        /* device time of the path kernel(s)              */
    double   total_ms;         /* wall time of rt_render incl. copies            */
    uint64_t lane_steps;       /* regeneration-loop steps summed over lanes      */
    uint64_t wave_steps;       /* 64 x (steps of the wave's longest lane): lane  */
                               /* utilisation of the path loop = lane/wave steps */
} rt_stats;

/* Hit-id sentinels in the (pixel, sample, bounce) dump */
#define RT_HIT_MISS      (-1)   /* closest-hit query returned None -> bg_color   */
#define RT_HIT_NONE      (-2)   /* bounce not reached (path ended earlier)       */

/* Ray-query result (intersections.rs:10-16 Intersection + winner id). */
typedef struct rt_hit {
    double t;
    double geometry_normal[3];  /* world space, rotated+normalised (intersections.rs:32-39) */
    double shading_normal[3];
    int32_t inside;
    int32_t prim;               /* global primitive id or RT_HIT_MISS            */
} rt_hit;

typedef struct rt_scene rt_scene;            /* opaque, device-resident       */
typedef struct rt_parsed_scene rt_parsed_scene; /* opaque, host-side parse result */

/* ======================= scene lifetime =================================== */
/* Replaces Scene::new + make_scenes (src/scene.rs:180-223) and BVH::new
   (src/bvh.rs:12-17); uploads the flattened scene to the CURRENT HIP device. */
int  rt_scene_create(const rt_scene_desc* desc, rt_scene** out);
void rt_scene_destroy(rt_scene* scene);

typedef struct rt_scene_info {
    uint32_t n_planes, n_boxes, n_ellipsoids;
    uint64_t n_triangles;
    uint32_t n_light_boxes, n_light_ellipsoids;
    uint64_t n_light_triangles;
    uint64_t bvh_nodes[6];       /* boxes, ellipsoids, triangles, light boxes, light ellipsoids, light triangles */
    uint32_t bvh_depth[6];
    double   build_ms;           /* host BVH build                                */
    double   upload_ms;          /* H2D copy                                      */
    uint64_t device_bytes;       /* the scene's arrays; the per-launch workspace (commit
                                    ring, split-tail row buffer <= 256 MB, chunk partials
                                    <= 4 GiB, stack spill) is grow-only, sized by the
                                    largest frame rendered, and not counted here      */
    /* bit i: scene box i (BVH order) doubles as the next light box, so the light
       pdf of a diffuse bounce comes from the next segment's box tests (DESIGN.md
       §4 "shared light tests"); 0 = separate light queries */
    uint32_t shared_light_mask;
    /* RT_LAYOUT_COMPACT_TRIS: the triangle BVH also has its compact layout (f32
       child boxes and vertices, every one an exact copy of the f64 value; DESIGN.md
       §2), which the resumable triangle-only kernel reads */
    /* RT_LAYOUT_LQ_SKIP: every light is a box whose world bounds the host could
       bound exactly (api.cpp lq_boxes), so the timed kernel may skip
       last-bounce light queries proven NaN-free */
    uint32_t layout_flags;
} rt_scene_info;
#define RT_LAYOUT_COMPACT_TRIS 0x1u
#define RT_LAYOUT_LQ_SKIP      0x2u
/* RT_LAYOUT_PAIR_NODES: the compact triangle BVH also has its pair layout (one 128-B
   line per inner node holding what a visit of either child tests, so a descent reads
   one line per two levels), which the resumable kernel reads when it is
   there (rt_tuning.compact auto or 2) */
#define RT_LAYOUT_PAIR_NODES   0x4u
int rt_scene_get_info(const rt_scene* scene, rt_scene_info* out);
/* Content hash of the scene's device arrays (BVHs, records, materials; not the
   per-launch workspace), computed on the scene's device.  Two handles built from the
   same description — or an rt_multi replica and devices[0]'s scene — hash equal;
   rt_multi_create checks every replica this way after the fill. */
int rt_scene_checksum(rt_scene* scene, uint64_t* out);

/* Kernel form of a scene's renders.  The library picks every
   field from the scene itself ("auto"); a caller may force one for tests and
   tuning.  The library reads no environment variables: the resolved form is a
   property of the scene handle, reported by rt_scene_get_tuning, so every rank
   and process rendering one frame runs the same kernel instance. */
typedef struct rt_tuning {
    uint32_t waves;          /* 0 auto (shape-only scenes 5; else 4 when the BVHs hold > 4096 nodes,
                                else 3); 3, 4 or 5 waves/SIMD (5: the shape-only fused kernel only,
                                other forms run 4 and report it) */
    int32_t  resume;         /* -1 auto (1 for a triangle BVH of > 4096 nodes); 0 fused segment,
                                1 resumable triangle traversal                                          */
    uint32_t kinds;          /* 0 auto (the scene's primitive kinds); 3 the all-kinds instance; 1 or 2
                                only as the scene's own kinds (the value rt_scene_get_tuning reports)   */
    uint32_t suspend_lanes;  /* 0 auto (compact layouts: 24 cache-resident BVH, 48 HBM-streamed; the f64
                                layout: 32 / 48); 1..64                                                 */
    uint32_t leaf_lanes;     /* 0 auto (compact layouts: 16 cache-resident BVH, 12 HBM-streamed; the f64
                                layout: 32 / 28); 1..64                                                 */
    uint32_t chunk_spp;      /* 0 the frame's rule (rt_sample_chunks); else the sample run length,
                                raised if need be to <= 64 runs and <= 4 GiB of partial sums
                                (rt_scene_sample_chunks reports the run length used)                    */
    int32_t  compact;        /* -1 auto (2 when the scene has RT_LAYOUT_PAIR_NODES, else 1 when it
                                has RT_LAYOUT_COMPACT_TRIS); 0 the f64 triangle-BVH layout; 1 the
                                compact one with 64-B nodes (triangle-only resumable kernel;
                                RT_ERR_UNSUPPORTED on a scene without RT_LAYOUT_COMPACT_TRIS); 2 the
                                compact one with its pair layout (RT_LAYOUT_PAIR_NODES)               */
    uint32_t tail_split;     /* 0 auto (8); 1 every wave-tile whole; 2..8: the queue's last wave-tiles
                                (three per resident wave) are handed out in this many parts of
                                consecutive sample rows and summed in sample order after the launch
                                (the same image: DESIGN.md section 5 "per-launch tail")            */
    /* Version 5 replaced version 4's last field (`sorted`, the regrouped-shading kernel) with
       tail_split; version 6 added compact = 2 (the same struct).  Auto is 0 for the unsigned fields and -1 for the signed ones (resume,
       compact): a zero-initialised struct is not all-auto.  NULL restores every field to auto. */
} rt_tuning;
/* NULL restores every field to auto.  Fields out of range -> RT_ERR_INVALID. */
int rt_scene_set_tuning(rt_scene* scene, const rt_tuning* tuning);
/* The form the next render of this scene runs: auto fields resolved (chunk_spp
   stays 0 when the frame's rule applies).  tail_split: after a render, the split that
   frame resolved to (1 when the split cannot apply: sample runs >= 65536 rows or no
   room for a row buffer); before any render since rt_scene_set_tuning, the setting. */
int rt_scene_get_tuning(const rt_scene* scene, rt_tuning* resolved);

/* ======================= the frame (hot path) ============================= */
/* Replaces generate_image's pixel loop (src/main.rs:85-103): for every pixel,
   the mean over spp of raytrace(Camera::fuzzy_ray(px)) (camera.rs:48-55,
   raytrace.rs:8-60).  out_mean_rgb: caller-owned [H][W][3] f64, row-major
   idx = y*W + x (main.rs:96-97), BEFORE aces_tonemap/correct_gamma
   (main.rs:104).  opt_hit_ids: NULL or caller-owned [W*H][spp][ray_depth]
   int32 (requires RT_FLAG_HIT_IDS).  opt_stats: NULL or filled. */
int rt_render(rt_scene* scene, const rt_render_params* params,
              double* out_mean_rgb, int32_t* opt_hit_ids, rt_stats* opt_stats);

/* Multi-GPU tile partition: 16x16 tiles, tile t belongs to
   rank t % world.  Each rank renders its tiles into a packed DEVICE buffer
   [n_tiles_padded][256][3] f64 (n_tiles_padded = ceil(total_tiles/world)),
   asynchronously on `hip_stream` (NULL = default stream). */
#define RT_TILE 16
int rt_tiles_per_rank(const rt_render_params* params, uint32_t world, uint32_t* n_tiles_padded);
/* The scene's per-call workspace (stack spill, chunk partials) is shared;
   successive calls are ordered on it across streams (Conventions: Streams). */
int rt_render_tiles_async(rt_scene* scene, const rt_render_params* params,
                          uint32_t rank, uint32_t world,
                          double* d_tile_rgb, void* hip_stream);

/* Diagnostics: the scene's raw device counter words (n <= 64), accumulated by
   RT_FLAG_STATS renders: words 0..9 are rt_stats' counters; word 10 counts the
   last-bounce light queries the timed (no-stats) kernel skips because they cannot
   be NaN (the stats render still runs them); words 11..13
   count the inner-node visits of closest-hit BVH traversals whose two child boxes
   were hit by none / one / both slab tests; builds compiled
   with -DRT_PHASES add wave cycles and loop counts per path-kernel region at
   words 16..51 (16 + kPhN - 1, phases.h; tools/phases.py).  Word 14 counts waves
   the stats kernel's progress guard stopped (kStallTrips trips without progress; a
   nonzero word makes rt_render / rt_read_stats return RT_ERR_DEVICE).  Words 52..59
   are the last stats launch's wave timeline (s_memrealtime, 100 MHz; cleared at
   each stats launch, not accumulated; tools/timeline.py): ~earliest start, last
   exit, ~earliest and last time a wave found the wave-tile queue drained, sum and
   max of drain-to-exit, sum of start-to-exit, waves.  Not needed to render. */
int rt_read_raw_stats(rt_scene* scene, uint64_t* out, uint32_t n);

/* Sample chunking of the work units: a pixel's spp samples are
   rendered in `chunks` runs of `chunk_spp` consecutive samples by different
   lanes; each run is summed in sample order from 0, the run sums are added in
   run order and divided by spp.  A function of (width, height, spp) only, so the
   image is identical for any rank count.  chunks == 1 is exactly main.rs:94-104's
   sequential sum; otherwise the result differs from it by f64 reassociation only
   (no replacement for main.rs; exposed so checkers can reproduce the order). */
int rt_sample_chunks(const rt_render_params* params, uint32_t* chunks, uint32_t* chunk_spp);
/* The chunking this scene's renders use: rt_sample_chunks unless its tuning
   forces a run length (rt_tuning.chunk_spp). */
int rt_scene_sample_chunks(const rt_scene* scene, const rt_render_params* params, uint32_t* chunks,
                           uint32_t* chunk_spp);
/* Work counters accumulated on the device by every rt_render_tiles_async call
   made with RT_FLAG_STATS since the last reset (synchronises the device). */
int rt_read_stats(rt_scene* scene, rt_stats* out, int reset);
/* Root side after the gather: d_gathered = [world][n_tiles_padded][256][3]
   (rank-major, as ncclGather lays it out) -> d_image [H][W][3]. */
int rt_unpack_tiles_async(const rt_render_params* params, uint32_t world,
                          const double* d_gathered, double* d_image, void* hip_stream);
/* The same unpack fused with correct_gamma(aces_tonemap(.)) and the PPM byte
   quantisation (main.rs:104, postprocessing.rs:5-37, ppm.rs:13-19): d_bytes is
   the P6 payload [H][W][3] u8, so the f64 image never leaves the device.  The
   bytes are the host path's (rt_tonemap_gamma + rt_save_ppm) bit for bit: the
   device computes aces_tonemap with the same IEEE operations, and the gamma +
   quantisation step is a search over 255 thresholds on the tonemapped value
   that the host derives from its own `pow` (post.cpp byte_thresholds). */
int rt_unpack_tiles_bytes_async(const rt_render_params* params, uint32_t world,
                                const double* d_gathered, uint8_t* d_bytes, void* hip_stream);
/* Device tonemap + gamma + PPM bytes of a mean-radiance image already in HBM
   ([n_pixels][3] f64 -> [n_pixels][3] u8). */
int rt_tonemap_bytes_async(const double* d_rgb, uint64_t n_pixels, uint8_t* d_bytes, void* hip_stream);

/* ======================= one process, several GPUs ======================== */
/* generate_image (src/main.rs:85-114) over several GPUs of one node, driven
   from ONE host thread exactly like rt_render (the Rust `main`, main.rs:73,
   keeps its single call per frame):
    - rt_multi_create builds the six BVHs once on the host (scene.rs:180-223,
      bvh.rs:12-17) and uploads one scene replica per listed device;
    - rt_multi_render deals the frame's 16x16 tiles round-robin (tile t ->
      device index t % n, the rt_render_tiles_async partition), renders every
      share on its own device and stream, makes ONE gather of the packed tiles
      to devices[0] (an RCCL ncclGather over xGMI; peer copies with
      RT_MULTI_PEER), then unpacks on devices[0] and copies the image to the
      host once.
   The image is bit-identical to rt_render's for any device count (the RNG is
   keyed by the global pixel and sample, the chunking by the frame alone).
   out_mean_rgb: NULL or caller-owned [H][W][3] f64 (main.rs:104 before the
   tonemap); out_ppm_bytes: NULL or caller-owned [H][W][3] u8, the P6 payload
   of correct_gamma(aces_tonemap(.)) made on the device (as
   rt_unpack_tiles_bytes_async); at least one is required.  opt_stats: work
   counters summed over the devices (RT_FLAG_STATS), kernel_ms = the slowest
   device's render, total_ms = the call's wall time.
   RCCL is loaded at rt_multi_create (dlopen of librccl.so.1); without it, or
   with a device listed twice, RT_MULTI_PEER is required. */
#define RT_MULTI_PEER 0x1u  /* gather with hipMemcpyPeerAsync instead of RCCL;
                               allows a device listed more than once (several
                               replicas on one GPU: a rehearsal of the N-way
                               partition on a one-GPU machine) */
typedef struct rt_multi rt_multi;
int  rt_multi_create(const rt_scene_desc* desc, const int* devices, uint32_t n_devices, uint32_t flags,
                     rt_multi** out);
int  rt_multi_render(rt_multi* m, const rt_render_params* params, double* out_mean_rgb,
                     uint8_t* out_ppm_bytes, rt_stats* opt_stats);
/* The replica on device index i (0 <= i < n) for per-device queries; owned by m. */
rt_scene* rt_multi_scene(rt_multi* m, uint32_t index);
void rt_multi_destroy(rt_multi* m);

/* ======================= ray queries ====================================== */
/* Closest hit for a batch of world rays [n][6] = (origin, dir) — replaces
   intersections.rs:42-62 `intersect(ray, &scene.primitives, +inf)`. */
int rt_intersect_rays(rt_scene* scene, const double* rays, uint32_t n, rt_hit* out);
/* The same query on device-resident buffers, stream-ordered (no host copies):
   d_rays [n][6] f64 and d_out [n] rt_hit in HBM.  method 0 runs one thread per
   ray; method 1 the persistent traversal (waves refill finished lanes from a
   queue), on the triangle BVH's compact layout when the scene has it and its
   tuning allows (rt_tuning.compact).  Both give identical hits.  Uses the scene's workspace, ordered
   after the scene's previous launch (Conventions: Streams). */
#define RT_TRACE_PER_RAY    0
#define RT_TRACE_PERSISTENT 1
int rt_intersect_rays_async(rt_scene* scene, const double* d_rays, uint32_t n, rt_hit* d_out, int method,
                            void* hip_stream);
/* Light-area pdf for a batch [n][6] = (surface pos, unit dir) — replaces
   ray_sampler.rs:132-139 Light::pdf (all-hits query intersections.rs:87-91). */
int rt_light_pdf_rays(rt_scene* scene, const double* pos_dir, uint32_t n, double* out_pdf);
/* The raw intersect_lights accumulation of Light::pdf for rays [n][6] used as
   given (no EPSILON offset, no 1/len): out_impact = sum over every light
   crossing of p_area * t^2/|d.n_g|; out_count = number of callbacks
   (intersections.rs:87-91; known-answer test primitives/triangle.rs:98-128). */
int rt_intersect_lights_rays(rt_scene* scene, const double* rays, uint32_t n,
                             double* out_impact, uint32_t* out_count);

/* ======================= host BVH builder ================================= */
/* BVH::new (bvh.rs:12-17, build_nodes :75-113) over primitive boxes
   [n][6] = (min xyz, max xyz) given in list order; host only, no device.
   Ties of equal midpoints are broken by list index (deterministic tree).
   Call with out_links == NULL to get *n_nodes; then with buffers of that size:
   out_links [n_nodes][4] = (left, right, start, end) (-1: none), out_bounds
   [n_nodes][6], out_order [n] = list index of the i-th primitive in BVH order. */
int rt_bvh_build(const double* boxes, uint64_t n, uint64_t* n_nodes, int64_t* out_links,
                 double* out_bounds, uint64_t* out_order, uint32_t* out_depth);

/* ======================= host input surface =============================== */
/* Custom text format (src/scene_parser.rs:5-85, defaults scene.rs:167-191). */
int rt_parse_custom_scene(const char* text, rt_parsed_scene** out);
/* glTF subset (src/gltf/parser.rs, src/gltf/scene_builder.rs:9-22); external
   .bin buffers resolved relative to the .gltf path (main.rs:54-59,77-83). */
int rt_load_gltf(const char* gltf_path, uint32_t width, uint32_t height,
                 uint32_t spp, rt_parsed_scene** out);
/* Views into the parse result (valid until rt_parsed_scene_free). */
int rt_parsed_scene_get(const rt_parsed_scene* ps, rt_scene_desc* desc,
                        rt_render_params* params);
void rt_parsed_scene_free(rt_parsed_scene* ps);

/* ======================= host output surface ============================== */
/* correct_gamma(aces_tonemap(x)) per pixel (postprocessing.rs:5-37). */
void rt_tonemap_gamma(const double* mean_rgb, uint64_t n_pixels, double* out_rgb);
/* Binary P6 PPM of an already tonemapped image (ppm.rs:4-19). */
int rt_save_ppm(const char* path, uint32_t width, uint32_t height, const double* rgb);
/* The device epilogue's table (host only): out[k-1] = the least tonemapped
   value a >= 0 whose PPM byte round(clamp(pow(a, 1/2.2))*255) is >= k, k =
   1..255, derived from this library's host pow and proven exact
   (RT_ERR_UNSUPPORTED if the proof fails). */
int rt_byte_thresholds(double* out255);

/* ======================= misc ============================================= */
const char* rt_last_error(void);
int rt_api_version(void);
/* Number of visible HIP devices (0 when none); never fails. */
int rt_device_count(void);
/* Diagnostic: device f64 sqrt (op 0), a/b (op 1), or the kernels' forms
   (rt_device.h): the split division dev_quot(a, b, dev_rcp(b)) (op 2), dev_sqrt(a)
   (op 3), dev_inv_len(a) = 1/sqrt(a) (op 4) and dev_quotf(a, b, dev_rcp(b)) (op 5,
   the split division with the signed-zero fixup), for n values, to check that the
   device rounds like the host (the bit-exact parity premise).
   b is read for ops 1, 2 and 5 only. */
int rt_probe_fp64(int op, const double* a, const double* b, uint32_t n, double* out);

#ifdef __cplusplus
}
#endif
#endif /* RT_API_H */
