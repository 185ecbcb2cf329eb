// api.cpp — the C ABI (include/rt_api.h): scene upload, frame render, tile
// partition, ray queries.  Replaces generate_image (main.rs:85-114) and the
// scene construction behind it (scene.rs:180-223).  Errors become return codes
// (the reference panics).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "../../include/rt_api.h"
#include "api_internal.h"
#include "render.h"
#include "rt_device.h"
#include "scene_build.h"

namespace rt {

static thread_local std::string g_last_error;

int set_error(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

}  // namespace rt

using namespace rt;

#define HIP_TRY(expr)                                                                         \
    do {                                                                                      \
        hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess)                                                                 \
            return set_error(e_ == hipErrorOutOfMemory ? RT_ERR_NOMEM : RT_ERR_DEVICE,        \
                             std::string(#expr) + ": " + hipGetErrorString(e_));              \
    } while (0)

struct rt_scene {
    int device = 0;
    DevScene dev{};
    std::vector<void*> allocs;
    std::vector<size_t> alloc_bytes;  // bytes of each scene array in allocs (scene_allocs: replicas)
    rt_scene_info info{};
    // spill workspace for the traversal stack (grown on demand)
    uint32_t* spill_n = nullptr;
    double* spill_t = nullptr;
    size_t spill_entries = 0;
    // chunk partial sums (KParams::chunks > 1), grown on demand
    double* part = nullptr;
    size_t part_entries = 0;
    // persistent path kernel: wave-tile queue and per-wave sample ring
    uint32_t* queue = nullptr;
    double* ring = nullptr;
    size_t ring_entries = 0;
    // rows of the queue's split tail wave-tiles (KParams::rows), grown on demand
    double* rows = nullptr;
    size_t rows_entries = 0;
    unsigned long long* d_stats = nullptr;
    // the path kernel reads the scene record and the frame constants by pointer
    DevScene* d_scene = nullptr;
    KParams* d_params = nullptr;
    // Completion of the last launch that used the workspace above (queue, ring,
    // partials, spill, d_params).  Each workspace-using launch first makes its
    // stream wait on it, then re-records it, so calls issued on different
    // streams never overlap on the shared workspace.
    hipEvent_t ws_done = nullptr;
    // bytes of the triangle BVH's compact layout (nodes + leaf blocks), 0 without one
    uint64_t compact_bytes = 0;
    uint64_t pair_bytes = 0;  // the pair layout's lines + the compact leaf blocks, 0 without one
    // requested kernel form (rt_scene_set_tuning); auto fields resolve per scene
    rt_tuning tune{0, -1, 0, 0, 0, 0, -1, 0};
    uint32_t last_tail_split = 0;  // the split the last prepared frame resolved to (0: none since set_tuning)
};

namespace {

// Set while scene_upload builds a replica (multi.cpp): the arrays are allocated
// but not copied from the host; the caller fills them device to device from the
// source scene's arrays (the same build, so the same allocation sequence).
thread_local bool g_replica = false;

template <class T>
int upload(rt_scene* s, const std::vector<T>& v, const T** out) {
    *out = nullptr;
    if (v.empty()) return RT_OK;
    void* p = nullptr;
    HIP_TRY(hipMalloc(&p, v.size() * sizeof(T)));
    s->allocs.push_back(p);
    s->alloc_bytes.push_back(v.size() * sizeof(T));
    if (!g_replica) HIP_TRY(hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    s->info.device_bytes += v.size() * sizeof(T);
    *out = (const T*)p;
    return RT_OK;
}

int upload_bvh(rt_scene* s, const HostBvhArrays& h, DevBvh& d) {
    int rc;
    std::memset(&d, 0, sizeof(d));
    if ((rc = upload(s, h.nodes, &d.nodes))) return rc;
    store3(d.root_min, h.root.min);
    store3(d.root_max, h.root.max);
    d.n_prims = h.n_prims;
    d.depth = h.depth;
    d.fast = h.fast ? 1u : 0u;
    d.tri_q = h.tri_q ? 1u : 0u;
    if ((rc = upload(s, h.shapes, &d.shapes))) return rc;
    if ((rc = upload(s, h.tris, &d.tris))) return rc;
    if ((rc = upload(s, h.tri_cold, &d.tri_cold))) return rc;
    if ((rc = upload(s, h.tri_inv_area, &d.tri_inv_area))) return rc;
    if ((rc = upload(s, h.mat, &d.mat))) return rc;
    if ((rc = upload(s, h.gid, &d.gid))) return rc;
    if ((rc = upload(s, h.cnodes, &d.cnodes))) return rc;
    if ((rc = upload(s, h.ctris, &d.ctris))) return rc;
    if ((rc = upload(s, h.pnodes, &d.pnodes))) return rc;
    return RT_OK;
}

void free_scene(rt_scene* s) {
    if (!s) return;
    int cur = 0;
    (void)hipGetDevice(&cur);
    (void)hipSetDevice(s->device);
    for (void* p : s->allocs) (void)hipFree(p);
    if (s->spill_n) (void)hipFree(s->spill_n);
    if (s->spill_t) (void)hipFree(s->spill_t);
    if (s->part) (void)hipFree(s->part);
    if (s->queue) (void)hipFree(s->queue);
    if (s->ring) (void)hipFree(s->ring);
    if (s->rows) (void)hipFree(s->rows);
    if (s->d_stats) (void)hipFree(s->d_stats);
    if (s->d_scene) (void)hipFree(s->d_scene);
    if (s->d_params) (void)hipFree(s->d_params);
    if (s->ws_done) (void)hipEventDestroy(s->ws_done);
    (void)hipSetDevice(cur);
    delete s;
}

struct SceneDeleter {
    void operator()(rt_scene* s) const { free_scene(s); }
};

// Makes the scene's device current for one entry point and restores the
// caller's current device on every return path.
struct DeviceGuard {
    int prev = -1;
    hipError_t err = hipSuccess;
    explicit DeviceGuard(int dev) {
        err = hipGetDevice(&prev);
        if (err == hipSuccess && prev != dev) err = hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};
#define DEVICE_GUARD(s)                                                                       \
    DeviceGuard guard_((s)->device);                                                          \
    if (guard_.err != hipSuccess)                                                             \
        return set_error(RT_ERR_DEVICE, std::string("hipSetDevice: ") + hipGetErrorString(guard_.err))

struct EventPair {  // hipEvent_t pair destroyed on every return path
    hipEvent_t a = nullptr, b = nullptr;
    ~EventPair() {
        if (a) (void)hipEventDestroy(a);
        if (b) (void)hipEventDestroy(b);
    }
};

// Stream ordering of the shared workspace: wait for the previous user, launch,
// then record (ws_begin / ws_end bracket every workspace-using launch).
hipError_t ws_begin(rt_scene* s, hipStream_t st) { return hipStreamWaitEvent(st, s->ws_done, 0); }
hipError_t ws_end(rt_scene* s, hipStream_t st) { return hipEventRecord(s->ws_done, st); }

int check_params(const rt_render_params* p) {
    if (!p) return set_error(RT_ERR_INVALID, "params is NULL");
    if (p->width == 0 || p->height == 0) return set_error(RT_ERR_INVALID, "width/height must be > 0");
    // the path kernel packs a wave-tile's pixel origin into 16 + 16 bits (render.hip store_unit)
    if (p->width > 65535 || p->height > 65535) return set_error(RT_ERR_INVALID, "width/height must be <= 65535");
    if (p->spp == 0) return set_error(RT_ERR_INVALID, "spp must be > 0");
    if (p->ray_depth > 255) return set_error(RT_ERR_INVALID, "ray_depth is a u8 in the reference (scene.rs:85)");
    if (p->fov_axis != RT_FOV_X && p->fov_axis != RT_FOV_Y) return set_error(RT_ERR_INVALID, "bad fov_axis");
    return RT_OK;
}

// Sample chunking of a frame (render.h sample_chunks); a scene's tuning may
// force the run length (rt_tuning.chunk_spp, tests and tuning experiments;
// rt_scene_sample_chunks reports it, so checkers stay consistent).  A forced run
// length is raised, if need be, to keep the frame's rule's limits: at most
// kMaxChunks runs, and the chunk partial sums within kPartBytes.
void frame_chunks(const rt_render_params* p, uint32_t force_spp, uint32_t& chunks, uint32_t& chunk_spp) {
    sample_chunks(p->width, p->height, p->spp, chunks, chunk_spp);
    if (force_spp > 0) {
        const uint64_t chunk_bytes =
            (uint64_t)((p->width + 15) / 16) * ((p->height + 15) / 16) * 256 * 3 * sizeof(double);
        const uint64_t max_chunks = std::max<uint64_t>(1, std::min<uint64_t>(kMaxChunks, kPartBytes / chunk_bytes));
        const uint32_t floor_spp = (uint32_t)((p->spp + max_chunks - 1) / max_chunks);
        chunk_spp = std::min(std::max(force_spp, floor_spp), p->spp);
        chunks = (p->spp + chunk_spp - 1) / chunk_spp;
    }
}

// Camera::new (camera.rs:17-46) on the host + the tile map of one rank.
KParams make_kparams(const rt_render_params* p, uint32_t rank, uint32_t world, uint32_t force_spp = 0) {
    KParams k;
    std::memset(&k, 0, sizeof(k));
    k.width = p->width; k.height = p->height; k.spp = p->spp; k.ray_depth = p->ray_depth;
    k.fw = (double)p->width; k.fh = (double)p->height;
    k.inv_fw = 1.0 / k.fw; k.inv_fh = 1.0 / k.fh;
    if (p->fov_axis == RT_FOV_Y) {
        k.tan_y = std::tan(p->fov / 2.0);
        double aspect = k.fh / k.fw;
        k.tan_x = k.tan_y / aspect;
    } else {
        k.tan_x = std::tan(p->fov / 2.0);
        double aspect = k.fw / k.fh;
        k.tan_y = k.tan_x / aspect;
    }
    for (int i = 0; i < 3; ++i) {
        k.cam_pos[i] = p->cam_position[i]; k.cam_right[i] = p->cam_right[i];
        k.cam_up[i] = p->cam_up[i]; k.cam_fwd[i] = p->cam_forward[i]; k.bg[i] = p->bg_color[i];
    }
    k.scale01 = inclusive_scale(0.0, 1.0);
    k.scale11 = inclusive_scale(-1.0, 1.0);
    k.seed = p->seed;
    k.rank = rank; k.world = world;
    k.tiles_x = (p->width + RT_TILE - 1) / RT_TILE;
    k.tiles_y = (p->height + RT_TILE - 1) / RT_TILE;
    k.n_tiles = (uint64_t)k.tiles_x * k.tiles_y;
    k.n_slots = (uint32_t)((k.n_tiles + world - 1) / world);
    frame_chunks(p, force_spp, k.chunks, k.chunk_spp);
    return k;
}

uint32_t slots_per_rank(const KParams& k) { return k.n_slots; }

// Before a workspace buffer is regrown: the last launch that used it is done.
int ws_idle(rt_scene* s) {
    HIP_TRY(hipEventSynchronize(s->ws_done));
    return RT_OK;
}

int ensure_part(rt_scene* s, const KParams& k) {
    if (k.chunks == 1) return RT_OK;
    const size_t need = (size_t)k.n_slots * k.chunks * 256 * 3;
    if (need <= s->part_entries) return RT_OK;
    if (int rc = ws_idle(s)) return rc;
    if (s->part) (void)hipFree(s->part);
    s->part = nullptr; s->part_entries = 0;
    HIP_TRY(hipMalloc(&s->part, need * sizeof(double)));
    s->part_entries = need;
    return RT_OK;
}

// Spill area for stack entries beyond the LDS short stack: depth bound of the
// deepest BVH, one slot per launched lane (`no_lds`: a kernel without an LDS
// stack, the 4/5-wave shape-only fused kernel, spills every entry).
int ensure_spill(rt_scene* s, uint64_t lanes, bool no_lds = false) {
    uint32_t depth = s->dev.max_depth;
    const uint32_t lds = no_lds ? 0u : (uint32_t)kMinShort;
    if (depth <= lds) return RT_OK;
    size_t need = (size_t)(depth - lds) * lanes;
    if (need <= s->spill_entries) return RT_OK;
    if (int rc = ws_idle(s)) return rc;
    if (s->spill_n) (void)hipFree(s->spill_n);
    if (s->spill_t) (void)hipFree(s->spill_t);
    s->spill_n = nullptr; s->spill_t = nullptr; s->spill_entries = 0;
    HIP_TRY(hipMalloc(&s->spill_n, need * sizeof(uint32_t)));
    HIP_TRY(hipMalloc(&s->spill_t, need * sizeof(double)));
    s->spill_entries = need;
    return RT_OK;
}

// Register budget of the path kernel for this scene.  Large BVHs make the loop
// latency-bound on dependent node loads, where a 4th wave per SIMD hides more
// than its register spill costs (C3: -9%).  Shape-only scenes with small shape
// BVHs run the fused kernel's shape-only instance at kShapeWaves (round 4: the
// path's T and L in LDS and no LDS stack take it to 128 VGPRs without spill, and
// a 5th wave hides more than its 42 VGPRs of spill cost).  That
// instance has no LDS stack: every push of a BVH walk goes to the global spill
// stack, which a single-leaf BVH (the Cornell box's) never touches; so a
// shape-only scene whose BVHs hold more than kShapeWavesNodes nodes runs the
// 3-wave instance, whose 12-entry LDS stack takes the pushes (round 5, advisor
// finding; measured in DESIGN.md §4).  Other small scenes run the general fused
// instance at 3.  rt_tuning.waves forces one (tests, tuning); 5 exists for the
// shape-only fused form only (other forms take 4).
bool path_resume(const rt_scene* s);
int path_kinds(const rt_scene* s);
uint32_t path_waves(const rt_scene* s) {
    const bool shape_fused = path_kinds(s) == 1 && !path_resume(s);
    if (s->tune.waves) return s->tune.waves == 5 && !shape_fused ? 4u : s->tune.waves;
    uint64_t nodes = 0;
    for (int k = 0; k < 6; ++k) nodes += s->info.bvh_nodes[k];
    if (shape_fused) return nodes <= kShapeWavesNodes ? kShapeWaves : 3u;
    return nodes > kDeepSceneNodes ? 4u : 3u;
}

// Resumable triangle traversal (path_kernel RES) for scenes with a
// deep triangle BVH, where a wave's traversal loop otherwise runs most trips
// with few live lanes (C3: 43%); scenes without one keep the fused segment,
// which carries less state across the loop (C2: 113 vs 130 ms at 64 spp).
// rt_tuning.resume forces one (tests, tuning).
bool path_resume(const rt_scene* s) {
    if (s->tune.resume >= 0) return s->tune.resume == 1;
    return s->info.bvh_nodes[2] > kDeepSceneNodes;
}

// The scene's primitive kinds: 1 = shapes (planes, boxes, ellipsoids), 2 =
// triangles, 3 = both (or neither).  One-kind scenes run kernel instances with no
// code or state for the other kind: triangle-only ones (every glTF scene) the
// 4-wave resumable kernel without a shape candidate carried across its loop
// (C3 -6%), shape-only ones (the Cornell box) the fused kernel without triangle
// traversal.  rt_tuning.kinds = 3 forces the general instances (tests, tuning).
int scene_kinds(const DevScene& d) {
    const bool shapes = d.n_planes || d.boxes.n_prims || d.ells.n_prims || d.lboxes.n_prims || d.lells.n_prims;
    const bool tris = d.tris.n_prims || d.ltris.n_prims;
    return shapes == tris ? 3 : (shapes ? 1 : 2);
}
int path_kinds(const rt_scene* s) { return s->tune.kinds == 3 ? 3 : scene_kinds(s->dev); }

// The triangle BVH's compact layout (rt_layout.h DevNodeC, half the bytes per
// node visit and triangle test, the same numbers): used by the triangle-only
// 4-wave resumable instance — the kernel of every deep glTF scene — whenever the
// host could build it (every coordinate an exact f32).  rt_tuning.compact = 0
// keeps the f64 layout (tests run both).
bool path_compact(const rt_scene* s) {
    return s->tune.compact != 0 && s->dev.tris.cnodes && path_waves(s) == 4 && path_resume(s) && path_kinds(s) == 2;
}
// The pair layout over the compact nodes (rt_layout.h kPairFloats, render.hip trav_step
// PAIR: two BVH levels per dependent line), whenever the scene has it (auto, or
// rt_tuning.compact = 2; 1 forces the 64-B compact nodes): C3 -3.5%, C5 -2.0% in
// alternating runs, the same images and counters (profiles/r06/variants_pair2_C*.log,
// DESIGN.md §4).
bool path_pairs(const rt_scene* s) {
    return (s->tune.compact == -1 || s->tune.compact == 2) && s->dev.tris.pnodes && path_compact(s);
}



// Suspend threshold of the resumable traversal (render.h kSuspendCached /
// kSuspendStreamed): by whether the triangle BVH and its hot records fit the
// Infinity Cache.  rt_tuning.suspend_lanes forces one (tuning).
// The triangle BVH and its hot records exceed the Infinity Cache, sized by the
// layout the kernel reads (path_compact: 64-B nodes and 36-B records, else 128 B
// and 80 B).
uint64_t bvh_hot_bytes(const rt_scene* s) {
    if (path_pairs(s)) return s->pair_bytes;
    if (path_compact(s)) return s->compact_bytes;
    return s->info.bvh_nodes[2] * sizeof(DevNode) + s->info.n_triangles * sizeof(DevTri);
}
bool bvh_streamed(const rt_scene* s) { return bvh_hot_bytes(s) > kCacheBytes; }
uint32_t path_suspend(const rt_scene* s) {
    if (s->tune.suspend_lanes) return s->tune.suspend_lanes;
    if (path_compact(s)) return bvh_streamed(s) ? kSuspendCoopStreamed : kSuspendCoopCached;  // leaf_coop
    return bvh_streamed(s) ? kSuspendStreamed : kSuspendCached;
}

// Leaf batch of the resumable traversal (render.hip trav_step: lanes waiting at
// leaves before the wave tests them), by the same cache criterion as the suspend
// threshold (render.h kLeafCached / kLeafStreamed; the compact layout's kernel, whose
// small leaves are tested cooperatively, kLeafCoop*).  rt_tuning.leaf_lanes forces one.
uint32_t path_leaf_batch(const rt_scene* s) {
    if (s->tune.leaf_lanes) return s->tune.leaf_lanes;
    if (path_compact(s)) return bvh_streamed(s) ? kLeafCoopStreamed : kLeafCoopCached;
    return bvh_streamed(s) ? kLeafStreamed : kLeafCached;
}

// Workspace of one path-kernel launch: persistent grid size, then the spill,
// ring and chunk-partial buffers sized for it (all grow-only, scene-owned).
int prepare_path(rt_scene* s, KParams& k, bool stats, bool hits, PathWork& W) {
    k.suspend = path_suspend(s);
    k.leaf_batch = path_leaf_batch(s);
    const uint64_t n_units = (uint64_t)k.n_slots * k.chunks * 4;
    if (n_units >= (1ull << 31)) return set_error(RT_ERR_INVALID, "frame too large for one launch");
    std::memset(&W, 0, sizeof(W));
    W.waves = path_waves(s);
    W.resume = path_resume(s);
    W.kinds = path_pairs(s) ? kKindsPair : (path_compact(s) ? kKindsCompact : path_kinds(s));
    HIP_TRY(path_grid(stats, hits, W.waves, W.resume, W.kinds, (uint32_t)n_units, &W.grid));
    const uint64_t lanes = (uint64_t)W.grid * 64u;
    int rc;
    // the 4/5-wave shape-only fused kernel has no LDS stack
    const bool no_lds = W.waves >= 4 && !W.resume && W.kinds == 1;
    if ((rc = ensure_spill(s, lanes, no_lds)) || (rc = ensure_part(s, k))) return rc;
    if (!s->queue) HIP_TRY(hipMalloc(&s->queue, kQueueWords * sizeof(uint32_t)));
    const size_t ring_need = (size_t)W.grid * kRingRows * 64 * 3;
    if (ring_need > s->ring_entries) {
        if (int rc2 = ws_idle(s)) return rc2;
        if (s->ring) (void)hipFree(s->ring);
        s->ring = nullptr; s->ring_entries = 0;
        HIP_TRY(hipMalloc(&s->ring, ring_need * sizeof(double)));
        s->ring_entries = ring_need;
    }
    // The queue's tail (render.hip queue_entry): the last wave-tiles —
    // kTailPerWave per resident wave, so a wave that took the last whole one finishes it
    // while the others still take parts — handed out in kTailSplit parts, so the launch
    // does not wait a whole wave-tile's time for the waves that took the last ones.
    // Capped at 256 MB of row buffer; rt_tuning.tail_split forces the split (1: whole
    // wave-tiles).
    const uint32_t split = s->tune.tail_split ? s->tune.tail_split : kTailSplit;
    uint64_t tail = 0;
    if (split > 1 && k.chunk_spp < (1u << 16)) {
        const uint64_t per_unit = (uint64_t)k.chunk_spp * 64 * 3;  // doubles
        tail = std::min<uint64_t>({n_units, (uint64_t)W.grid * kTailPerWave, (kTailRowBytes / 8) / per_unit});
        if (tail * per_unit > s->rows_entries) {
            if (int rc2 = ws_idle(s)) return rc2;
            if (s->rows) (void)hipFree(s->rows);
            s->rows = nullptr; s->rows_entries = 0;
            HIP_TRY(hipMalloc(&s->rows, tail * per_unit * sizeof(double)));
            s->rows_entries = tail * per_unit;
        }
    }
    k.n_tail = (uint32_t)tail;
    k.tail_split = tail ? split : 1u;
    s->last_tail_split = k.tail_split;  // rt_scene_get_tuning reports what the frame resolved to
    k.rows = s->rows;
    W.queue = s->queue; W.ring = s->ring; W.part = s->part;
    W.d_scene = s->d_scene; W.d_params = s->d_params;
    W.spill_n = s->spill_n; W.spill_t = s->spill_t;
    return RT_OK;
}

// device counters (render.hip wave_flush order) -> rt_stats (timings untouched)
int copy_stats(rt_scene* s, rt_stats* out) {
    unsigned long long c[kStatStall + 1];
    HIP_TRY(hipMemcpy(c, s->d_stats, sizeof(c), hipMemcpyDeviceToHost));
    // the stats instance's progress guard (render.h kStatStall): a wave that looped
    // without progress exited early, so the frame is incomplete — fail loudly
    if (c[kStatStall])
        return set_error(RT_ERR_DEVICE, "path kernel: " + std::to_string(c[kStatStall]) + " wave(s) made no progress "
                                        "for " + std::to_string(kStallTrips) + " loop trips (livelock guard)");
    out->paths = c[0]; out->segments = c[1]; out->aabb_tests = c[2]; out->tri_tests = c[3];
    out->shape_tests = c[4]; out->shaded_hits = c[5]; out->light_queries = c[6]; out->light_hits = c[7];
    out->lane_steps = c[8]; out->wave_steps = c[9];
    return RT_OK;
}

// DevScene::slt_mask: the scene boxes (BVH order) that are the light boxes, in
// order, when the light pdf can come from the closest-hit box tests (render.hip
// boxes_slt): only box lights, both box BVHs single leaves (bvh.rs:77), and the
// light copies (scene.rs:209-213) byte-identical to the selected scene records.
uint32_t slt_mask(const HostScene& hs) {
    const auto &B = hs.bvh[0], &L = hs.bvh[3];
    if (L.shapes.empty() || !hs.bvh[4].shapes.empty() || !hs.bvh[5].tris.empty()) return 0;
    if (B.depth != 1 || L.depth != 1 || B.shapes.size() > 32) return 0;
    uint32_t mask = 0;
    size_t j = 0;
    for (size_t i = 0; i < B.shapes.size() && j < L.shapes.size(); ++i)
        if (std::memcmp(&B.shapes[i], &L.shapes[j], sizeof(DevShape)) == 0) { mask |= 1u << i; ++j; }
    return j == L.shapes.size() ? mask : 0;
}

// DevScene::lq_boxes / lq_box: the light boxes' world-space bounds, grown by a
// margin of 1e-6 of the coordinates' magnitude (+1e-100) that dwarfs the rounding
// of the model-space map and of the query's slab arithmetic.  model_ray maps a
// world point p to M (p - pos) with M = x -> rotate(conj(rot), x), cgmath's
// rotate_vector: for a quaternion of norm n = |rot|^2 that is n R^T + (1 - n) I,
// a rotation only when n == 1 (the parser, like the reference, does not
// normalise ROTATION).  The box surface is therefore pos + M^-1 (+-half sizes):
// the eight corners come through the inverse of M, built from rotate() on the
// basis vectors and inverted here.  Zero (no skipping) unless every light is a
// box, there are at most kLqBoxes, every box and density is finite and positive,
// and M is well conditioned (n within 10% of 1, the inverse checked).
uint32_t lq_boxes(const HostScene& hs, double (*out)[6]) {
    const auto& L = hs.bvh[3].shapes;
    if (L.empty() || L.size() > kLqBoxes || !hs.bvh[4].shapes.empty() || !hs.bvh[5].tris.empty()) return 0;
    for (size_t i = 0; i < L.size(); ++i) {
        const DevShape& b = L[i];
        const double pb = b.aux[0];
        if (!(pb > 0.0) || !std::isfinite(pb)) return 0;
        const Quat q = load_quat(b.rot);
        const double n = q.s * q.s + dot(q.v, q.v);
        if (!(std::fabs(n - 1.0) <= 0.1)) return 0;
        const Quat c = conjugate(q);
        double M[3][3], Mi[3][3];
        for (int k = 0; k < 3; ++k) {  // column k = M e_k
            const V3 col = rotate(c, v3(k == 0, k == 1, k == 2));
            M[0][k] = col.x; M[1][k] = col.y; M[2][k] = col.z;
        }
        const double det = M[0][0] * (M[1][1] * M[2][2] - M[1][2] * M[2][1]) -
                           M[0][1] * (M[1][0] * M[2][2] - M[1][2] * M[2][0]) +
                           M[0][2] * (M[1][0] * M[2][1] - M[1][1] * M[2][0]);
        if (!(std::fabs(det) > 0.5)) return 0;
        for (int r = 0; r < 3; ++r)
            for (int k = 0; k < 3; ++k) {  // adjugate / det
                const int r1 = (k + 1) % 3, r2 = (k + 2) % 3, c1 = (r + 1) % 3, c2 = (r + 2) % 3;
                Mi[r][k] = (M[r1][c1] * M[r2][c2] - M[r1][c2] * M[r2][c1]) / det;
            }
        for (int r = 0; r < 3; ++r)  // M Mi == I to 1e-12
            for (int k = 0; k < 3; ++k) {
                const double e = M[r][0] * Mi[0][k] + M[r][1] * Mi[1][k] + M[r][2] * Mi[2][k];
                if (!(std::fabs(e - (r == k ? 1.0 : 0.0)) <= 1e-12)) return 0;
            }
        V3 lo = v3(INFINITY, INFINITY, INFINITY), hi = v3(-INFINITY, -INFINITY, -INFINITY);
        for (int k = 0; k < 8; ++k) {
            const double h[3] = {(k & 1) ? b.shape[0] : -b.shape[0], (k & 2) ? b.shape[1] : -b.shape[1],
                                 (k & 4) ? b.shape[2] : -b.shape[2]};
            const V3 p = load3(b.pos) + v3(Mi[0][0] * h[0] + Mi[0][1] * h[1] + Mi[0][2] * h[2],
                                           Mi[1][0] * h[0] + Mi[1][1] * h[1] + Mi[1][2] * h[2],
                                           Mi[2][0] * h[0] + Mi[2][1] * h[1] + Mi[2][2] * h[2]);
            lo = v3(std::min(lo.x, p.x), std::min(lo.y, p.y), std::min(lo.z, p.z));
            hi = v3(std::max(hi.x, p.x), std::max(hi.y, p.y), std::max(hi.z, p.z));
        }
        const double mag = std::max({std::fabs(lo.x), std::fabs(lo.y), std::fabs(lo.z), std::fabs(hi.x),
                                     std::fabs(hi.y), std::fabs(hi.z)});
        if (!std::isfinite(mag) || mag > 0x1p400) return 0;
        const double m = 1e-6 * (1.0 + mag) + 1e-100;
        const double v[6] = {lo.x - m, lo.y - m, lo.z - m, hi.x + m, hi.y + m, hi.z + m};
        for (int k = 0; k < 6; ++k) out[i][k] = v[k];
    }
    return (uint32_t)L.size();
}

template <class T>
struct DevBuf {  // RAII device buffer for per-call scratch
    T* p = nullptr;
    ~DevBuf() { if (p) (void)hipFree(p); }
    hipError_t alloc(size_t n) { return hipMalloc((void**)&p, (n ? n : 1) * sizeof(T)); }
};

}  // namespace

extern "C" {

const char* rt_last_error(void) { return g_last_error.c_str(); }
int rt_api_version(void) { return RT_API_VERSION; }
int rt_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int rt_scene_create(const rt_scene_desc* desc, rt_scene** out) {
    if (!desc || !out) return set_error(RT_ERR_INVALID, "desc/out is NULL");
    *out = nullptr;
    HostScene hs;
    const int rc = rt::scene_build_host(*desc, hs);
    return rc ? rc : rt::scene_upload(hs, out, false);
}

}  // extern "C"

namespace rt {

int scene_build_host(const rt_scene_desc& desc, HostScene& hs) {
    std::string err = build_scene(desc, hs);
    if (!err.empty()) return set_error(RT_ERR_INVALID, err);
    for (int k = 0; k < 6; ++k)  // traversal stack words carry node indices in 30 bits (render.hip child_word)
        if (hs.bvh[k].nodes.size() >= (1u << 30)) return set_error(RT_ERR_INVALID, "BVH exceeds 2^30 nodes");
    return RT_OK;
}

// Scene::new's device side: the flattened scene on the CURRENT HIP device.
// replica: allocate every scene array but copy none from the host (multi.cpp
// fills them from devices[0]'s copy over xGMI, scene_allocs); the small records
// (DevScene, stats) are still written here.
int scene_upload(const HostScene& hs, rt_scene** out, bool replica) {
    *out = nullptr;
    struct ReplicaFlag {
        explicit ReplicaFlag(bool r) { g_replica = r; }
        ~ReplicaFlag() { g_replica = false; }
    } flag(replica);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return set_error(RT_ERR_DEVICE, "no HIP device visible (the hot path has no CPU fallback)");
    std::unique_ptr<rt_scene, SceneDeleter> owner(new rt_scene());  // frees everything on an error return
    rt_scene* s = owner.get();
    HIP_TRY(hipGetDevice(&s->device));
    HIP_TRY(hipEventCreateWithFlags(&s->ws_done, hipEventDisableTiming));
    auto t0 = std::chrono::steady_clock::now();
    int rc = RT_OK;
    DevScene& d = s->dev;
    d.n_planes = (uint32_t)hs.planes.size();
    if ((rc = upload(s, hs.planes, &d.planes)) || (rc = upload(s, hs.plane_mat, &d.plane_mat)) ||
        (rc = upload(s, hs.plane_gid, &d.plane_gid)) || (rc = upload(s, hs.mats, &d.mats)) ||
        (rc = upload_bvh(s, hs.bvh[0], d.boxes)) || (rc = upload_bvh(s, hs.bvh[1], d.ells)) ||
        (rc = upload_bvh(s, hs.bvh[2], d.tris)) || (rc = upload_bvh(s, hs.bvh[3], d.lboxes)) ||
        (rc = upload_bvh(s, hs.bvh[4], d.lells)) || (rc = upload_bvh(s, hs.bvh[5], d.ltris)))
        return rc;
    // ellipsoid reciprocals for dev_quot: computed by the device's own rcp + Newton steps
    // (a replica receives the source's records with them already written)
    if (!replica) {
        HIP_TRY(launch_ell_rcp(const_cast<DevShape*>(d.ells.shapes), d.ells.n_prims, 0));
        HIP_TRY(launch_ell_rcp(const_cast<DevShape*>(d.lells.shapes), d.lells.n_prims, 0));
        HIP_TRY(hipStreamSynchronize(0));
    }
    {  // world normals of plane sides and box faces: rotated(Hit, rot) of render.hip materialise
        std::vector<double> pn(hs.planes.size() * 6), bn(hs.bvh[0].shapes.size() * 24, 0.0);
        for (size_t i = 0; i < hs.planes.size(); ++i) {
            const DevShape& p = hs.planes[i];
            const Quat q = load_quat(p.rot);
            for (int side = 0; side < 2; ++side)
                store3(&pn[i * 6 + side * 3], normalize(rotate(q, load3(p.shape) * (side ? 1.0 : -1.0))));
        }
        for (size_t i = 0; i < hs.bvh[0].shapes.size(); ++i) {
            const Quat q = load_quat(hs.bvh[0].shapes[i].rot);
            for (uint32_t a = 0; a < 8; ++a) {
                if ((a & 3u) == 3u) continue;
                const double sg = (a & 4u) ? 1.0 : -1.0;
                const uint32_t dim = a & 3u;
                const V3 n = dim == 0 ? v3(sg, 0.0, 0.0) : dim == 1 ? v3(0.0, sg, 0.0) : v3(0.0, 0.0, sg);
                store3(&bn[i * 24 + a * 3], normalize(rotate(q, n)));
            }
        }
        if ((rc = upload(s, pn, &d.plane_nrm)) || (rc = upload(s, bn, &d.box_nrm))) return rc;
    }
    d.n_lights = d.lboxes.n_prims + d.lells.n_prims + d.ltris.n_prims;
    // UINT64_MAX - (2^64 - n) % n (oracle.c usize_zone); unused without lights
    d.light_zone = d.n_lights ? UINT64_MAX - (0ull - (uint64_t)d.n_lights) % (uint64_t)d.n_lights : 0;
    d.slt_mask = slt_mask(hs);
    std::memset(d.lq_box, 0, sizeof(d.lq_box));
    d.lq_boxes = lq_boxes(hs, d.lq_box);
    d.max_depth = 0;
    const DevBvh* all[6] = {&d.boxes, &d.ells, &d.tris, &d.lboxes, &d.lells, &d.ltris};
    for (int k = 0; k < 6; ++k) {
        d.max_depth = std::max(d.max_depth, all[k]->depth);
        s->info.bvh_nodes[k] = hs.bvh[k].nodes.size();
        s->info.bvh_depth[k] = hs.bvh[k].depth;
    }
    HIP_TRY(hipMalloc(&s->d_scene, sizeof(DevScene)));
    HIP_TRY(hipMemcpy(s->d_scene, &s->dev, sizeof(DevScene), hipMemcpyHostToDevice));
    HIP_TRY(hipMalloc(&s->d_params, sizeof(KParams)));
    HIP_TRY(hipMalloc(&s->d_stats, kStatsWords * sizeof(unsigned long long)));
    HIP_TRY(hipMemset(s->d_stats, 0, kStatsWords * sizeof(unsigned long long)));
    s->info.n_planes = d.n_planes;
    s->info.n_boxes = d.boxes.n_prims;
    s->info.n_ellipsoids = d.ells.n_prims;
    s->info.n_triangles = d.tris.n_prims;
    s->info.n_light_boxes = d.lboxes.n_prims;
    s->info.n_light_ellipsoids = d.lells.n_prims;
    s->info.n_light_triangles = d.ltris.n_prims;
    s->info.shared_light_mask = d.slt_mask;
    s->compact_bytes = hs.bvh[2].cnodes.size() * sizeof(DevNodeC) + hs.bvh[2].ctris.size() * sizeof(float);
    s->pair_bytes = (hs.bvh[2].pnodes.size() + hs.bvh[2].ctris.size()) * sizeof(float);
    s->info.layout_flags = (d.tris.cnodes ? RT_LAYOUT_COMPACT_TRIS : 0u) | (d.lq_boxes ? RT_LAYOUT_LQ_SKIP : 0u) |
                           (d.tris.pnodes ? RT_LAYOUT_PAIR_NODES : 0u);
    s->info.build_ms = hs.build_ms;
    s->info.upload_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    *out = owner.release();
    return RT_OK;
}

const std::vector<void*>& scene_allocs(const rt_scene* s, const std::vector<size_t>** bytes) {
    *bytes = &s->alloc_bytes;
    return s->allocs;
}
void scene_add_upload_ms(rt_scene* s, double ms) { s->info.upload_ms += ms; }

}  // namespace rt

extern "C" {

void rt_scene_destroy(rt_scene* s) { free_scene(s); }

int rt_scene_get_info(const rt_scene* s, rt_scene_info* out) {
    if (!s || !out) return set_error(RT_ERR_INVALID, "scene/out is NULL");
    *out = s->info;
    return RT_OK;
}

int rt_tiles_per_rank(const rt_render_params* p, uint32_t world, uint32_t* n) {
    int rc = check_params(p);
    if (rc) return rc;
    if (world == 0 || !n) return set_error(RT_ERR_INVALID, "world must be > 0");
    *n = slots_per_rank(make_kparams(p, 0, world));
    return RT_OK;
}

int rt_sample_chunks(const rt_render_params* p, uint32_t* chunks, uint32_t* chunk_spp) {
    int rc = check_params(p);
    if (rc) return rc;
    if (!chunks || !chunk_spp) return set_error(RT_ERR_INVALID, "output is NULL");
    frame_chunks(p, 0, *chunks, *chunk_spp);
    return RT_OK;
}

int rt_scene_sample_chunks(const rt_scene* s, const rt_render_params* p, uint32_t* chunks, uint32_t* chunk_spp) {
    int rc = check_params(p);
    if (rc) return rc;
    if (!s || !chunks || !chunk_spp) return set_error(RT_ERR_INVALID, "scene/output is NULL");
    frame_chunks(p, s->tune.chunk_spp, *chunks, *chunk_spp);
    return RT_OK;
}

int rt_scene_set_tuning(rt_scene* s, const rt_tuning* t) {
    if (!s) return set_error(RT_ERR_INVALID, "scene is NULL");
    if (!t) { s->tune = rt_tuning{0, -1, 0, 0, 0, 0, -1, 0}; s->last_tail_split = 0; return RT_OK; }
    if (t->waves != 0 && (t->waves < 3 || t->waves > 5)) return set_error(RT_ERR_INVALID, "waves must be 0, 3, 4 or 5");
    if (t->resume < -1 || t->resume > 1) return set_error(RT_ERR_INVALID, "resume must be -1, 0 or 1");
    if (t->kinds > 3) return set_error(RT_ERR_INVALID, "kinds must be 0..3");
    // 1 / 2 (what rt_scene_get_tuning reports for a one-kind scene): only the scene's own kinds
    if ((t->kinds == 1 || t->kinds == 2) && (int)t->kinds != scene_kinds(s->dev))
        return set_error(RT_ERR_INVALID, "kinds 1/2 must be the scene's own primitive kinds (0 or 3 otherwise)");
    if (t->suspend_lanes > 64 || t->leaf_lanes > 64) return set_error(RT_ERR_INVALID, "lane counts must be <= 64");
    if (t->compact < -1 || t->compact > 2) return set_error(RT_ERR_INVALID, "compact must be -1, 0, 1 or 2");
    if (t->compact >= 1 && !s->dev.tris.cnodes)
        return set_error(RT_ERR_UNSUPPORTED, "compact >= 1: the scene has no compact triangle layout");
    if (t->compact == 2 && !s->dev.tris.pnodes)
        return set_error(RT_ERR_UNSUPPORTED, "compact = 2: the scene has no pair layout");
    if (t->tail_split > 8) return set_error(RT_ERR_INVALID, "tail_split must be 0..8");
    s->tune = *t;
    s->last_tail_split = 0;
    return RT_OK;
}

int rt_scene_checksum(rt_scene* s, uint64_t* out) {
    if (!s || !out) return set_error(RT_ERR_INVALID, "scene/out is NULL");
    DEVICE_GUARD(s);
    const size_t n = s->allocs.size();
    DevBuf<unsigned long long> sums;
    HIP_TRY(sums.alloc(std::max<size_t>(n, 1)));
    for (size_t k = 0; k < n; ++k) HIP_TRY(launch_checksum(s->allocs[k], s->alloc_bytes[k], sums.p + k, 0));
    std::vector<unsigned long long> h(n);
    HIP_TRY(hipDeviceSynchronize());
    if (n) HIP_TRY(hipMemcpy(h.data(), sums.p, n * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    uint64_t acc = 0xcbf29ce484222325ull;  // arrays in allocation order, each with its size
    for (size_t k = 0; k < n; ++k) acc = (acc ^ (h[k] + 0x9e3779b97f4a7c15ull * s->alloc_bytes[k])) * 0x100000001b3ull;
    *out = acc;
    return RT_OK;
}

int rt_scene_get_tuning(const rt_scene* s, rt_tuning* out) {
    if (!s || !out) return set_error(RT_ERR_INVALID, "scene/out is NULL");
    out->waves = path_waves(s);
    out->resume = path_resume(s) ? 1 : 0;
    out->kinds = (uint32_t)path_kinds(s);
    out->suspend_lanes = path_suspend(s);
    out->leaf_lanes = path_leaf_batch(s);
    out->chunk_spp = s->tune.chunk_spp;
    out->compact = path_pairs(s) ? 2 : (path_compact(s) ? 1 : 0);
    out->tail_split = s->last_tail_split ? s->last_tail_split : (s->tune.tail_split ? s->tune.tail_split : kTailSplit);
    return RT_OK;
}

int rt_render_tiles_async(rt_scene* s, const rt_render_params* p, uint32_t rank, uint32_t world,
                          double* d_tile_rgb, void* stream) {
    int rc = check_params(p);
    if (rc) return rc;
    if (!s || !d_tile_rgb) return set_error(RT_ERR_INVALID, "scene/output is NULL");
    if (world == 0 || rank >= world) return set_error(RT_ERR_INVALID, "rank must be < world");
    DEVICE_GUARD(s);
    KParams k = make_kparams(p, rank, world, s->tune.chunk_spp);
    const bool want_stats = (p->flags & RT_FLAG_STATS) != 0;
    PathWork W;
    if ((rc = prepare_path(s, k, want_stats, false, W))) return rc;
    const hipStream_t st = (hipStream_t)stream;
    HIP_TRY(ws_begin(s, st));
    HIP_TRY(launch_path(s->dev, k, W, d_tile_rgb, nullptr, want_stats ? s->d_stats : nullptr, st));
    HIP_TRY(ws_end(s, st));
    return RT_OK;
}

int rt_read_stats(rt_scene* s, rt_stats* out, int reset) {
    if (!s || !out) return set_error(RT_ERR_INVALID, "scene/out is NULL");
    DEVICE_GUARD(s);
    HIP_TRY(hipDeviceSynchronize());
    std::memset(out, 0, sizeof(*out));
    int rc = copy_stats(s, out);
    if (rc) return rc;
    if (reset) HIP_TRY(hipMemset(s->d_stats, 0, kStatsWords * sizeof(unsigned long long)));
    return RT_OK;
}

int rt_read_raw_stats(rt_scene* s, uint64_t* out, uint32_t n) {
    if (!s || !out || n > (uint32_t)kStatsWords) return set_error(RT_ERR_INVALID, "scene/out NULL or n > 64");
    DEVICE_GUARD(s);
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(out, s->d_stats, n * sizeof(uint64_t), hipMemcpyDeviceToHost));
    return RT_OK;
}

int rt_unpack_tiles_async(const rt_render_params* p, uint32_t world, const double* d_gathered, double* d_image,
                          void* stream) {
    int rc = check_params(p);
    if (rc) return rc;
    if (!d_gathered || !d_image || world == 0) return set_error(RT_ERR_INVALID, "bad unpack arguments");
    KParams k = make_kparams(p, 0, world);
    HIP_TRY(launch_unpack(d_gathered, d_image, p->width, p->height, k.tiles_x, world, slots_per_rank(k),
                          (hipStream_t)stream));
    return RT_OK;
}

int rt_unpack_tiles_bytes_async(const rt_render_params* p, uint32_t world, const double* d_gathered,
                                uint8_t* d_bytes, void* stream) {
    int rc = check_params(p);
    if (rc) return rc;
    if (!d_gathered || !d_bytes || world == 0) return set_error(RT_ERR_INVALID, "bad unpack arguments");
    KParams k = make_kparams(p, 0, world);
    HIP_TRY(launch_unpack_bytes(d_gathered, d_bytes, p->width, p->height, k.tiles_x, world, slots_per_rank(k),
                                (hipStream_t)stream));
    return RT_OK;
}

int rt_tonemap_bytes_async(const double* d_rgb, uint64_t n_pixels, uint8_t* d_bytes, void* stream) {
    if ((!d_rgb || !d_bytes) && n_pixels) return set_error(RT_ERR_INVALID, "rgb/bytes is NULL");
    HIP_TRY(launch_tonemap_bytes(d_rgb, 3 * n_pixels, d_bytes, (hipStream_t)stream));
    return RT_OK;
}

int rt_render(rt_scene* s, const rt_render_params* p, double* out_mean_rgb, int32_t* opt_hit_ids,
              rt_stats* opt_stats) {
    auto t0 = std::chrono::steady_clock::now();
    int rc = check_params(p);
    if (rc) return rc;
    if (!s || !out_mean_rgb) return set_error(RT_ERR_INVALID, "scene/output is NULL");
    DEVICE_GUARD(s);
    KParams k = make_kparams(p, 0, 1, s->tune.chunk_spp);
    const uint32_t slots = slots_per_rank(k);
    const uint64_t npx = (uint64_t)p->width * p->height;
    const bool want_hits = opt_hit_ids && (p->flags & RT_FLAG_HIT_IDS);
    const bool want_stats = opt_stats && (p->flags & RT_FLAG_STATS);
    PathWork W;
    if ((rc = prepare_path(s, k, want_stats, want_hits, W))) return rc;
    DevBuf<double> tiles, img;
    DevBuf<int32_t> hits;
    HIP_TRY(tiles.alloc((size_t)slots * 256 * 3));
    HIP_TRY(img.alloc(npx * 3));
    const uint64_t nhits = npx * p->spp * p->ray_depth;
    if (want_hits) HIP_TRY(hits.alloc(nhits));
    if (want_stats) HIP_TRY(hipMemset(s->d_stats, 0, kStatsWords * sizeof(unsigned long long)));
    EventPair ev;
    HIP_TRY(hipEventCreate(&ev.a));
    HIP_TRY(hipEventCreate(&ev.b));
    HIP_TRY(ws_begin(s, 0));
    HIP_TRY(hipEventRecord(ev.a, 0));
    hipError_t le = launch_path(s->dev, k, W, tiles.p, want_hits ? hits.p : nullptr,
                                want_stats ? s->d_stats : nullptr, 0);
    HIP_TRY(hipEventRecord(ev.b, 0));
    if (le != hipSuccess) return set_error(RT_ERR_DEVICE, std::string("path kernel launch: ") + hipGetErrorString(le));
    HIP_TRY(ws_end(s, 0));
    HIP_TRY(launch_unpack(tiles.p, img.p, p->width, p->height, k.tiles_x, 1, slots, 0));
    HIP_TRY(hipDeviceSynchronize());
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, ev.a, ev.b);
    HIP_TRY(hipMemcpy(out_mean_rgb, img.p, npx * 3 * sizeof(double), hipMemcpyDeviceToHost));
    if (want_hits) HIP_TRY(hipMemcpy(opt_hit_ids, hits.p, nhits * sizeof(int32_t), hipMemcpyDeviceToHost));
    if (opt_stats) {
        std::memset(opt_stats, 0, sizeof(*opt_stats));
        if (want_stats && (rc = copy_stats(s, opt_stats))) return rc;
        opt_stats->kernel_ms = ms;
        opt_stats->total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    return RT_OK;
}

int rt_intersect_rays(rt_scene* s, const double* rays, uint32_t n, rt_hit* out) {
    if (!s || (!rays && n) || (!out && n)) return set_error(RT_ERR_INVALID, "bad arguments");
    if (n == 0) return RT_OK;
    DEVICE_GUARD(s);
    int rc = ensure_spill(s, ((uint64_t)n + 255) / 256 * 256);
    if (rc) return rc;
    DevBuf<double> r;
    DevBuf<rt_hit> h;
    HIP_TRY(r.alloc((size_t)n * 6));
    HIP_TRY(h.alloc(n));
    HIP_TRY(hipMemcpy(r.p, rays, (size_t)n * 6 * sizeof(double), hipMemcpyHostToDevice));
    HIP_TRY(ws_begin(s, 0));
    HIP_TRY(launch_intersect(s->dev, r.p, n, h.p, s->spill_n, s->spill_t, 0));
    HIP_TRY(ws_end(s, 0));
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(out, h.p, (size_t)n * sizeof(rt_hit), hipMemcpyDeviceToHost));
    return RT_OK;
}

int rt_intersect_rays_async(rt_scene* s, const double* d_rays, uint32_t n, rt_hit* d_out, int method,
                            void* hip_stream) {
    if (!s || (!d_rays && n) || (!d_out && n)) return set_error(RT_ERR_INVALID, "bad arguments");
#ifdef RT_WF_PROBE
    if (method == 2) {  // experiment: the traversal-only kernel (render.hip trace_tri_kernel)
        if (n == 0) return RT_OK;
        DEVICE_GUARD(s);
        if (!s->dev.tris.cnodes || path_kinds(s) != 2) return set_error(RT_ERR_INVALID, "probe: compact triangles only");
        uint32_t grid = 0;
        HIP_TRY(trace_tri_grid(n, &grid));
        int rc = ensure_spill(s, (uint64_t)grid * 64);
        if (rc) return rc;
        if (!s->queue) HIP_TRY(hipMalloc(&s->queue, kQueueWords * sizeof(uint32_t)));
        const hipStream_t st = (hipStream_t)hip_stream;
        HIP_TRY(ws_begin(s, st));
        HIP_TRY(launch_trace_tri(s->dev, d_rays, n, d_out, s->queue, s->spill_n, s->spill_t, grid, st));
        HIP_TRY(ws_end(s, st));
        return RT_OK;
    }
#endif
    if (method != RT_TRACE_PER_RAY && method != RT_TRACE_PERSISTENT) return set_error(RT_ERR_INVALID, "bad method");
    if (n == 0) return RT_OK;
    DEVICE_GUARD(s);
    const hipStream_t st = (hipStream_t)hip_stream;
    if (method == RT_TRACE_PER_RAY) {
        int rc = ensure_spill(s, ((uint64_t)n + 255) / 256 * 256);
        if (rc) return rc;
        HIP_TRY(ws_begin(s, st));
        HIP_TRY(launch_intersect(s->dev, d_rays, n, d_out, s->spill_n, s->spill_t, st));
        HIP_TRY(ws_end(s, st));
        return RT_OK;
    }
    uint32_t grid = 0;
    HIP_TRY(trace_grid(n, &grid));
    // the ray counter may run past n by one refill per wave: keep it in 32 bits
    if ((uint64_t)n + (uint64_t)grid * 64 >= (1ull << 32)) return set_error(RT_ERR_INVALID, "too many rays");
    int rc = ensure_spill(s, (uint64_t)grid * 64);
    if (rc) return rc;
    if (!s->queue) HIP_TRY(hipMalloc(&s->queue, kQueueWords * sizeof(uint32_t)));
    HIP_TRY(ws_begin(s, st));
    // the persistent form reads the compact triangle layout's pair lines, or its 64-B nodes, or the
    // f64 layout, as rt_tuning.compact says (auto: the pair lines when the scene has them)
    HIP_TRY(launch_trace(s->dev, d_rays, n, d_out, s->queue, s->spill_n, s->spill_t, grid,
                         s->tune.compact == 0 ? 0 : (s->tune.compact == 1 ? 1 : 2), st));
    HIP_TRY(ws_end(s, st));
    return RT_OK;
}

static int light_query(rt_scene* s, const double* rays, uint32_t n, int mode, double* out, uint32_t* cnt) {
    if (!s || (!rays && n) || (!out && n)) return set_error(RT_ERR_INVALID, "bad arguments");
    if (n == 0) return RT_OK;
    DEVICE_GUARD(s);
    int rc = ensure_spill(s, ((uint64_t)n + 255) / 256 * 256);
    if (rc) return rc;
    DevBuf<double> r, o;
    DevBuf<uint32_t> c;
    HIP_TRY(r.alloc((size_t)n * 6));
    HIP_TRY(o.alloc(n));
    if (cnt) HIP_TRY(c.alloc(n));
    HIP_TRY(hipMemcpy(r.p, rays, (size_t)n * 6 * sizeof(double), hipMemcpyHostToDevice));
    HIP_TRY(ws_begin(s, 0));
    HIP_TRY(launch_light(s->dev, r.p, n, mode, o.p, cnt ? c.p : nullptr, s->spill_n, s->spill_t, 0));
    HIP_TRY(ws_end(s, 0));
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(out, o.p, (size_t)n * sizeof(double), hipMemcpyDeviceToHost));
    if (cnt) HIP_TRY(hipMemcpy(cnt, c.p, (size_t)n * sizeof(uint32_t), hipMemcpyDeviceToHost));
    return RT_OK;
}

int rt_light_pdf_rays(rt_scene* s, const double* pos_dir, uint32_t n, double* out_pdf) {
    return light_query(s, pos_dir, n, 1, out_pdf, nullptr);
}

// Extra query (not in the reference's call graph as a batch): the raw
// intersect_lights accumulation of Light::pdf without the epsilon offset and
// the 1/len normalisation, plus the number of callbacks.  Used by the
// triangle::aaa known-answer test (primitives/triangle.rs:98-128).
int rt_intersect_lights_rays(rt_scene* s, const double* rays, uint32_t n, double* out_impact, uint32_t* out_count) {
    return light_query(s, rays, n, 0, out_impact, out_count);
}

int rt_bvh_build(const double* boxes, uint64_t n, uint64_t* n_nodes, int64_t* out_links, double* out_bounds,
                 uint64_t* out_order, uint32_t* out_depth) {
    if ((!boxes && n) || !n_nodes) return set_error(RT_ERR_INVALID, "boxes/n_nodes is NULL");
    std::vector<Box3> b(n);
    for (uint64_t i = 0; i < n; ++i) b[i] = Box3{load3(boxes + 6 * i), load3(boxes + 6 * i + 3)};
    HostBvh h = build_bvh(b);
    if (out_links && *n_nodes < h.nodes.size()) return set_error(RT_ERR_INVALID, "output too small");
    *n_nodes = h.nodes.size();
    if (out_depth) *out_depth = h.depth;
    if (!out_links) return RT_OK;
    for (size_t i = 0; i < h.nodes.size(); ++i) {
        const HostNode& nd = h.nodes[i];
        out_links[4 * i] = nd.left; out_links[4 * i + 1] = nd.right;
        out_links[4 * i + 2] = (int64_t)nd.start; out_links[4 * i + 3] = (int64_t)nd.end;
        if (out_bounds) { store3(out_bounds + 6 * i, nd.box.min); store3(out_bounds + 6 * i + 3, nd.box.max); }
    }
    if (out_order) for (uint64_t i = 0; i < n; ++i) out_order[i] = h.order[i];
    return RT_OK;
}

// Diagnostic: device f64 sqrt (op 0), division (op 1), the split division
// dev_quot(a, b, dev_rcp(b)) (op 2), dev_sqrt(a) (op 3), dev_inv_len(a)
// (op 4) and dev_quotf(a, b, dev_rcp(b)) (op 5) for bit-exactness checks.
int rt_probe_fp64(int op, const double* a, const double* b, uint32_t n, double* out) {
    const bool two = op == 1 || op == 2 || op == 5;
    if (!a || !out || (two && !b) || op < 0 || op > 5) return set_error(RT_ERR_INVALID, "bad arguments");
    if (n == 0) return RT_OK;
    DevBuf<double> da, db, dout;
    HIP_TRY(da.alloc(n));
    HIP_TRY(db.alloc(n));
    HIP_TRY(dout.alloc(n));
    HIP_TRY(hipMemcpy(da.p, a, n * sizeof(double), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(db.p, two ? b : a, n * sizeof(double), hipMemcpyHostToDevice));
    HIP_TRY(launch_fp64_probe(da.p, db.p, dout.p, n, op, 0));
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(out, dout.p, n * sizeof(double), hipMemcpyDeviceToHost));
    return RT_OK;
}

}  // extern "C"
