// render.h — host-side view of the device kernels (render.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/rt_api.h"
#include "rt_layout.h"

namespace rt {

// Per-frame constants of the path kernel: Camera (camera.rs:6-46, computed on
// the host exactly as Camera::new), Scene::{ray_depth, bg_color, samples},
// and the tile partition of this rank.
struct KParams {
    uint32_t width, height, spp, ray_depth;
    double fw, fh, tan_x, tan_y;
    double inv_fw, inv_fh;     // RN(1/fw), RN(1/fh) for the exact reciprocal division
    double cam_pos[3], cam_right[3], cam_up[3], cam_fwd[3];
    double bg[3];
    double scale01, scale11;   // UniformFloat::new_inclusive scales for [0,1], [-1,1]
    uint64_t seed;
    uint32_t rank, world;
    uint32_t tiles_x, tiles_y;
    uint64_t n_tiles;
    // sample chunking (DESIGN.md §4 "work units"): a work unit is (tile slot,
    // chunk of chunk_spp consecutive samples); chunks == 1 writes means directly
    uint32_t chunks, chunk_spp;
    uint32_t n_slots;
    uint32_t suspend;     // live lanes below which the resumable kernel suspends traversal (api.cpp path_suspend)
    uint32_t leaf_batch;  // lanes waiting at leaves before the resumable kernel tests them (api.cpp path_suspend)
    // the queue's last n_tail wave-tiles are handed out in tail_split parts whose rows
    // go to `rows` ([n_tail][chunk_spp][64][3]); render.hip queue_entry / tail_combine_kernel
    uint32_t n_tail, tail_split;
    double* rows;
};

// device work counters: paths, segments, aabb, tri, shape, shaded, light queries,
// light hits, lane steps, wave steps (64 x longest lane) — rt_stats order
constexpr int kNStats = 10;
constexpr int kStatsWords = 64;   // device counter words (rt_read_raw_stats)
constexpr int kStatLqSkip = 10;  // raw word: last-bounce light queries the timed kernel skips
// raw words 11..13: inner-node visits of closest-hit traversals whose child boxes
// were hit by none / one / both of the two slab tests (stats instances only)
constexpr int kStatKids0 = 11;
// raw word 14 (stats path kernel only): waves that made no progress for kStallTrips
// consecutive loop trips and exited (render.hip path_kernel's progress guard; the
// host turns a nonzero word into RT_ERR_DEVICE, api.cpp copy_stats).  A trip makes
// progress when it pulls a wave-tile, hands out a path, steps a traversal, shades a
// segment or commits a row; a wave with nothing of that left has exited, so an idle
// trip can only be a livelock (the round-5 RT_RING_ROWS=16 build's).
constexpr int kStatStall = 14;
constexpr uint32_t kStallTrips = 256;
constexpr int kTimeline = 52;     // stats path kernel: wave timeline words 52..59 (render.hip, tools/timeline.py)
constexpr int kPhaseWord0 = 16;   // RT_PHASES builds: region cycles + loop counts at words 16..51 (16 + kPhN - 1)

// Chunk count for a frame: a function of (W, H, spp) only, so the image does not
// depend on the number of GPUs.  Doubles while the frame has < kChunkLanes
// work units or the chunks would still hold >= kMinChunkSpp samples (many short
// wave-tiles balance the ranks of a multi-GPU frame; the path kernel streams
// rows across wave-tiles, so short ones cost no drain), capped at spp and
// kMaxChunks, and by kPartBytes: the chunk partial sums ([tiles][chunks][256][3]
// f64, written and reduced once per frame) stay within 4 GiB over all ranks
// (C2/C3: 32 chunks, 1.6 GB; C4 3840x2160: 16 chunks, 3.2 GB — 64 would be
// 12.7 GB); then trimmed so no chunk is empty.  (Round 5 tried 8M runs, which gave C5
// 8-spp chunks: 4.5% faster with the 8-row commit window, but 1.5% slower than these
// 4-spp chunks once the window is 64 rows, so 32M stays: profiles/r05/variants_chunk*_C5.log.)
constexpr uint64_t kChunkLanes = 32000000;
constexpr uint32_t kMinChunkSpp = 8;
constexpr uint32_t kMaxChunks = 64;
#ifndef RT_PART_BYTES
#define RT_PART_BYTES (4ull << 30)
#endif
constexpr uint64_t kPartBytes = RT_PART_BYTES;
inline void sample_chunks(uint32_t W, uint32_t H, uint32_t spp, uint32_t& chunks, uint32_t& chunk_spp) {
    const uint64_t px = (uint64_t)W * H;
    const uint64_t chunk_bytes = (uint64_t)((W + 15) / 16) * ((H + 15) / 16) * 256 * 3 * sizeof(double);
    uint32_t k = 1;
    while (k * 2 <= spp && k < kMaxChunks && chunk_bytes * (k * 2) <= kPartBytes &&
           (px * k < kChunkLanes || spp / (k * 2) >= kMinChunkSpp))
        k *= 2;
    chunk_spp = (spp + k - 1) / k;
    chunks = (spp + chunk_spp - 1) / chunk_spp;
}

// PathWork::kinds value of a triangle-only scene whose triangle BVH runs in the
// compact layout (rt_layout.h DevNodeC): kTris | 4, only with the 4-wave
// resumable instance (api.cpp path_kinds).
constexpr int kKindsCompact = 6;
// ... with its inner nodes read from the pair layout (rt_layout.h kPairFloats):
// kTris | 4 | 8, the same instance family (api.cpp path_pairs).
constexpr int kKindsPair = 14;

// Device workspace of one path-kernel launch (owned by the scene).
struct PathWork {
    const DevScene* d_scene;  // the scene record in device memory (uploaded once)
    KParams* d_params;        // frame constants slot, staged by launch_path
    uint32_t waves;       // register budget of the kernel instance: 3 or 4 waves/SIMD
    bool resume;          // resumable triangle traversal (path_kernel RES)
    int kinds;            // the scene's primitive kinds, kShapes 1 | kTris 2 (path_kernel KM); kKindsCompact
    uint32_t grid;        // persistent waves (path_grid)
    uint32_t* queue;      // wave-tile counter, zeroed by launch_path
    double* ring;         // [grid][kRing=64][64][3] finished-path radiance
    double* part;         // [n_slots*chunks][256][3] chunk partial sums (chunks > 1)
    uint32_t* spill_n;    // traversal-stack spill, stride grid*64
    double* spill_t;
};
// Rows of a wave's commit window (round 5: 64, was 8).  A path still running in
// the oldest open row holds the window; the resumable kernel's lanes then idle once
// the window's paths are all taken.  32 rows: C5 -4.9% (207.3 -> 197.0 ms at 64 spp),
// C3 -0.7%, C2 +0.1%.  64 rows lost at first (C5 212 ms, C3 +8%: with 64 open
// wave-tile entries the 4-wave kernel's LDS no longer fit 16 waves a CU); with 16
// entries (render.hip kUQ) it fits and gains again: C5 -1.6%, C3 -0.3%
// (profiles/r05/variants_ring*_C*.log, variants_u16_C*.log).
#ifndef RT_RING_ROWS
#define RT_RING_ROWS 64
#endif
constexpr uint32_t kRingRows = RT_RING_ROWS;   // render.hip kRing (power of two, <= 64)
// Suspend threshold of the resumable triangle traversal (path_kernel RES): fewer
// live lanes than this and the wave lets its waiting lanes shade and start new
// rays.  A cache-resident BVH (C3, ~40 MB) ran best at 24 in round 2 (16: +0.3%,
// 32: +3.7%); with the path's T and L in LDS a suspension costs less (no spill
// traffic per trip) and 32 wins (C3 203.8 -> 201.1 ms at 64 spp, 16: +4.9%;
// profiles/r03/variants/variants_suspend_tl_C3.log, variants_suspend32_C3.log: 28 +0.3%, 36 +0.4%, 40 +2.4%, 48 +7.9%);
// one that streams from HBM (C5, ~1.4 GB, past the 256-MiB Infinity Cache) at 40
// (16: +16.6%, 24: +5.3%, 48: +1.6%; profiles/r02/variants/variants_suspend*.log):
// there every lane sent back to issue its next ray adds memory-level parallelism.
// Round 5, with the 32-row commit window: streamed 40 -> 48 and its leaf batch
// 24 -> 28, C5 196.7 -> 192.4 ms at 64 spp (56: 196.6, 64: 273; the cached pair
// 32/32 still best on C3; profiles/r05/variants_knobs*_C*.log).
constexpr uint32_t kSuspendCached = 32, kSuspendStreamed = 48;
// Leaf batch of the same kernel (lanes waiting at leaves before the wave tests
// them): C3 16 -> 32 lanes 236.3 -> 227.1 ms, C5 16 -> 24 lanes 260.3 -> 249.5 ms at
// 64 spp (profiles/r02/variants/variants_leaflanes*.log).
constexpr uint32_t kLeafCached = 32, kLeafStreamed = 28;
// The compact layout's kernel tests small leaves cooperatively (render.hip
// leaf_coop: a leaf step costs one round per 64 records, not max(count) trips), so
// it waits for fewer lanes at leaves and suspends later on a cached BVH. Round 6,
// alternating runs (profiles/r06/variants_coop_grid*_C*.log): C3 at 64 spp
// 24 / 16 173.4-174.1 ms (32 / 32 serial 177.1-177.5; 20 / 16 173.6, 24 / 12
// 174.4, 16 / 12 174.8, 32 / 16 176.1, 40 / 16 179.4), C5 at 16 spp 48 / 12
// 50.9-51.0 ms (48 / 28 serial 54.7-55.6; 44 / 12 50.9, 40 / 12 50.6-51.0,
// 48 / 10 51.6, 48 / 14 51.3, 48 / 20 53.2, 56 / 12 52.8, 32 / 12 52.1).
constexpr uint32_t kSuspendCoopCached = 24, kSuspendCoopStreamed = 48;
constexpr uint32_t kLeafCoopCached = 16, kLeafCoopStreamed = 12;
constexpr uint64_t kCacheBytes = 256ull << 20;  // MI355X Infinity Cache (MALL)
constexpr uint64_t kDeepSceneNodes = 4096;  // BVH nodes above which the 4-wave kernel runs
constexpr uint32_t kTailSplit = 8;                      // parts per tail wave-tile (api.cpp prepare_path)
#ifndef RT_TAIL_PER_WAVE
#define RT_TAIL_PER_WAVE 3
#endif
constexpr uint64_t kTailPerWave = RT_TAIL_PER_WAVE;     // tail wave-tiles per resident wave
constexpr uint64_t kTailRowBytes = 256ull << 20;        // row buffer cap of the split tail
constexpr uint32_t kShapeWaves = 5;  // waves/SIMD of the shape-only fused kernel (api.cpp path_waves)
constexpr uint64_t kShapeWavesNodes = 64;  // BVH nodes of a shape-only scene up to which it runs at kShapeWaves
constexpr size_t kQueueWords = 16;  // wave-tile counter (word 0), padded to a 64-B line

hipError_t path_grid(bool stats, bool hits, uint32_t waves, bool resume, int kinds, uint32_t n_units,
                     uint32_t* grid);
hipError_t launch_path(const DevScene& S, const KParams& P, const PathWork& W, double* out, int32_t* hit_ids,
                       unsigned long long* stats, hipStream_t st);
hipError_t launch_reduce_chunks(const double* part, double* out, const KParams& P, hipStream_t st);
// compact: 0 the f64 triangle layout, 1 the compact one, 2 its pair lines (when the scene has them)
hipError_t launch_trace(const DevScene& S, const double* rays, uint32_t n, rt_hit* out, uint32_t* queue,
                        uint32_t* spill_n, double* spill_t, uint32_t grid, int compact, hipStream_t st);
hipError_t trace_grid(uint32_t n, uint32_t* grid);
#ifdef RT_WF_PROBE
hipError_t launch_trace_tri(const DevScene& S, const double* rays, uint32_t n, rt_hit* out, uint32_t* queue,
                            uint32_t* spill_n, double* spill_t, uint32_t grid, hipStream_t st);
hipError_t trace_tri_grid(uint32_t n, uint32_t* grid);
#endif
hipError_t launch_intersect(const DevScene& S, const double* rays, uint32_t n, rt_hit* out, uint32_t* spill_n,
                            double* spill_t, hipStream_t st);
hipError_t launch_light(const DevScene& S, const double* rays, uint32_t n, int mode, double* out, uint32_t* cnt,
                        uint32_t* spill_n, double* spill_t, hipStream_t st);
// post_dev.hip: tonemap + gamma + PPM bytes (standalone, and fused into the unpack)
hipError_t launch_tonemap_bytes(const double* rgb, uint64_t n_values, uint8_t* out, hipStream_t st);
hipError_t launch_unpack_bytes(const double* g, uint8_t* bytes, uint32_t W, uint32_t H, uint32_t tiles_x,
                               uint32_t world, uint32_t per_rank, hipStream_t st);
hipError_t launch_unpack(const double* g, double* img, uint32_t W, uint32_t H, uint32_t tiles_x, uint32_t world,
                         uint32_t per_rank, hipStream_t st);
// ellipsoid records: aux = dev_rcp(radii), the device's own reciprocals (rt_device.h)
hipError_t launch_ell_rcp(DevShape* shapes, uint32_t n, hipStream_t st);
// checksum_kernel: order-free content hash of a device array (rt_scene_checksum)
hipError_t launch_checksum(const void* p, uint64_t bytes, unsigned long long* d_out, hipStream_t st);
hipError_t launch_fp64_probe(const double* a, const double* b, double* out, uint32_t n, int op, hipStream_t st);

}  // namespace rt
