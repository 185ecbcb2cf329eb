// multi.cpp — one process, several GPUs: rt_multi_* of include/rt_api.h.
//
// generate_image (main.rs:85-114) over the GPUs of one node from a single host
// thread, so the Rust `main` (main.rs:73) keeps one call per frame:
//   * the host builds the six BVHs once (scene.rs:180-223, bvh.rs:12-17) and
//     uploads them to devices[0] only; every other listed device gets its
//     replica from devices[0] over xGMI — one ncclBroadcast per scene array
//     (peer copies under RT_MULTI_PEER) — instead of its own host copy (C5:
//     ~1.7 GB per device over PCIe otherwise);
//   * the frame's 16x16 tiles are dealt round-robin (tile t -> device index
//     t % n), each device renders its share on its own stream
//     (rt_render_tiles_async, the same partition torchrun ranks use);
//   * ONE gather of the packed tiles to devices[0]: an RCCL ncclGather over
//     xGMI (the communicator spans the listed devices, ncclCommInitAll), or
//     peer copies (RT_MULTI_PEER);
//   * devices[0] unpacks (and, for PPM bytes, tonemaps) and copies the image
//     to the host once.
// RCCL is loaded with dlopen at rt_multi_create: the library itself has no
// link-time dependency on it, and a missing RCCL is an error code, not a
// load failure.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <memory>
#include <set>
#include <string>
#include <vector>

#include "../../include/rt_api.h"
#include "api_internal.h"
#include "scene_build.h"

using rt::set_error;

namespace {

#define MHIP(expr)                                                                            \
    do {                                                                                      \
        hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess)                                                                 \
            return set_error(e_ == hipErrorOutOfMemory ? RT_ERR_NOMEM : RT_ERR_DEVICE,        \
                             std::string(#expr) + ": " + hipGetErrorString(e_));              \
    } while (0)

// The RCCL entry points the gather needs, resolved from librccl.so.1.
struct Rccl {
    void* handle = nullptr;
    decltype(&ncclCommInitAll) comm_init_all = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
    decltype(&ncclCommAbort) comm_abort = nullptr;
    decltype(&ncclGather) gather = nullptr;
    decltype(&ncclBroadcast) broadcast = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;

    bool bind(void* h) {
        comm_init_all = (decltype(comm_init_all))dlsym(h, "ncclCommInitAll");
        comm_destroy = (decltype(comm_destroy))dlsym(h, "ncclCommDestroy");
        comm_abort = (decltype(comm_abort))dlsym(h, "ncclCommAbort");
        gather = (decltype(gather))dlsym(h, "ncclGather");
        broadcast = (decltype(broadcast))dlsym(h, "ncclBroadcast");
        group_start = (decltype(group_start))dlsym(h, "ncclGroupStart");
        group_end = (decltype(group_end))dlsym(h, "ncclGroupEnd");
        error_string = (decltype(error_string))dlsym(h, "ncclGetErrorString");
        if (!comm_init_all || !comm_destroy || !comm_abort || !gather || !broadcast || !group_start || !group_end ||
            !error_string)
            return false;
        handle = h;
        return true;
    }
    int load() {
        if (handle) return RT_OK;
        // One RCCL per process, like one HIP runtime: an RCCL already loaded (a
        // host that links it, or torch's copy) is used as is; otherwise ROCm's.
        for (const char* name : {"librccl.so", "librccl.so.1"})
            if (void* h = dlopen(name, RTLD_NOW | RTLD_NOLOAD))
                if (bind(h)) return RT_OK;
        for (const char* name : {"librccl.so.1", "/opt/rocm/lib/librccl.so.1"})
            if (void* h = dlopen(name, RTLD_NOW | RTLD_LOCAL))
                if (bind(h)) return RT_OK;
        return set_error(RT_ERR_UNSUPPORTED, "no RCCL with ncclGather/ncclBroadcast/ncclCommInitAll found (librccl.so.1): "
                                             "use RT_MULTI_PEER");
    }
};

// Restores the caller's current device on every return path.
struct KeepDevice {
    int prev = -1;
    KeepDevice() { (void)hipGetDevice(&prev); }
    ~KeepDevice() { if (prev >= 0) (void)hipSetDevice(prev); }
};

template <class T>
int grow(T*& p, size_t& cap, size_t need) {  // device buffer on the current device, grow-only
    if (need <= cap) return RT_OK;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    MHIP(hipMalloc((void**)&p, need * sizeof(T)));
    cap = need;
    return RT_OK;
}

}  // namespace

struct rt_multi {
    std::vector<int> devs;
    std::vector<rt_scene*> scenes;
    std::vector<hipStream_t> streams;
    std::vector<hipEvent_t> ev0, ev1;         // render start / end per device
    std::vector<double*> tiles;               // packed tiles of device i (on device i)
    std::vector<size_t> tile_cap;
    double* gathered = nullptr;               // [n][slots][256][3] on devs[0]
    size_t gathered_cap = 0;
    double* image = nullptr;                  // [H][W][3] f64 on devs[0]
    size_t image_cap = 0;
    uint8_t* bytes = nullptr;                 // [H][W][3] u8 on devs[0]
    size_t bytes_cap = 0;
    bool peer = false;
    Rccl rccl;
    std::vector<ncclComm_t> comms;
    bool comms_aborted = false;               // a failed gather aborted them: the handle cannot gather again
};

namespace {

void free_multi(rt_multi* m) {
    if (!m) return;
    KeepDevice keep;
    for (size_t i = 0; i < m->comms.size(); ++i)
        if (m->comms[i]) (void)m->rccl.comm_destroy(m->comms[i]);
    for (size_t i = 0; i < m->devs.size(); ++i) {
        (void)hipSetDevice(m->devs[i]);
        if (i < m->streams.size() && m->streams[i]) (void)hipStreamSynchronize(m->streams[i]);
        if (i < m->tiles.size() && m->tiles[i]) (void)hipFree(m->tiles[i]);
        if (i < m->ev0.size() && m->ev0[i]) (void)hipEventDestroy(m->ev0[i]);
        if (i < m->ev1.size() && m->ev1[i]) (void)hipEventDestroy(m->ev1[i]);
        if (i < m->streams.size() && m->streams[i]) (void)hipStreamDestroy(m->streams[i]);
        if (i < m->scenes.size() && m->scenes[i]) rt_scene_destroy(m->scenes[i]);
    }
    if (!m->devs.empty()) {
        (void)hipSetDevice(m->devs[0]);
        if (m->gathered) (void)hipFree(m->gathered);
        if (m->image) (void)hipFree(m->image);
        if (m->bytes) (void)hipFree(m->bytes);
    }
    // the RCCL library stays loaded (its proxy threads may outlive the communicators)
    delete m;
}

struct MultiDeleter {
    void operator()(rt_multi* m) const { free_multi(m); }
};

// Error return after work was queued: wait for every device's stream (so no
// launch of this frame is left running against buffers the caller may free),
// errors ignored — the call already failed.  Disarmed on success.
struct Drain {
    rt_multi* m;
    bool armed = false;
    ~Drain() {
        if (!armed) return;
        for (size_t i = 0; i < m->devs.size(); ++i) {
            (void)hipSetDevice(m->devs[i]);
            (void)hipStreamSynchronize(m->streams[i]);
        }
    }
};

// The replicas' scene arrays from devices[0]'s (scene_upload's allocation order is
// the build's, the same on every device): one ncclBroadcast per array, root 0, all
// ranks in one group — over xGMI, devices[0]'s copy fans out without touching the
// host — or, under RT_MULTI_PEER, one peer copy per array and replica.  The fill
// time is added to each replica's rt_scene_info.upload_ms.
int replicate_scene(rt_multi* m) {
    const uint32_t n = (uint32_t)m->devs.size();
    if (n < 2) return RT_OK;
    const std::vector<size_t>* bytes0 = nullptr;
    const std::vector<void*>& src = rt::scene_allocs(m->scenes[0], &bytes0);
    std::vector<const std::vector<void*>*> dst(n);
    for (uint32_t i = 0; i < n; ++i) {
        const std::vector<size_t>* b = nullptr;
        dst[i] = &rt::scene_allocs(m->scenes[i], &b);
        if (*b != *bytes0) return set_error(RT_ERR_DEVICE, "replica scene layout differs from devices[0]'s");
    }
    const auto t0 = std::chrono::steady_clock::now();
    if (m->peer) {
        for (uint32_t i = 1; i < n; ++i) {
            MHIP(hipSetDevice(m->devs[i]));
            for (size_t k = 0; k < src.size(); ++k)
                MHIP(hipMemcpyPeerAsync((*dst[i])[k], m->devs[i], src[k], m->devs[0], (*bytes0)[k], m->streams[i]));
        }
    } else {
        for (size_t k = 0; k < src.size(); ++k) {
            ncclResult_t r = m->rccl.group_start();
            for (uint32_t i = 0; i < n && r == ncclSuccess; ++i)
                r = m->rccl.broadcast(src[k], i == 0 ? src[k] : (*dst[i])[k], (*bytes0)[k], ncclUint8, 0, m->comms[i],
                                      m->streams[i]);
            const ncclResult_t r2 = m->rccl.group_end();
            if (r != ncclSuccess || r2 != ncclSuccess) {
                for (ncclComm_t& c : m->comms)
                    if (c) { (void)m->rccl.comm_abort(c); c = nullptr; }
                m->comms_aborted = true;
                for (uint32_t i = 0; i < n; ++i) {
                    (void)hipSetDevice(m->devs[i]);
                    (void)hipStreamSynchronize(m->streams[i]);
                }
                return set_error(RT_ERR_DEVICE, std::string("ncclBroadcast: ") + m->rccl.error_string(r ? r : r2));
            }
        }
    }
    for (uint32_t i = 0; i < n; ++i) {
        MHIP(hipSetDevice(m->devs[i]));
        MHIP(hipStreamSynchronize(m->streams[i]));
    }
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    for (uint32_t i = 1; i < n; ++i) rt::scene_add_upload_ms(m->scenes[i], ms);
    // every replica must hold devices[0]'s bytes (a wrong root, buffer pairing or array
    // order would otherwise render silently wrong frames): content hashes on each device
    uint64_t h0 = 0;
    if (int rc = rt_scene_checksum(m->scenes[0], &h0)) return rc;
    for (uint32_t i = 1; i < n; ++i) {
        uint64_t h = 0;
        if (int rc = rt_scene_checksum(m->scenes[i], &h)) return rc;
        if (h != h0)
            return set_error(RT_ERR_DEVICE, "scene replica on device " + std::to_string(m->devs[i]) +
                                                " differs from devices[0]'s after the " +
                                                (m->peer ? "peer copies" : "ncclBroadcast"));
    }
    return RT_OK;
}

}  // namespace

extern "C" {

int rt_multi_create(const rt_scene_desc* desc, const int* devices, uint32_t n, uint32_t flags, rt_multi** out) {
    if (!desc || !devices || !out || n == 0) return set_error(RT_ERR_INVALID, "desc/devices/out NULL or n == 0");
    *out = nullptr;
    if (flags & ~RT_MULTI_PEER) return set_error(RT_ERR_INVALID, "unknown rt_multi flags");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return set_error(RT_ERR_DEVICE, "no HIP device visible (the hot path has no CPU fallback)");
    for (uint32_t i = 0; i < n; ++i)
        if (devices[i] < 0 || devices[i] >= ndev)
            return set_error(RT_ERR_INVALID, "device " + std::to_string(devices[i]) + " is not visible");
    const bool peer = (flags & RT_MULTI_PEER) != 0;
    if (!peer && std::set<int>(devices, devices + n).size() != n)
        return set_error(RT_ERR_INVALID, "a device is listed twice: RCCL needs one rank per GPU (use RT_MULTI_PEER)");
    rt::HostScene hs;
    if (int rc = rt::scene_build_host(*desc, hs)) return rc;  // the BVHs, once for every device
    std::unique_ptr<rt_multi, MultiDeleter> owner(new rt_multi());
    rt_multi* m = owner.get();
    m->peer = peer;
    KeepDevice keep;
    for (uint32_t i = 0; i < n; ++i) {
        m->devs.push_back(devices[i]);
        m->scenes.push_back(nullptr);
        m->streams.push_back(nullptr);
        m->ev0.push_back(nullptr);
        m->ev1.push_back(nullptr);
        m->tiles.push_back(nullptr);
        m->tile_cap.push_back(0);
        MHIP(hipSetDevice(devices[i]));
        // devices[0] from the host; the others allocate only (filled below from devices[0])
        if (int rc = rt::scene_upload(hs, &m->scenes[i], i > 0)) return rc;
        MHIP(hipStreamCreateWithFlags(&m->streams[i], hipStreamNonBlocking));
        MHIP(hipEventCreate(&m->ev0[i]));
        MHIP(hipEventCreate(&m->ev1[i]));
    }
    if (!peer) {
        if (int rc = m->rccl.load()) return rc;
        m->comms.assign(n, nullptr);
        const ncclResult_t r = m->rccl.comm_init_all(m->comms.data(), (int)n, m->devs.data());
        if (r != ncclSuccess) {
            m->comms.assign(n, nullptr);
            return set_error(RT_ERR_DEVICE, std::string("ncclCommInitAll: ") + m->rccl.error_string(r));
        }
    }
    if (int rc = replicate_scene(m)) return rc;
    *out = owner.release();
    return RT_OK;
}

void rt_multi_destroy(rt_multi* m) { free_multi(m); }

rt_scene* rt_multi_scene(rt_multi* m, uint32_t index) {
    if (!m || index >= m->scenes.size()) return nullptr;
    return m->scenes[index];
}

int rt_multi_render(rt_multi* m, const rt_render_params* p, double* out_mean_rgb, uint8_t* out_ppm_bytes,
                    rt_stats* opt_stats) {
    const auto t0 = std::chrono::steady_clock::now();
    if (!m || !p) return set_error(RT_ERR_INVALID, "multi/params is NULL");
    if (!out_mean_rgb && !out_ppm_bytes) return set_error(RT_ERR_INVALID, "no output requested");
    if (p->flags & RT_FLAG_HIT_IDS) return set_error(RT_ERR_INVALID, "hit-id dumps are rt_render's (one device)");
    if (m->comms_aborted)
        return set_error(RT_ERR_DEVICE, "a previous gather failed and aborted the RCCL communicators: "
                                        "destroy and recreate the rt_multi handle");
    const uint32_t n = (uint32_t)m->devs.size();
    uint32_t slots = 0;
    if (int rc = rt_tiles_per_rank(p, n, &slots)) return rc;  // also validates params
    const size_t cnt = (size_t)slots * 256 * 3;                // f64 per device share
    const size_t npx = (size_t)p->width * p->height;
    const bool want_stats = opt_stats && (p->flags & RT_FLAG_STATS);
    KeepDevice keep;
    rt_stats st{};
    if (want_stats)  // counters of this frame only
        for (uint32_t i = 0; i < n; ++i)
            if (int rc = rt_read_stats(m->scenes[i], &st, 1)) return rc;
    for (uint32_t i = 0; i < n; ++i) {
        MHIP(hipSetDevice(m->devs[i]));
        // the previous frame's gather may still read these tiles (another stream)
        if (cnt > m->tile_cap[i]) MHIP(hipDeviceSynchronize());
        if (int rc = grow(m->tiles[i], m->tile_cap[i], cnt)) return rc;
    }
    MHIP(hipSetDevice(m->devs[0]));
    if (n * cnt > m->gathered_cap || 3 * npx > m->image_cap || 3 * npx > m->bytes_cap)
        MHIP(hipDeviceSynchronize());
    if (int rc = grow(m->gathered, m->gathered_cap, n * cnt)) return rc;
    if (out_mean_rgb)
        if (int rc = grow(m->image, m->image_cap, 3 * npx)) return rc;
    if (out_ppm_bytes)
        if (int rc = grow(m->bytes, m->bytes_cap, 3 * npx)) return rc;

    // every share on its own device and stream (the launches overlap across devices);
    // from here on an error return first drains every stream
    Drain drain{m};
    drain.armed = true;
    for (uint32_t i = 0; i < n; ++i) {
        MHIP(hipSetDevice(m->devs[i]));
        MHIP(hipEventRecord(m->ev0[i], m->streams[i]));
        if (int rc = rt_render_tiles_async(m->scenes[i], p, i, n, m->tiles[i], m->streams[i])) return rc;
        MHIP(hipEventRecord(m->ev1[i], m->streams[i]));
    }
    // ONE gather of the packed tiles to devices[0] (rank-major, ncclGather's layout)
    if (m->peer) {
        MHIP(hipSetDevice(m->devs[0]));
        for (uint32_t i = 0; i < n; ++i) {
            MHIP(hipStreamWaitEvent(m->streams[0], m->ev1[i], 0));
            MHIP(hipMemcpyPeerAsync(m->gathered + (size_t)i * cnt, m->devs[0], m->tiles[i], m->devs[i],
                                    cnt * sizeof(double), m->streams[0]));
        }
    } else {
        ncclResult_t r = m->rccl.group_start();
        for (uint32_t i = 0; i < n && r == ncclSuccess; ++i)
            r = m->rccl.gather(m->tiles[i], i == 0 ? m->gathered : nullptr, cnt, ncclFloat64, 0, m->comms[i],
                               m->streams[i]);
        const ncclResult_t r2 = m->rccl.group_end();
        if (r != ncclSuccess || r2 != ncclSuccess) {
            // ranks already enqueued would wait forever on a collective the others never
            // join: abort the communicators (not destroy) before the streams are drained
            for (ncclComm_t& c : m->comms)
                if (c) { (void)m->rccl.comm_abort(c); c = nullptr; }
            m->comms_aborted = true;
            return set_error(RT_ERR_DEVICE, std::string("ncclGather: ") + m->rccl.error_string(r ? r : r2));
        }
    }
    // root: unpack (main.rs:96-104) and/or the fused tonemap + PPM bytes, then one D2H copy each
    MHIP(hipSetDevice(m->devs[0]));
    const hipStream_t s0 = m->streams[0];
    if (out_mean_rgb) {
        if (int rc = rt_unpack_tiles_async(p, n, m->gathered, m->image, s0)) return rc;
        MHIP(hipMemcpyAsync(out_mean_rgb, m->image, 3 * npx * sizeof(double), hipMemcpyDeviceToHost, s0));
    }
    if (out_ppm_bytes) {
        if (int rc = rt_unpack_tiles_bytes_async(p, n, m->gathered, m->bytes, s0)) return rc;
        MHIP(hipMemcpyAsync(out_ppm_bytes, m->bytes, 3 * npx, hipMemcpyDeviceToHost, s0));
    }
    float kern_ms = 0.f;
    for (uint32_t i = 0; i < n; ++i) {
        MHIP(hipSetDevice(m->devs[i]));
        MHIP(hipStreamSynchronize(m->streams[i]));
        float ms = 0.f;
        MHIP(hipEventElapsedTime(&ms, m->ev0[i], m->ev1[i]));
        kern_ms = std::max(kern_ms, ms);
    }
    if (opt_stats) {
        std::memset(opt_stats, 0, sizeof(*opt_stats));
        if (want_stats)
            for (uint32_t i = 0; i < n; ++i) {
                if (int rc = rt_read_stats(m->scenes[i], &st, 1)) return rc;
                opt_stats->paths += st.paths; opt_stats->segments += st.segments;
                opt_stats->aabb_tests += st.aabb_tests; opt_stats->tri_tests += st.tri_tests;
                opt_stats->shape_tests += st.shape_tests; opt_stats->shaded_hits += st.shaded_hits;
                opt_stats->light_queries += st.light_queries; opt_stats->light_hits += st.light_hits;
                opt_stats->lane_steps += st.lane_steps; opt_stats->wave_steps += st.wave_steps;
            }
        opt_stats->kernel_ms = kern_ms;
        opt_stats->total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    drain.armed = false;
    return RT_OK;
}

}  // extern "C"
