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
};

hipError_t launch_path(const DevScene& S, const KParams& P, uint32_t n_slots, double* out, int32_t* hit_ids,
                       unsigned long long* stats, uint32_t* spill_n, double* spill_t, hipStream_t st);
hipError_t launch_intersect(const DevScene& S, const double* rays, uint32_t n, rt_hit* out, uint32_t* spill_n,
                            double* spill_t, hipStream_t st);
hipError_t launch_light(const DevScene& S, const double* rays, uint32_t n, int mode, double* out, uint32_t* cnt,
                        uint32_t* spill_n, double* spill_t, hipStream_t st);
hipError_t launch_unpack(const double* g, double* img, uint32_t W, uint32_t H, uint32_t tiles_x, uint32_t world,
                         uint32_t per_rank, hipStream_t st);
hipError_t launch_fp64_probe(const double* a, const double* b, double* out, uint32_t n, int op, hipStream_t st);

}  // namespace rt
