// api_internal.h — shared internals of the C ABI implementation.
#pragma once
#include <string>
#include <vector>

#include "../../include/rt_api.h"

namespace rt {

int set_error(int code, const std::string& msg);  // records rt_last_error, returns code

// post.cpp: the 255 byte thresholds of the gamma + PPM quantisation on a
// tonemapped value, derived from the host pow and proven exact; false if the
// proof fails (the device epilogue then uses its own pow).
bool byte_thresholds(double thr[255]);

struct HostScene;
// rt_scene_create in two halves (api.cpp): the host build (six BVHs, flattened
// records) and the upload of that build to the current HIP device, so a
// multi-GPU frame (multi.cpp) builds once and uploads one replica per device.
int scene_build_host(const rt_scene_desc& desc, HostScene& hs);
int scene_upload(const HostScene& hs, rt_scene** out, bool replica);
// A scene's device arrays in allocation order (with their sizes): a replica built
// from the same HostScene allocates the same sequence, so array k of the replica
// is filled from array k of the source (multi.cpp: ncclBroadcast or peer copies).
const std::vector<void*>& scene_allocs(const rt_scene* s, const std::vector<size_t>** bytes);
void scene_add_upload_ms(rt_scene* s, double ms);  // the replica's device-to-device fill time

}  // namespace rt

// Host-side parse result of the input surfaces (custom text / glTF).
struct rt_parsed_scene {
    std::vector<rt_material> mats;
    std::vector<rt_shape> shapes;
    std::vector<double> tri_v, tri_n, tri_pos, tri_rot;
    std::vector<uint32_t> tri_mat;
    uint32_t tri_mode = RT_TRI_CUSTOM;
    rt_render_params params{};
};
