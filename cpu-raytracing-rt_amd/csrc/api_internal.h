// api_internal.h — shared internals of the C ABI implementation.
#pragma once
#include <string>
#include <vector>

#include "../../include/rt_api.h"

namespace rt {

int set_error(int code, const std::string& msg);  // records rt_last_error, returns code

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
