// gltf.cpp — glTF subset input surface (gltf/parser.rs, gltf/scene_builder.rs).
// Placeholder until the reader lands.
#include "../../include/rt_api.h"
#include "api_internal.h"

extern "C" int rt_load_gltf(const char* path, uint32_t, uint32_t, uint32_t, rt_parsed_scene** out) {
    if (out) *out = nullptr;
    (void)path;
    return rt::set_error(RT_ERR_UNSUPPORTED, "glTF reader not built yet");
}
