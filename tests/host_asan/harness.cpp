// harness.cpp — the host half of the C ABI (custom-scene parser, glTF reader, BVH
// builder, tonemap + PPM) built for the host alone with AddressSanitizer and UBSan
// (tests/test_host_asan.py builds and runs it; no GPU, no HIP calls).
//
//   harness OUT_DIR FILE...   (*.gltf -> rt_load_gltf, anything else -> rt_parse_custom_scene)
//
// Per input: parse, then rt::build_scene (the six BVHs and the flattened records of
// rt_scene_create), then structural checks of every BVH; prints one line per input:
// "ok <nodes> <prims>", "parse-error <msg>" or "build-error <msg>".  A malformed
// input must end in an error line, never in a sanitizer report or a crash.  Last, the
// output surface: rt_tonemap_gamma and rt_save_ppm on values incl. NaN, inf, negatives.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <limits>
#include <sstream>
#include <string>
#include <vector>

#include "../../cpu-raytracing-rt_amd/csrc/api_internal.h"
#include "../../cpu-raytracing-rt_amd/csrc/scene_build.h"

namespace rt {
static thread_local std::string g_err;
int set_error(int code, const std::string& msg) {  // api.cpp's, without the device part
    g_err = msg;
    return code;
}
}  // namespace rt
extern "C" const char* rt_last_error(void) { return rt::g_err.c_str(); }

static bool ends_with(const std::string& s, const char* suf) {
    const size_t n = strlen(suf);
    return s.size() >= n && s.compare(s.size() - n, n, suf) == 0;
}

// every child index, range and permutation entry of a flattened BVH in bounds
static std::string check_bvh(const rt::HostBvhArrays& b) {
    const size_t n = b.nodes.size();
    uint64_t leaf_prims = 0;
    for (size_t i = 0; i < n; ++i) {
        const rt::DevNode& d = b.nodes[i];
        if (d.left < 0 != (d.right < 0)) return "node with one child";
        if (d.left >= 0) {
            if ((size_t)d.left >= n || (size_t)d.right >= n || (size_t)d.left <= i || (size_t)d.right <= i)
                return "child index out of range";
        } else {
            if ((uint64_t)d.start + d.count > b.n_prims) return "leaf range out of range";
            leaf_prims += d.count;
        }
    }
    if (n && leaf_prims != b.n_prims) return "leaves do not cover the primitives once";
    if (!b.gid.empty() && b.gid.size() != b.n_prims) return "gid size";
    if (!b.mat.empty() && b.mat.size() != b.n_prims) return "material size";
    return "";
}

// The pair layout over the compact nodes (scene_build.cpp build_pairs, rt_layout.h
// kPairFloats): every half is its child's record — a leaf child's box twice, an internal
// child's compact node — and the union of its two boxes is the child's box as the
// compact parent stores it (what the device takes as the box).  Counts checked lines.
static size_t g_pair_lines = 0, g_pair_bvhs = 0;
static std::string check_pairs(const rt::HostBvhArrays& b) {
    if (b.pnodes.empty()) return "";
    if (b.pnodes.size() % rt::kPairFloats) return "pair array not whole lines";
    const size_t n_int = b.pnodes.size() / rt::kPairFloats;
    const auto& cn = b.cnodes;
    if (cn.size() < n_int) return "more pair lines than compact slots";
    auto same = [](const float* a, const float* x, int n) { return std::memcmp(a, x, n * sizeof(float)) == 0; };
    for (size_t c = 0; c < n_int; ++c) {
        if (cn[c].count != 0) return "pair line for a leaf slot";
        for (int side = 0; side < 2; ++side) {
            const float* h = &b.pnodes[c * rt::kPairFloats + side * rt::kPairHalf];
            uint32_t w[4];
            std::memcpy(w, h + 12, sizeof(w));
            const uint32_t cw = side ? cn[c].rw : cn[c].lw;
            const float* mn = side ? cn[c].rmin : cn[c].lmin;
            const float* mx = side ? cn[c].rmax : cn[c].lmax;
            if (w[2] != cw) return "pair half: wrong own word";
            if (cw & (rt::kPackedLeaf | rt::kLeafRef)) {
                if (w[3] != rt::kPairLeaf || !same(h, mn, 3) || !same(h + 3, mx, 3) || !same(h + 6, h, 6))
                    return "pair half: leaf box";
            } else {
                if (w[3] != 0 || cw >= n_int) return "pair half: internal child out of range";
                const rt::DevNodeC& k = cn[cw];
                if (!same(h, k.lmin, 3) || !same(h + 3, k.lmax, 3) || !same(h + 6, k.rmin, 3) ||
                    !same(h + 9, k.rmax, 3) || w[0] != k.lw || w[1] != k.rw)
                    return "pair half: not the child's compact node";
                for (int a = 0; a < 3; ++a)
                    if (std::fmin(h[a], h[6 + a]) != mn[a] || std::fmax(h[3 + a], h[9 + a]) != mx[a])
                        return "pair half: union is not the child's box";
            }
        }
    }
    g_pair_lines += n_int;
    ++g_pair_bvhs;
    return "";
}

int main(int argc, char** argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: harness OUT_DIR FILE...\n");
        return 2;
    }
    const std::string out_dir = argv[1];
    for (int i = 2; i < argc; ++i) {
        const std::string path = argv[i];
        rt_parsed_scene* ps = nullptr;
        int rc;
        if (ends_with(path, ".gltf")) {
            rc = rt_load_gltf(path.c_str(), 16, 12, 2, &ps);
        } else {
            std::ifstream f(path, std::ios::binary);
            std::stringstream ss;
            ss << f.rdbuf();
            rc = rt_parse_custom_scene(ss.str().c_str(), &ps);
        }
        if (rc != 0) {
            printf("%s parse-error %s\n", path.c_str(), rt_last_error());
            if (ps) rt_parsed_scene_free(ps);
            continue;
        }
        rt_scene_desc d;
        rt_render_params p;
        if (rt_parsed_scene_get(ps, &d, &p) != 0) {
            printf("%s parse-error (get) %s\n", path.c_str(), rt_last_error());
            rt_parsed_scene_free(ps);
            continue;
        }
        rt::HostScene hs;
        const std::string err = rt::build_scene(d, hs);
        if (!err.empty()) {
            printf("%s build-error %s\n", path.c_str(), err.c_str());
        } else {
            size_t nodes = 0, prims = hs.planes.size();
            std::string bad;
            for (const auto& b : hs.bvh) {
                nodes += b.nodes.size();
                prims += b.n_prims;
                std::string e = check_bvh(b);
                if (e.empty()) e = check_pairs(b);
                if (!e.empty()) bad = e;
            }
            if (!bad.empty()) {
                printf("%s INVALID %s\n", path.c_str(), bad.c_str());
                rt_parsed_scene_free(ps);
                return 1;
            }
            printf("%s ok %zu %zu\n", path.c_str(), nodes, prims);
        }
        rt_parsed_scene_free(ps);
    }
    // output surface on hostile values
    const double inf = std::numeric_limits<double>::infinity(), nan = std::nan("");
    std::vector<double> img = {0.0, -1.0, 1e300, inf, -inf, nan, 0.5, 2.0, 1e-300, 4.9e-324, 100.0, 0.18};
    std::vector<double> out(img.size());
    rt_tonemap_gamma(img.data(), img.size() / 3, out.data());
    if (rt_save_ppm((out_dir + "/t.ppm").c_str(), 2, 2, out.data()) != 0) {
        printf("ppm-error %s\n", rt_last_error());
        return 1;
    }
    if (rt_save_ppm((out_dir + "/no/such/dir/t.ppm").c_str(), 2, 2, out.data()) == 0) {
        printf("ppm to a missing directory did not fail\n");
        return 1;
    }
    double thr[255];
    printf("thresholds %d\n", rt_byte_thresholds(thr));
    printf("pairs %zu %zu\n", g_pair_bvhs, g_pair_lines);
    printf("done\n");
    return 0;
}
