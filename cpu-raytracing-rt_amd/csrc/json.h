// json.h — minimal JSON DOM for the glTF reader (the reference uses
// serde_json, gltf/parser.rs:189-191).  Strict RFC 8259 grammar; numbers keep
// their text so integer fields can be checked like serde's usize.
#pragma once
#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <vector>

namespace rt {

struct Json {
    enum Kind { Null, Bool, Number, String, Array, Object } kind = Null;
    bool b = false;
    double num = 0.0;
    bool is_int = false;       // number had no fraction/exponent
    bool negative = false;
    uint64_t uint_val = 0;     // valid when is_int && !negative
    std::string str;
    std::vector<Json> arr;
    std::map<std::string, Json> obj;

    const Json* get(const std::string& k) const {
        if (kind != Object) return nullptr;
        auto it = obj.find(k);
        return it == obj.end() ? nullptr : &it->second;
    }
};

// Returns empty string on success, else an error message with the byte offset.
std::string json_parse(const std::string& text, Json& out);

}  // namespace rt
