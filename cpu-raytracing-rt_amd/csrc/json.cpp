// json.cpp — recursive-descent JSON parser (see json.h).
#include "json.h"

#include <cerrno>
#include <cstdlib>

namespace rt {
namespace {

struct P {
    const std::string& s;
    size_t i = 0;
    std::string err;
    int depth = 0;

    bool fail(const char* what) {
        if (err.empty()) err = std::string(what) + " at byte " + std::to_string(i);
        return false;
    }
    void ws() {
        while (i < s.size() && (s[i] == ' ' || s[i] == '\t' || s[i] == '\n' || s[i] == '\r')) ++i;
    }
    bool lit(const char* w) {
        size_t n = 0;
        while (w[n]) ++n;
        if (s.compare(i, n, w) != 0) return fail("bad literal");
        i += n;
        return true;
    }
    static void utf8(std::string& o, uint32_t cp) {
        if (cp < 0x80) o.push_back((char)cp);
        else if (cp < 0x800) { o.push_back((char)(0xC0 | (cp >> 6))); o.push_back((char)(0x80 | (cp & 0x3F))); }
        else if (cp < 0x10000) {
            o.push_back((char)(0xE0 | (cp >> 12))); o.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
            o.push_back((char)(0x80 | (cp & 0x3F)));
        } else {
            o.push_back((char)(0xF0 | (cp >> 18))); o.push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
            o.push_back((char)(0x80 | ((cp >> 6) & 0x3F))); o.push_back((char)(0x80 | (cp & 0x3F)));
        }
    }
    bool hex4(uint32_t& v) {
        if (i + 4 > s.size()) return fail("short \\u escape");
        v = 0;
        for (int k = 0; k < 4; ++k) {
            char c = s[i++];
            v <<= 4;
            if (c >= '0' && c <= '9') v |= (uint32_t)(c - '0');
            else if (c >= 'a' && c <= 'f') v |= (uint32_t)(c - 'a' + 10);
            else if (c >= 'A' && c <= 'F') v |= (uint32_t)(c - 'A' + 10);
            else return fail("bad \\u escape");
        }
        return true;
    }
    bool string(std::string& o) {
        if (i >= s.size() || s[i] != '"') return fail("expected string");
        ++i;
        for (;;) {
            if (i >= s.size()) return fail("unterminated string");
            unsigned char c = (unsigned char)s[i++];
            if (c == '"') return true;
            if (c < 0x20) return fail("control character in string");
            if (c != '\\') { o.push_back((char)c); continue; }
            if (i >= s.size()) return fail("bad escape");
            char e = s[i++];
            switch (e) {
            case '"': o.push_back('"'); break;
            case '\\': o.push_back('\\'); break;
            case '/': o.push_back('/'); break;
            case 'b': o.push_back('\b'); break;
            case 'f': o.push_back('\f'); break;
            case 'n': o.push_back('\n'); break;
            case 'r': o.push_back('\r'); break;
            case 't': o.push_back('\t'); break;
            case 'u': {
                uint32_t cp;
                if (!hex4(cp)) return false;
                if (cp >= 0xD800 && cp < 0xDC00) {
                    uint32_t lo;
                    if (i + 2 > s.size() || s[i] != '\\' || s[i + 1] != 'u') return fail("lone surrogate");
                    i += 2;
                    if (!hex4(lo) || lo < 0xDC00 || lo > 0xDFFF) return fail("bad surrogate pair");
                    cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
                }
                utf8(o, cp);
                break;
            }
            default: return fail("bad escape");
            }
        }
    }
    bool number(Json& v) {
        size_t st = i;
        bool neg = false, frac = false;
        if (s[i] == '-') { neg = true; ++i; }
        if (i >= s.size() || !std::isdigit((unsigned char)s[i])) return fail("bad number");
        if (s[i] == '0') ++i;
        else while (i < s.size() && std::isdigit((unsigned char)s[i])) ++i;
        if (i < s.size() && s[i] == '.') {
            frac = true;
            ++i;
            if (i >= s.size() || !std::isdigit((unsigned char)s[i])) return fail("bad fraction");
            while (i < s.size() && std::isdigit((unsigned char)s[i])) ++i;
        }
        if (i < s.size() && (s[i] == 'e' || s[i] == 'E')) {
            frac = true;
            ++i;
            if (i < s.size() && (s[i] == '+' || s[i] == '-')) ++i;
            if (i >= s.size() || !std::isdigit((unsigned char)s[i])) return fail("bad exponent");
            while (i < s.size() && std::isdigit((unsigned char)s[i])) ++i;
        }
        std::string t = s.substr(st, i - st);
        v.kind = Json::Number;
        v.num = std::strtod(t.c_str(), nullptr);  // correctly rounded, like serde_json's float parse
        v.is_int = !frac;
        v.negative = neg;
        if (!frac && !neg) {
            errno = 0;
            unsigned long long u = std::strtoull(t.c_str(), nullptr, 10);
            if (errno == ERANGE) v.is_int = false;
            v.uint_val = u;
        }
        return true;
    }
    bool value(Json& v) {
        if (++depth > 256) return fail("nesting too deep");
        ws();
        if (i >= s.size()) return fail("unexpected end");
        char c = s[i];
        bool ok;
        if (c == '{') {
            v.kind = Json::Object;
            ++i;
            ws();
            if (i < s.size() && s[i] == '}') { ++i; ok = true; }
            else {
                ok = true;
                for (;;) {
                    ws();
                    std::string k;
                    if (!string(k)) { ok = false; break; }
                    ws();
                    if (i >= s.size() || s[i] != ':') { ok = fail("expected ':'"); break; }
                    ++i;
                    Json child;
                    if (!value(child)) { ok = false; break; }
                    v.obj[k] = std::move(child);  // serde: duplicate keys are an error; last wins here
                    ws();
                    if (i < s.size() && s[i] == ',') { ++i; continue; }
                    if (i < s.size() && s[i] == '}') { ++i; break; }
                    ok = fail("expected ',' or '}'");
                    break;
                }
            }
        } else if (c == '[') {
            v.kind = Json::Array;
            ++i;
            ws();
            if (i < s.size() && s[i] == ']') { ++i; ok = true; }
            else {
                ok = true;
                for (;;) {
                    Json child;
                    if (!value(child)) { ok = false; break; }
                    v.arr.push_back(std::move(child));
                    ws();
                    if (i < s.size() && s[i] == ',') { ++i; continue; }
                    if (i < s.size() && s[i] == ']') { ++i; break; }
                    ok = fail("expected ',' or ']'");
                    break;
                }
            }
        } else if (c == '"') {
            v.kind = Json::String;
            ok = string(v.str);
        } else if (c == 't') { v.kind = Json::Bool; v.b = true; ok = lit("true"); }
        else if (c == 'f') { v.kind = Json::Bool; v.b = false; ok = lit("false"); }
        else if (c == 'n') { v.kind = Json::Null; ok = lit("null"); }
        else ok = number(v);
        --depth;
        return ok;
    }
};

}  // namespace

std::string json_parse(const std::string& text, Json& out) {
    P p{text};
    if (!p.value(out)) return p.err;
    p.ws();
    if (p.i != text.size()) { p.fail("trailing characters"); return p.err; }
    return "";
}

}  // namespace rt
