// json.hpp -- a small JSON DOM with boost::property_tree read semantics.
//
// The reference reads both of its inputs (the MP5 shape JSON and the mc-settings JSON) with
// boost::property_tree::read_json (object_factory.hpp:741-758, polygoniser_settings.hpp:161-164).
// ptree keeps every scalar as its source text and converts on access with a C++ stream, so a
// numeric field read as float is strtof of the text, an int read of "1.5" or "true" fails (and a
// get<>(path, default) then returns the default), and a bool read accepts true/false/1/0.
// This DOM keeps the same model: scalars are text, conversions happen at the accessor.
#pragma once
#include <cerrno>
#include <climits>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace impli {

struct JsonError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

class Json {
public:
    enum Kind { Null, Scalar, Array, Object };
    Kind kind = Null;
    std::string text;                                   // Scalar: source text (strings unquoted)
    bool quoted = false;                                // Scalar came from a JSON string
    std::vector<std::pair<std::string, Json>> items;    // Array (empty keys) / Object

    static Json parse(const char* s) {
        Parser p{s, s + std::strlen(s)};
        p.ws();
        Json j = p.value();
        p.ws();
        if (p.c != p.e) throw JsonError("trailing characters in JSON");
        return j;
    }

    // property-tree style lookup ("box.xmin"); nullptr when absent
    const Json* find(const std::string& path) const {
        const Json* cur = this;
        size_t pos = 0;
        while (true) {
            size_t dot = path.find('.', pos);
            std::string key = path.substr(pos, dot == std::string::npos ? std::string::npos : dot - pos);
            if (cur->kind != Object) return nullptr;
            const Json* next = nullptr;
            for (auto& kv : cur->items)
                if (kv.first == key) { next = &kv.second; break; }
            if (!next) return nullptr;
            cur = next;
            if (dot == std::string::npos) return cur;
            pos = dot + 1;
        }
    }

    // get<float>(path, default): strtof of the whole text, default on absence or bad data
    bool get_float(const std::string& path, float* out) const {
        const Json* j = find(path);
        return j && j->as_float(out);
    }
    float get_float(const std::string& path, float dflt) const {
        float v;
        return get_float(path, &v) ? v : dflt;
    }
    int get_int(const std::string& path, int dflt) const {
        const Json* j = find(path);
        int v;
        return (j && j->as_int(&v)) ? v : dflt;
    }
    bool get_bool(const std::string& path, bool dflt) const {
        const Json* j = find(path);
        if (!j || j->kind != Scalar) return dflt;
        std::string t = trim(j->text);
        if (t == "true" || t == "1") return true;
        if (t == "false" || t == "0") return false;
        return dflt;
    }
    std::string get_string(const std::string& path, const std::string& dflt) const {
        const Json* j = find(path);
        return (j && j->kind == Scalar) ? j->text : dflt;
    }

    bool as_float(float* out) const {
        if (kind != Scalar) return false;
        std::string t = trim(text);
        if (t.empty()) return false;
        char* end = nullptr;
        float v = std::strtof(t.c_str(), &end);
        if (end != t.c_str() + t.size()) return false;
        *out = v;
        return true;
    }
    bool as_int(int* out) const {
        if (kind != Scalar) return false;
        std::string t = trim(text);
        if (t.empty()) return false;
        char* end = nullptr;
        errno = 0;
        long v = std::strtol(t.c_str(), &end, 10);
        if (end != t.c_str() + t.size()) return false;
        if (errno == ERANGE || v < INT_MIN || v > INT_MAX) return false;   // a stream read into int fails too
        *out = (int)v;
        return true;
    }

private:
    static std::string trim(const std::string& s) {
        size_t a = s.find_first_not_of(" \t\r\n"), b = s.find_last_not_of(" \t\r\n");
        return a == std::string::npos ? std::string() : s.substr(a, b - a + 1);
    }

    // nesting bound: the parser recurses per array / object level, so untrusted input could
    // otherwise exhaust the stack (the MP5 compiler itself stops at kMaxDepth levels of nodes)
    static constexpr int kMaxNesting = 256;

    struct Parser {
        const char* c;
        const char* e;
        int nest = 0;
        struct Level {
            Parser* p;
            explicit Level(Parser* q) : p(q) {
                if (++p->nest > kMaxNesting) p->fail("nested too deeply");
            }
            ~Level() { --p->nest; }
        };
        void ws() { while (c < e && (*c == ' ' || *c == '\t' || *c == '\n' || *c == '\r')) ++c; }
        [[noreturn]] void fail(const char* m) { throw JsonError(std::string("JSON parse error: ") + m); }
        Json value() {
            ws();
            if (c >= e) fail("unexpected end");
            if (*c == '{') return object();
            if (*c == '[') return array();
            if (*c == '"') {
                Json j;
                j.kind = Scalar;
                j.quoted = true;
                j.text = str();
                return j;
            }
            const char* s = c;
            while (c < e && *c != ',' && *c != '}' && *c != ']' && *c != ' ' && *c != '\n' && *c != '\r' && *c != '\t') ++c;
            if (c == s) fail("empty value");
            Json j;
            std::string tok(s, c);
            if (tok == "null") { j.kind = Scalar; j.text = "null"; return j; }   // ptree stores "null"
            j.kind = Scalar;
            j.text = tok;
            return j;
        }
        std::string str() {
            ++c;
            std::string out;
            while (c < e && *c != '"') {
                if (*c == '\\') {
                    ++c;
                    if (c >= e) fail("bad escape");
                    switch (*c) {
                        case 'n': out += '\n'; break;
                        case 't': out += '\t'; break;
                        case 'r': out += '\r'; break;
                        case 'b': out += '\b'; break;
                        case 'f': out += '\f'; break;
                        case 'u': {
                            if (e - c < 5) fail("bad \\u escape");
                            unsigned cp = (unsigned)std::strtoul(std::string(c + 1, c + 5).c_str(), nullptr, 16);
                            if (cp < 0x80) out += (char)cp;
                            else if (cp < 0x800) { out += (char)(0xC0 | (cp >> 6)); out += (char)(0x80 | (cp & 0x3F)); }
                            else { out += (char)(0xE0 | (cp >> 12)); out += (char)(0x80 | ((cp >> 6) & 0x3F)); out += (char)(0x80 | (cp & 0x3F)); }
                            c += 4;
                            break;
                        }
                        default: out += *c;
                    }
                    ++c;
                } else {
                    out += *c++;
                }
            }
            if (c >= e) fail("unterminated string");
            ++c;
            return out;
        }
        Json array() {
            Level lv(this);
            Json j;
            j.kind = Array;
            ++c;
            ws();
            if (c < e && *c == ']') { ++c; return j; }
            while (true) {
                j.items.emplace_back(std::string(), value());
                ws();
                if (c < e && *c == ',') { ++c; continue; }
                if (c < e && *c == ']') { ++c; break; }
                fail("expected , or ]");
            }
            return j;
        }
        Json object() {
            Level lv(this);
            Json j;
            j.kind = Object;
            ++c;
            ws();
            if (c < e && *c == '}') { ++c; return j; }
            while (true) {
                ws();
                if (c >= e || *c != '"') fail("expected key");
                std::string k = str();
                ws();
                if (c >= e || *c != ':') fail("expected :");
                ++c;
                j.items.emplace_back(k, value());
                ws();
                if (c < e && *c == ',') { ++c; continue; }
                if (c < e && *c == '}') { ++c; break; }
                fail("expected , or }");
            }
            return j;
        }
    };
};

}  // namespace impli
