// Minimal JSON value / parser / serializer for the stdio protocol.  Serialisation follows Python's
// json.dumps(obj, ensure_ascii=False) byte-for-byte: ", " and ": " separators, shortest round-trip float
// repr (1.0, 0.25, 1e-05), non-ASCII emitted as UTF-8, control characters escaped.
#pragma once
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace qjson {

struct Value {
    enum Type { Null, Bool, Int, Float, Str, Arr, Obj } type = Null;
    bool b = false;
    int64_t i = 0;
    double f = 0;
    std::string s;
    std::vector<Value> a;
    std::vector<std::pair<std::string, Value>> o;  // insertion order (Python dicts keep it)

    Value() = default;
    static Value null() { return Value(); }
    static Value boolean(bool v) { Value x; x.type = Bool; x.b = v; return x; }
    static Value integer(int64_t v) { Value x; x.type = Int; x.i = v; return x; }
    static Value number(double v) { Value x; x.type = Float; x.f = v; return x; }
    static Value str(const std::string& v) { Value x; x.type = Str; x.s = v; return x; }
    static Value object() { Value x; x.type = Obj; return x; }

    const Value* get(const std::string& k) const {
        if (type != Obj) return nullptr;
        for (auto& kv : o)
            if (kv.first == k) return &kv.second;
        return nullptr;
    }
    Value& set(const std::string& k, Value v) {
        for (auto& kv : o)
            if (kv.first == k) { kv.second = std::move(v); return kv.second; }
        o.emplace_back(k, std::move(v));
        return o.back().second;
    }
    bool truthy() const {  // Python truthiness
        switch (type) {
            case Null: return false;
            case Bool: return b;
            case Int: return i != 0;
            case Float: return f != 0;
            case Str: return !s.empty();
            case Arr: return !a.empty();
            case Obj: return !o.empty();
        }
        return false;
    }
};

struct ParseError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

class Parser {
   public:
    Parser(const char* p, size_t n) : p_(p), e_(p + n) {}
    Value parse() {
        ws();
        Value v = value();
        ws();
        if (p_ != e_) throw ParseError("trailing data");
        return v;
    }

   private:
    const char *p_, *e_;
    void ws() {
        while (p_ < e_ && (*p_ == ' ' || *p_ == '\t' || *p_ == '\n' || *p_ == '\r')) p_++;
    }
    char peek() { return p_ < e_ ? *p_ : 0; }
    void expect(char c) {
        if (peek() != c) throw ParseError("unexpected character");
        p_++;
    }
    bool lit(const char* s) {
        size_t n = strlen(s);
        if ((size_t)(e_ - p_) >= n && !memcmp(p_, s, n)) { p_ += n; return true; }
        return false;
    }
    Value value() {
        char c = peek();
        if (c == '{') return object();
        if (c == '[') return array();
        if (c == '"') return Value::str(string());
        if (lit("true")) return Value::boolean(true);
        if (lit("false")) return Value::boolean(false);
        if (lit("null")) return Value::null();
        if (lit("NaN")) return Value::number(NAN);
        if (lit("Infinity")) return Value::number(INFINITY);
        if (lit("-Infinity")) return Value::number(-INFINITY);
        if (c == '-' || (c >= '0' && c <= '9')) return number();
        throw ParseError("unexpected token");
    }
    Value object() {
        expect('{');
        Value v = Value::object();
        ws();
        if (peek() == '}') { p_++; return v; }
        for (;;) {
            ws();
            std::string k = string();
            ws();
            expect(':');
            ws();
            v.set(k, value());
            ws();
            if (peek() == ',') { p_++; continue; }
            expect('}');
            return v;
        }
    }
    Value array() {
        expect('[');
        Value v;
        v.type = Value::Arr;
        ws();
        if (peek() == ']') { p_++; return v; }
        for (;;) {
            ws();
            v.a.push_back(value());
            ws();
            if (peek() == ',') { p_++; continue; }
            expect(']');
            return v;
        }
    }
    Value number() {
        const char* s = p_;
        bool flt = false;
        if (peek() == '-') p_++;
        if (!(peek() >= '0' && peek() <= '9')) throw ParseError("bad number");
        while (peek() >= '0' && peek() <= '9') p_++;
        if (peek() == '.') { flt = true; p_++; while (peek() >= '0' && peek() <= '9') p_++; }
        if (peek() == 'e' || peek() == 'E') {
            flt = true;
            p_++;
            if (peek() == '+' || peek() == '-') p_++;
            while (peek() >= '0' && peek() <= '9') p_++;
        }
        std::string t(s, p_);
        if (!flt) {
            errno = 0;
            long long v = strtoll(t.c_str(), nullptr, 10);
            if (errno == 0) return Value::integer(v);
        }
        return Value::number(strtod(t.c_str(), nullptr));
    }
    static void put_utf8(std::string& o, uint32_t cp) {
        if (cp < 0x80) o += (char)cp;
        else if (cp < 0x800) { o += (char)(0xC0 | (cp >> 6)); o += (char)(0x80 | (cp & 0x3F)); }
        else if (cp < 0x10000) {
            o += (char)(0xE0 | (cp >> 12)); o += (char)(0x80 | ((cp >> 6) & 0x3F)); o += (char)(0x80 | (cp & 0x3F));
        } else {
            o += (char)(0xF0 | (cp >> 18)); o += (char)(0x80 | ((cp >> 12) & 0x3F));
            o += (char)(0x80 | ((cp >> 6) & 0x3F)); o += (char)(0x80 | (cp & 0x3F));
        }
    }
    uint32_t hex4() {
        if (e_ - p_ < 4) throw ParseError("bad escape");
        uint32_t v = 0;
        for (int k = 0; k < 4; k++) {
            char c = *p_++;
            v <<= 4;
            if (c >= '0' && c <= '9') v |= c - '0';
            else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
            else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
            else throw ParseError("bad escape");
        }
        return v;
    }
    std::string string() {
        expect('"');
        std::string o;
        const char* run = p_;
        while (p_ < e_) {
            char c = *p_;
            if (c == '"') {
                o.append(run, p_);
                p_++;
                return o;
            }
            if ((unsigned char)c < 0x20) throw ParseError("control character in string");
            if (c == '\\') {
                o.append(run, p_);
                p_++;
                char k = peek();
                p_++;
                switch (k) {
                    case '"': o += '"'; break;
                    case '\\': o += '\\'; break;
                    case '/': o += '/'; break;
                    case 'b': o += '\b'; break;
                    case 'f': o += '\f'; break;
                    case 'n': o += '\n'; break;
                    case 'r': o += '\r'; break;
                    case 't': o += '\t'; break;
                    case 'u': {
                        uint32_t cp = hex4();
                        if (cp >= 0xD800 && cp < 0xDC00 && e_ - p_ >= 6 && p_[0] == '\\' && p_[1] == 'u') {
                            const char* save = p_;
                            p_ += 2;
                            uint32_t lo = hex4();
                            if (lo >= 0xDC00 && lo < 0xE000) cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
                            else p_ = save;
                        }
                        put_utf8(o, cp);
                        break;
                    }
                    default: throw ParseError("bad escape");
                }
                run = p_;
                continue;
            }
            p_++;
        }
        throw ParseError("unterminated string");
    }
};

inline Value parse(const std::string& s) { return Parser(s.data(), s.size()).parse(); }

// Python float repr
inline std::string float_repr(double v) {
    if (std::isnan(v)) return "NaN";
    if (std::isinf(v)) return v > 0 ? "Infinity" : "-Infinity";
    char buf[64];
    int prec = 1;
    for (; prec <= 17; prec++) {
        snprintf(buf, sizeof buf, "%.*e", prec - 1, v);
        if (strtod(buf, nullptr) == v) break;
    }
    // buf = d.ddde±XX with `prec` significant digits
    char* e = strchr(buf, 'e');
    int exp10 = atoi(e + 1);
    std::string mant(buf, e);
    bool neg = mant[0] == '-';
    if (neg) mant.erase(0, 1);
    std::string digits;
    for (char c : mant)
        if (c != '.') digits += c;
    while (digits.size() > 1 && digits.back() == '0') digits.pop_back();
    std::string out;
    if (exp10 < -4 || exp10 >= 16) {
        out = digits.substr(0, 1);
        if (digits.size() > 1) out += "." + digits.substr(1);
        char eb[16];
        snprintf(eb, sizeof eb, "e%c%02d", exp10 < 0 ? '-' : '+', exp10 < 0 ? -exp10 : exp10);
        out += eb;
    } else if (exp10 < 0) {
        out = "0." + std::string((size_t)(-exp10 - 1), '0') + digits;
    } else {
        if ((int)digits.size() <= exp10 + 1) {
            out = digits + std::string((size_t)(exp10 + 1 - (int)digits.size()), '0') + ".0";
        } else {
            out = digits.substr(0, (size_t)exp10 + 1) + "." + digits.substr((size_t)exp10 + 1);
        }
    }
    return neg ? "-" + out : out;
}

inline void dump_str(std::string& o, const std::string& s) {
    o += '"';
    for (unsigned char c : s) {
        switch (c) {
            case '"': o += "\\\""; break;
            case '\\': o += "\\\\"; break;
            case '\n': o += "\\n"; break;
            case '\r': o += "\\r"; break;
            case '\t': o += "\\t"; break;
            case '\b': o += "\\b"; break;
            case '\f': o += "\\f"; break;
            default:
                if (c < 0x20) {
                    char b[8];
                    snprintf(b, sizeof b, "\\u%04x", c);
                    o += b;
                } else {
                    o += (char)c;
                }
        }
    }
    o += '"';
}

inline void dump(std::string& o, const Value& v) {
    switch (v.type) {
        case Value::Null: o += "null"; break;
        case Value::Bool: o += v.b ? "true" : "false"; break;
        case Value::Int: o += std::to_string(v.i); break;
        case Value::Float: o += float_repr(v.f); break;
        case Value::Str: dump_str(o, v.s); break;
        case Value::Arr:
            o += '[';
            for (size_t k = 0; k < v.a.size(); k++) {
                if (k) o += ", ";
                dump(o, v.a[k]);
            }
            o += ']';
            break;
        case Value::Obj:
            o += '{';
            for (size_t k = 0; k < v.o.size(); k++) {
                if (k) o += ", ";
                dump_str(o, v.o[k].first);
                o += ": ";
                dump(o, v.o[k].second);
            }
            o += '}';
            break;
    }
}

inline std::string dumps(const Value& v) {
    std::string o;
    dump(o, v);
    return o;
}

}  // namespace qjson
