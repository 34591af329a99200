// pt_json.hpp — minimal JSON reader for the scene schema (the role serde_json
// plays for Scene::from_json, src/world/mod.rs:46-49).  Numbers are parsed with
// std::from_chars (correctly rounded, like serde_json on the values scenes use,
// and independent of the host application's locale, which strtod is not).
// Nesting is limited to 128 levels, serde_json's default recursion limit, so a
// hostile file cannot exhaust the caller's stack.
#pragma once

#include <charconv>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace ptjson {

struct ParseError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

struct Value {
    enum Kind { Null, Bool, Number, String, Array, Object } kind = Null;
    bool b = false;
    double num = 0.0;
    bool is_integer = false;  // literal had no fraction/exponent
    std::string str;
    std::vector<Value> arr;
    std::vector<std::pair<std::string, Value>> obj;  // file order kept

    const Value *find(const char *key) const {
        for (auto &kv : obj)
            if (kv.first == key) return &kv.second;
        return nullptr;
    }
    const char *kind_name() const {
        static const char *n[] = {"null", "boolean", "number", "string", "sequence", "map"};
        return n[kind];
    }
};

class Parser {
  public:
    Parser(const char *s, size_t n) : p_(s), end_(s + n), begin_(s) {}

    Value parse() {
        Value v = value();
        ws();
        if (p_ != end_) fail("trailing characters");
        return v;
    }

  private:
    static constexpr int kMaxDepth = 128;  // serde_json's recursion limit
    const char *p_, *end_, *begin_;
    int depth_ = 0;

    [[noreturn]] void fail(const std::string &what) {
        size_t line = 1, col = 1;
        for (const char *q = begin_; q < p_ && q < end_; ++q) {
            if (*q == '\n') {
                line++;
                col = 1;
            } else {
                col++;
            }
        }
        throw ParseError(what + " at line " + std::to_string(line) + " column " + std::to_string(col));
    }
    void ws() {
        while (p_ < end_ && (*p_ == ' ' || *p_ == '\t' || *p_ == '\n' || *p_ == '\r')) ++p_;
    }
    bool lit(const char *s) {
        size_t n = std::strlen(s);
        if ((size_t)(end_ - p_) >= n && std::memcmp(p_, s, n) == 0) {
            p_ += n;
            return true;
        }
        return false;
    }
    struct Nest {  // one level of array / object nesting
        Parser &p;
        explicit Nest(Parser &q) : p(q) {
            if (++p.depth_ > kMaxDepth) p.fail("recursion limit exceeded");
        }
        ~Nest() { --p.depth_; }
    };
    Value value() {
        ws();
        if (p_ >= end_) fail("EOF while parsing a value");
        Value v;
        char c = *p_;
        if (c == '{') {
            Nest n(*this);
            return object();
        }
        if (c == '[') {
            Nest n(*this);
            return array();
        }
        if (c == '"') {
            v.kind = Value::String;
            v.str = string();
            return v;
        }
        if (lit("true")) {
            v.kind = Value::Bool;
            v.b = true;
            return v;
        }
        if (lit("false")) {
            v.kind = Value::Bool;
            return v;
        }
        if (lit("null")) return v;
        if (c == '-' || (c >= '0' && c <= '9')) return number();
        fail("expected value");
    }
    Value number() {
        const char *s = p_;
        if (*p_ == '-') ++p_;
        if (p_ >= end_ || !(*p_ >= '0' && *p_ <= '9')) fail("invalid number");
        if (*p_ == '0') {
            ++p_;
        } else {
            while (p_ < end_ && *p_ >= '0' && *p_ <= '9') ++p_;
        }
        bool integer = true;
        if (p_ < end_ && *p_ == '.') {
            integer = false;
            ++p_;
            if (p_ >= end_ || !(*p_ >= '0' && *p_ <= '9')) fail("invalid number");
            while (p_ < end_ && *p_ >= '0' && *p_ <= '9') ++p_;
        }
        if (p_ < end_ && (*p_ == 'e' || *p_ == 'E')) {
            integer = false;
            ++p_;
            if (p_ < end_ && (*p_ == '+' || *p_ == '-')) ++p_;
            if (p_ >= end_ || !(*p_ >= '0' && *p_ <= '9')) fail("invalid number");
            while (p_ < end_ && *p_ >= '0' && *p_ <= '9') ++p_;
        }
        Value v;
        v.kind = Value::Number;
        const auto r = std::from_chars(s, p_, v.num);  // JSON's grammar is a subset of from_chars' general format
        if (r.ec == std::errc::result_out_of_range) {
            // serde_json: an overflow is "number out of range", an underflow rounds to a (signed) zero
            if (decimal_exponent(s, p_) >= 0) fail("number out of range");
            v.num = *s == '-' ? -0.0 : 0.0;
        } else if (r.ec != std::errc() || r.ptr != p_) {
            fail("invalid number");
        }
        v.is_integer = integer;
        return v;
    }
    // floor(log10 |x|) of a valid JSON number literal with a non-zero digit (else -1): the position of its
    // first non-zero digit relative to the decimal point, plus the explicit exponent
    static long decimal_exponent(const char *s, const char *e) {
        const char *q = *s == '-' ? s + 1 : s;
        long int_digits = 0, first_int = 0, frac_place = 0, mag = 0;
        bool frac = false, seen = false;
        for (; q < e && *q != 'e' && *q != 'E'; ++q) {
            if (*q == '.') {
                frac = true;
            } else if (!frac) {
                int_digits++;
                if (!seen && *q != '0') seen = true, first_int = int_digits;
            } else {
                frac_place++;
                if (!seen && *q != '0') seen = true, mag = -frac_place;
            }
        }
        if (!seen) return -1;
        if (first_int) mag = int_digits - first_int;
        long exp10 = 0;
        if (q < e) {  // exponent part
            ++q;
            bool neg = false;
            if (*q == '+' || *q == '-') neg = *q++ == '-';
            for (; q < e; ++q) exp10 = exp10 < 100000000 ? exp10 * 10 + (*q - '0') : exp10;
            if (neg) exp10 = -exp10;
        }
        return mag + exp10;
    }
    static void put_utf8(std::string &o, unsigned cp) {
        if (cp < 0x80) {
            o += (char)cp;
        } else if (cp < 0x800) {
            o += (char)(0xC0 | (cp >> 6));
            o += (char)(0x80 | (cp & 0x3F));
        } else if (cp < 0x10000) {
            o += (char)(0xE0 | (cp >> 12));
            o += (char)(0x80 | ((cp >> 6) & 0x3F));
            o += (char)(0x80 | (cp & 0x3F));
        } else {
            o += (char)(0xF0 | (cp >> 18));
            o += (char)(0x80 | ((cp >> 12) & 0x3F));
            o += (char)(0x80 | ((cp >> 6) & 0x3F));
            o += (char)(0x80 | (cp & 0x3F));
        }
    }
    unsigned hex4() {
        if (end_ - p_ < 4) fail("EOF in \\u escape");
        unsigned v = 0;
        for (int i = 0; i < 4; i++) {
            char c = *p_++;
            v <<= 4;
            if (c >= '0' && c <= '9') v |= c - '0';
            else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
            else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
            else fail("invalid \\u escape");
        }
        return v;
    }
    std::string string() {
        ++p_;  // opening quote
        std::string o;
        for (;;) {
            if (p_ >= end_) fail("EOF while parsing a string");
            char c = *p_++;
            if (c == '"') break;
            if ((unsigned char)c < 0x20) fail("control character in string");
            if (c != '\\') {
                o += c;
                continue;
            }
            if (p_ >= end_) fail("EOF in escape");
            char e = *p_++;
            switch (e) {
            case '"': o += '"'; break;
            case '\\': o += '\\'; break;
            case '/': o += '/'; break;
            case 'b': o += '\b'; break;
            case 'f': o += '\f'; break;
            case 'n': o += '\n'; break;
            case 'r': o += '\r'; break;
            case 't': o += '\t'; break;
            case 'u': {
                unsigned cp = hex4();
                if (cp >= 0xDC00 && cp < 0xE000) fail("lone trailing surrogate in hex escape");
                if (cp >= 0xD800 && cp < 0xDC00) {
                    if (!(lit("\\u"))) fail("lone leading surrogate in hex escape");
                    unsigned lo = hex4();
                    if (lo < 0xDC00 || lo >= 0xE000) fail("invalid low surrogate in hex escape");
                    cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
                }
                put_utf8(o, cp);
                break;
            }
            default: fail("invalid escape");
            }
        }
        return o;
    }
    Value array() {
        ++p_;
        Value v;
        v.kind = Value::Array;
        ws();
        if (p_ < end_ && *p_ == ']') {
            ++p_;
            return v;
        }
        for (;;) {
            v.arr.push_back(value());
            ws();
            if (p_ >= end_) fail("EOF while parsing a list");
            if (*p_ == ',') {
                ++p_;
                continue;
            }
            if (*p_ == ']') {
                ++p_;
                return v;
            }
            fail("expected `,` or `]`");
        }
    }
    Value object() {
        ++p_;
        Value v;
        v.kind = Value::Object;
        ws();
        if (p_ < end_ && *p_ == '}') {
            ++p_;
            return v;
        }
        for (;;) {
            ws();
            if (p_ >= end_ || *p_ != '"') fail("key must be a string");
            std::string k = string();
            ws();
            if (p_ >= end_ || *p_ != ':') fail("expected `:`");
            ++p_;
            v.obj.emplace_back(std::move(k), value());
            ws();
            if (p_ >= end_) fail("EOF while parsing an object");
            if (*p_ == ',') {
                ++p_;
                continue;
            }
            if (*p_ == '}') {
                ++p_;
                return v;
            }
            fail("expected `,` or `}`");
        }
    }
};

inline Value parse(const char *s, size_t n) { return Parser(s, n).parse(); }

}  // namespace ptjson
