// pt_json.hpp — minimal JSON reader for the scene schema (the role serde_json
// plays for Scene::from_json, src/world/mod.rs:46-49).  Numbers are parsed with
// strtod (correctly rounded, like serde_json on the values scenes use).
#pragma once

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
    const char *p_, *end_, *begin_;

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
    Value value() {
        ws();
        if (p_ >= end_) fail("EOF while parsing a value");
        Value v;
        char c = *p_;
        if (c == '{') return object();
        if (c == '[') return array();
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
        std::string tok(s, p_);
        Value v;
        v.kind = Value::Number;
        v.num = std::strtod(tok.c_str(), nullptr);
        v.is_integer = integer;
        return v;
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
                if (cp >= 0xD800 && cp < 0xDC00) {
                    if (!(lit("\\u"))) fail("lone surrogate");
                    unsigned lo = hex4();
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
