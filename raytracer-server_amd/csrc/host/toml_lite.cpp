#include "toml_lite.hpp"

#include <cmath>
#include <cstdlib>
#include <stdexcept>

namespace rt::toml {

const Value* Value::get(const std::string& key) const {
    for (const auto& kv : table)
        if (kv.first == key) return &kv.second;
    return nullptr;
}
Value* Value::get_mut(const std::string& key) {
    for (auto& kv : table)
        if (kv.first == key) return &kv.second;
    return nullptr;
}

const char* kind_name(Value::Kind k) {
    switch (k) {
        case Value::Kind::Table: return "table";
        case Value::Kind::Array: return "array";
        case Value::Kind::String: return "string";
        case Value::Kind::Int: return "integer";
        case Value::Kind::Float: return "float";
        case Value::Kind::Bool: return "boolean";
    }
    return "?";
}

namespace {

struct ParseError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

class Parser {
   public:
    explicit Parser(const std::string& s) : s_(s) {}

    void run(Value* root) {
        root->kind = Value::Kind::Table;
        Value* cur = root;
        while (true) {
            skip_ws_comments_newlines();
            if (eof()) break;
            char c = peek();
            if (c == '[') {
                bool aot = s_.compare(p_, 2, "[[") == 0;
                p_ += aot ? 2 : 1;
                std::vector<std::string> path = parse_key_path();
                skip_ws();
                if (aot) expect("]]");
                else expect("]");
                expect_line_end();
                cur = open_header(root, path, aot);
            } else {
                std::vector<std::string> path = parse_key_path();
                skip_ws();
                expect("=");
                skip_ws();
                Value v = parse_value();
                assign(cur, path, std::move(v));
                expect_line_end();
            }
        }
    }

    int line() const {
        int l = 1;
        for (size_t i = 0; i < p_ && i < s_.size(); ++i)
            if (s_[i] == '\n') ++l;
        return l;
    }

   private:
    const std::string& s_;
    size_t p_ = 0;

    bool eof() const { return p_ >= s_.size(); }
    char peek() const { return eof() ? '\0' : s_[p_]; }
    [[noreturn]] void fail(const std::string& m) { throw ParseError(m); }

    void skip_ws() {
        while (!eof() && (s_[p_] == ' ' || s_[p_] == '\t')) ++p_;
    }
    void skip_comment() {
        if (peek() == '#')
            while (!eof() && s_[p_] != '\n') ++p_;
    }
    void skip_ws_comments_newlines() {
        while (!eof()) {
            char c = s_[p_];
            if (c == ' ' || c == '\t' || c == '\r' || c == '\n') ++p_;
            else if (c == '#') skip_comment();
            else break;
        }
    }
    void expect(const char* t) {
        size_t n = std::char_traits<char>::length(t);
        if (s_.compare(p_, n, t) != 0) fail(std::string("expected '") + t + "'");
        p_ += n;
    }
    void expect_line_end() {
        skip_ws();
        skip_comment();
        if (eof()) return;
        if (peek() == '\r') ++p_;
        if (peek() != '\n') fail("expected end of line");
        ++p_;
    }

    static bool bare_char(char c) {
        return (c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z') || (c >= '0' && c <= '9') || c == '_' || c == '-';
    }
    std::string parse_key() {
        skip_ws();
        char c = peek();
        if (c == '"') return parse_basic_string();
        if (c == '\'') return parse_literal_string();
        size_t st = p_;
        while (!eof() && bare_char(s_[p_])) ++p_;
        if (st == p_) fail("expected a key");
        return s_.substr(st, p_ - st);
    }
    std::vector<std::string> parse_key_path() {
        std::vector<std::string> path{parse_key()};
        skip_ws();
        while (peek() == '.') {
            ++p_;
            path.push_back(parse_key());
            skip_ws();
        }
        return path;
    }

    static void append_utf8(std::string& out, uint32_t cp) {
        if (cp < 0x80) out += (char)cp;
        else if (cp < 0x800) { out += (char)(0xC0 | (cp >> 6)); out += (char)(0x80 | (cp & 0x3F)); }
        else if (cp < 0x10000) { out += (char)(0xE0 | (cp >> 12)); out += (char)(0x80 | ((cp >> 6) & 0x3F)); out += (char)(0x80 | (cp & 0x3F)); }
        else { out += (char)(0xF0 | (cp >> 18)); out += (char)(0x80 | ((cp >> 12) & 0x3F)); out += (char)(0x80 | ((cp >> 6) & 0x3F)); out += (char)(0x80 | (cp & 0x3F)); }
    }
    std::string parse_basic_string() {
        if (s_.compare(p_, 3, "\"\"\"") == 0) fail("multi-line strings are not supported");
        ++p_;
        std::string out;
        while (true) {
            if (eof() || peek() == '\n') fail("unterminated string");
            char c = s_[p_++];
            if (c == '"') break;
            if (c != '\\') { out += c; continue; }
            if (eof()) fail("unterminated escape");
            char e = s_[p_++];
            switch (e) {
                case 'b': out += '\b'; break;
                case 't': out += '\t'; break;
                case 'n': out += '\n'; break;
                case 'f': out += '\f'; break;
                case 'r': out += '\r'; break;
                case '"': out += '"'; break;
                case '\\': out += '\\'; break;
                case 'u': case 'U': {
                    int n = e == 'u' ? 4 : 8;
                    if (p_ + n > s_.size()) fail("bad unicode escape");
                    uint32_t cp = (uint32_t)std::strtoul(s_.substr(p_, n).c_str(), nullptr, 16);
                    p_ += n;
                    append_utf8(out, cp);
                    break;
                }
                default: fail("bad escape");
            }
        }
        return out;
    }
    std::string parse_literal_string() {
        if (s_.compare(p_, 3, "'''") == 0) fail("multi-line strings are not supported");
        ++p_;
        size_t st = p_;
        while (!eof() && s_[p_] != '\'' && s_[p_] != '\n') ++p_;
        if (peek() != '\'') fail("unterminated string");
        std::string out = s_.substr(st, p_ - st);
        ++p_;
        return out;
    }

    Value parse_value() {
        Value v;
        char c = peek();
        if (c == '"' || c == '\'') {
            v.kind = Value::Kind::String;
            v.str = c == '"' ? parse_basic_string() : parse_literal_string();
            return v;
        }
        if (c == '[') return parse_array();
        if (c == '{') return parse_inline_table();
        if (s_.compare(p_, 4, "true") == 0 && !bare_char(p_ + 4 < s_.size() ? s_[p_ + 4] : ' ')) {
            p_ += 4; v.kind = Value::Kind::Bool; v.b = true; return v;
        }
        if (s_.compare(p_, 5, "false") == 0 && !bare_char(p_ + 5 < s_.size() ? s_[p_ + 5] : ' ')) {
            p_ += 5; v.kind = Value::Kind::Bool; v.b = false; return v;
        }
        return parse_number();
    }

    Value parse_number() {
        size_t st = p_;
        while (!eof()) {
            char c = s_[p_];
            if (bare_char(c) || c == '+' || c == '.') ++p_;
            else break;
        }
        std::string tok = s_.substr(st, p_ - st);
        if (tok.empty()) fail("expected a value");
        std::string clean;
        for (size_t i = 0; i < tok.size(); ++i) {
            if (tok[i] == '_') {
                if (i == 0 || i + 1 == tok.size() || !std::isdigit((unsigned char)tok[i - 1]) || !std::isdigit((unsigned char)tok[i + 1]))
                    fail("bad underscore in number '" + tok + "'");
                continue;
            }
            clean += tok[i];
        }
        Value v;
        std::string body = clean;
        bool neg = false;
        if (!body.empty() && (body[0] == '+' || body[0] == '-')) { neg = body[0] == '-'; body = body.substr(1); }
        if (body == "inf" || body == "nan") {
            v.kind = Value::Kind::Float;
            v.f = body == "inf" ? (neg ? -INFINITY : INFINITY) : NAN;
            return v;
        }
        if (body.size() > 2 && body[0] == '0' && (body[1] == 'x' || body[1] == 'o' || body[1] == 'b')) {
            int base = body[1] == 'x' ? 16 : body[1] == 'o' ? 8 : 2;
            char* end = nullptr;
            long long x = std::strtoll(body.c_str() + 2, &end, base);
            if (*end) fail("bad integer '" + tok + "'");
            v.kind = Value::Kind::Int;
            v.i = neg ? -x : x;
            return v;
        }
        bool is_float = body.find_first_of(".eE") != std::string::npos;
        if (body.empty() || !std::isdigit((unsigned char)body[0])) fail("bad number '" + tok + "'");
        if (body.size() > 1 && body[0] == '0' && std::isdigit((unsigned char)body[1])) fail("leading zero in '" + tok + "'");
        char* end = nullptr;
        if (is_float) {
            if (body.back() == '.' || body.find(".e") != std::string::npos || body.find(".E") != std::string::npos)
                fail("bad float '" + tok + "'");
            double x = std::strtod(clean.c_str(), &end);
            if (*end) fail("bad float '" + tok + "'");
            v.kind = Value::Kind::Float;
            v.f = x;
        } else {
            errno = 0;
            long long x = std::strtoll(clean.c_str(), &end, 10);
            if (*end || errno) fail("bad integer '" + tok + "'");
            v.kind = Value::Kind::Int;
            v.i = x;
        }
        return v;
    }

    Value parse_array() {
        ++p_;  // '['
        Value v;
        v.kind = Value::Kind::Array;
        while (true) {
            skip_ws_comments_newlines();
            if (peek() == ']') { ++p_; break; }
            v.array.push_back(parse_value());
            skip_ws_comments_newlines();
            if (peek() == ',') { ++p_; continue; }
            if (peek() == ']') { ++p_; break; }
            fail("expected ',' or ']' in array");
        }
        return v;
    }

    Value parse_inline_table() {
        ++p_;  // '{'
        Value v;
        v.kind = Value::Kind::Table;
        v.defined = true;
        skip_ws();
        if (peek() == '}') { ++p_; return v; }
        while (true) {
            skip_ws_comments_newlines();
            std::vector<std::string> path = parse_key_path();
            skip_ws();
            expect("=");
            skip_ws();
            Value x = parse_value();
            assign(&v, path, std::move(x));
            skip_ws_comments_newlines();
            if (peek() == ',') { ++p_; continue; }
            if (peek() == '}') { ++p_; break; }
            fail("expected ',' or '}' in inline table");
        }
        return v;
    }

    Value* descend(Value* t, const std::string& k, bool create) {
        Value* x = t->get_mut(k);
        if (!x) {
            if (!create) return nullptr;
            Value nt;
            nt.kind = Value::Kind::Table;
            t->table.emplace_back(k, std::move(nt));
            return &t->table.back().second;
        }
        if (x->kind == Value::Kind::Array && x->array_of_tables) return &x->array.back();
        if (x->kind != Value::Kind::Table) fail("key '" + k + "' is not a table");
        return x;
    }

    void assign(Value* t, const std::vector<std::string>& path, Value v) {
        for (size_t i = 0; i + 1 < path.size(); ++i) t = descend(t, path[i], true);
        if (t->get(path.back())) fail("duplicate key '" + path.back() + "'");
        t->table.emplace_back(path.back(), std::move(v));
    }

    Value* open_header(Value* root, const std::vector<std::string>& path, bool aot) {
        Value* t = root;
        for (size_t i = 0; i + 1 < path.size(); ++i) t = descend(t, path[i], true);
        const std::string& k = path.back();
        Value* x = t->get_mut(k);
        if (aot) {
            if (!x) {
                Value arr;
                arr.kind = Value::Kind::Array;
                arr.array_of_tables = true;
                t->table.emplace_back(k, std::move(arr));
                x = &t->table.back().second;
            } else if (!(x->kind == Value::Kind::Array && x->array_of_tables)) {
                fail("key '" + k + "' is not an array of tables");
            }
            Value nt;
            nt.kind = Value::Kind::Table;
            nt.defined = true;
            x->array.push_back(std::move(nt));
            return &x->array.back();
        }
        if (!x) {
            Value nt;
            nt.kind = Value::Kind::Table;
            nt.defined = true;
            t->table.emplace_back(k, std::move(nt));
            return &t->table.back().second;
        }
        if (x->kind != Value::Kind::Table) fail("key '" + k + "' is not a table");
        if (x->defined) fail("table '" + k + "' defined twice");
        x->defined = true;
        return x;
    }
};

}  // namespace

bool parse(const std::string& text, Value* root, std::string* err) {
    Parser ps(text);
    try {
        *root = Value();
        ps.run(root);
    } catch (const ParseError& e) {
        if (err) *err = "line " + std::to_string(ps.line()) + ": " + e.what();
        return false;
    }
    return true;
}

}  // namespace rt::toml
