// Minimal TOML reader for the reference's scene schema (scenes/*.toml, SceneSpec scene.rs:292-348).
// Supports: comments, [table], [[array.of.tables]], dotted/bare/quoted keys, strings (basic and
// literal), integers, floats (exponent, underscores, inf/nan), booleans, multi-line arrays with
// trailing commas, inline tables. Dates and multi-line strings are not needed by the schema and
// are rejected with a parse error.
#pragma once

#include <cstdint>
#include <memory>
#include <string>
#include <utility>
#include <vector>

namespace rt::toml {

struct Value {
    enum class Kind { Table, Array, String, Int, Float, Bool };
    Kind kind = Kind::Table;
    std::vector<std::pair<std::string, Value>> table;  // insertion order kept
    std::vector<Value> array;
    std::string str;
    int64_t i = 0;
    double f = 0.0;
    bool b = false;
    bool array_of_tables = false;  // created by [[...]]
    bool defined = false;          // table explicitly defined by a [header]

    const Value* get(const std::string& key) const;
    Value* get_mut(const std::string& key);
    bool is_number() const { return kind == Kind::Int || kind == Kind::Float; }
    double as_f64() const { return kind == Kind::Int ? (double)i : f; }
};

// Parses `text`; on failure returns false and fills `err` with "line N: message".
bool parse(const std::string& text, Value* root, std::string* err);

const char* kind_name(Value::Kind k);

}  // namespace rt::toml
