// yaml.hpp — the YAML subset rray scene files use, typed like yaml-rust2 0.8 (Yaml::from_str).
//
// Block mappings / sequences (incl. "- key: v" items and sequences at their parent key's indent),
// flow sequences / mappings, plain / single / double quoted scalars, comments, "---" documents,
// and LF, CRLF or bare-CR line endings (examples/area_light.yaml uses bare CR).
#pragma once
#include <cstdint>
#include <memory>
#include <string>
#include <utility>
#include <vector>

namespace rr {
namespace yaml {

struct Node {
    enum Kind { BadValue, Null, Bool, Integer, Real, String, Array, Hash } kind = BadValue;
    bool b = false;
    int64_t i = 0;
    std::string s;  // Real: original text; String: value
    std::vector<Node> seq;
    std::vector<std::pair<std::string, Node>> map;

    // Yaml's Index<&str>: missing key / not a hash -> BadValue
    const Node& operator[](const std::string& key) const;
    const Node& operator[](size_t idx) const;
    bool is_bad() const { return kind == BadValue; }
    bool is_array() const { return kind == Array; }
};

// Parses the first document of `text`.  Returns false and sets `err` on a syntax error.
bool load_first(const std::string& text, Node& out, std::string& err);

// yaml-rust2 scalar resolution of a plain (unquoted) scalar
Node plain_scalar(const std::string& v);
// Rust's `str::parse::<f64>` grammar check + value (correctly rounded, same as strtod)
bool rust_parse_f64(const std::string& v, double& out);

}  // namespace yaml
}  // namespace rr
