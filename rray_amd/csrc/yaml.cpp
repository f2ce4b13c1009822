// yaml.cpp — YAML subset parser for rray scenes (see yaml.hpp).
#include "yaml.hpp"

#include <cctype>
#include <cerrno>
#include <cstdlib>
#include <cstring>

namespace rr {
namespace yaml {

namespace {
const Node kBad;

struct Line {
    int indent;
    std::string text;  // comment-stripped, right-trimmed
    int lineno;
};

std::string rtrim(const std::string& s) {
    size_t e = s.size();
    while (e > 0 && (s[e - 1] == ' ' || s[e - 1] == '\t')) --e;
    return s.substr(0, e);
}
std::string trim(const std::string& s) {
    size_t b = 0;
    while (b < s.size() && (s[b] == ' ' || s[b] == '\t')) ++b;
    return rtrim(s.substr(b));
}

// remove a comment: '#' at the start or after whitespace, outside quotes
std::string strip_comment(const std::string& s) {
    char q = 0;
    for (size_t i = 0; i < s.size(); ++i) {
        char ch = s[i];
        if (q) {
            if (ch == q) {
                if (q == '\'' && i + 1 < s.size() && s[i + 1] == '\'') {
                    ++i;
                    continue;
                }
                q = 0;
            } else if (q == '"' && ch == '\\') {
                ++i;
            }
            continue;
        }
        if (ch == '\'' || ch == '"') {
            // quotes only open a scalar at a token start
            if (i == 0 || s[i - 1] == ' ' || s[i - 1] == '[' || s[i - 1] == ',' || s[i - 1] == '{' ||
                s[i - 1] == ':' || s[i - 1] == '-')
                q = ch;
            continue;
        }
        if (ch == '#' && (i == 0 || s[i - 1] == ' ' || s[i - 1] == '\t')) return s.substr(0, i);
    }
    return s;
}

// position of the mapping ':' (followed by space/end), outside quotes and flow brackets; -1 if none
int map_colon(const std::string& s) {
    char q = 0;
    int depth = 0;
    if (!s.empty() && (s[0] == '[' || s[0] == '{')) return -1;
    for (size_t i = 0; i < s.size(); ++i) {
        char ch = s[i];
        if (q) {
            if (ch == q) q = 0;
            continue;
        }
        if ((ch == '\'' || ch == '"') && (i == 0 || s[i - 1] == ' ')) {
            q = ch;
            continue;
        }
        if (ch == '[' || ch == '{') ++depth;
        if (ch == ']' || ch == '}') --depth;
        if (ch == ':' && depth == 0 && (i + 1 == s.size() || s[i + 1] == ' ')) return (int)i;
    }
    return -1;
}

bool is_seq_item(const std::string& t) { return !t.empty() && t[0] == '-' && (t.size() == 1 || t[1] == ' '); }

Node make_string(const std::string& v) {
    Node n;
    n.kind = Node::String;
    n.s = v;
    return n;
}

bool unquote(const std::string& t, std::string& out, std::string& err) {
    char q = t[0];
    out.clear();
    size_t i = 1;
    for (; i < t.size(); ++i) {
        char ch = t[i];
        if (ch == q) {
            if (q == '\'' && i + 1 < t.size() && t[i + 1] == '\'') {
                out += '\'';
                ++i;
                continue;
            }
            break;
        }
        if (q == '"' && ch == '\\' && i + 1 < t.size()) {
            char e = t[++i];
            switch (e) {
                case 'n': out += '\n'; break;
                case 't': out += '\t'; break;
                case 'r': out += '\r'; break;
                case '0': out += '\0'; break;
                default: out += e; break;
            }
            continue;
        }
        out += ch;
    }
    if (i >= t.size()) {
        err = "unterminated quoted scalar";
        return false;
    }
    if (!trim(t.substr(i + 1)).empty()) {
        err = "trailing characters after quoted scalar";
        return false;
    }
    return true;
}

struct Parser {
    std::vector<Line> lines;
    size_t cur = 0;
    std::string err;

    bool fail(const std::string& m) {
        if (err.empty())
            err = m + (cur < lines.size() ? " (line " + std::to_string(lines[cur].lineno) + ")" : std::string());
        return false;
    }

    // ---- flow collections / inline scalars
    bool parse_flow(const std::string& s, size_t& p, Node& out) {
        while (p < s.size() && s[p] == ' ') ++p;
        if (p >= s.size()) return fail("unexpected end of flow collection");
        char ch = s[p];
        if (ch == '[') {
            out = Node();
            out.kind = Node::Array;
            ++p;
            for (;;) {
                while (p < s.size() && s[p] == ' ') ++p;
                if (p < s.size() && s[p] == ']') {
                    ++p;
                    return true;
                }
                Node item;
                if (!parse_flow(s, p, item)) return false;
                out.seq.push_back(item);
                while (p < s.size() && s[p] == ' ') ++p;
                if (p < s.size() && s[p] == ',') {
                    ++p;
                    continue;
                }
                if (p < s.size() && s[p] == ']') {
                    ++p;
                    return true;
                }
                return fail("expected ',' or ']' in flow sequence");
            }
        }
        if (ch == '{') {
            out = Node();
            out.kind = Node::Hash;
            ++p;
            for (;;) {
                while (p < s.size() && s[p] == ' ') ++p;
                if (p < s.size() && s[p] == '}') {
                    ++p;
                    return true;
                }
                Node key;
                if (!parse_flow_scalar(s, p, key, true)) return false;
                while (p < s.size() && s[p] == ' ') ++p;
                Node val;
                val.kind = Node::Null;
                if (p < s.size() && s[p] == ':') {
                    ++p;
                    if (!parse_flow(s, p, val)) return false;
                }
                out.map.emplace_back(key.kind == Node::String || key.kind == Node::Real ? key.s : key_text(key), val);
                while (p < s.size() && s[p] == ' ') ++p;
                if (p < s.size() && s[p] == ',') {
                    ++p;
                    continue;
                }
                if (p < s.size() && s[p] == '}') {
                    ++p;
                    return true;
                }
                return fail("expected ',' or '}' in flow mapping");
            }
        }
        return parse_flow_scalar(s, p, out, false);
    }
    static std::string key_text(const Node& k) {
        switch (k.kind) {
            case Node::Integer: return std::to_string(k.i);
            case Node::Bool: return k.b ? "true" : "false";
            case Node::Null: return "null";
            default: return k.s;
        }
    }
    bool parse_flow_scalar(const std::string& s, size_t& p, Node& out, bool is_key) {
        while (p < s.size() && s[p] == ' ') ++p;
        if (p < s.size() && (s[p] == '\'' || s[p] == '"')) {
            char q = s[p];
            size_t e = p + 1;
            for (; e < s.size(); ++e) {
                if (s[e] == q) {
                    if (q == '\'' && e + 1 < s.size() && s[e + 1] == '\'') {
                        ++e;
                        continue;
                    }
                    break;
                }
                if (q == '"' && s[e] == '\\') ++e;
            }
            if (e >= s.size()) return fail("unterminated quoted scalar");
            std::string v;
            if (!unquote(s.substr(p, e - p + 1), v, err)) return fail(err);
            out = make_string(v);
            p = e + 1;
            return true;
        }
        size_t e = p;
        while (e < s.size() && s[e] != ',' && s[e] != ']' && s[e] != '}' && !(is_key && s[e] == ':')) ++e;
        out = plain_scalar(trim(s.substr(p, e - p)));
        p = e;
        return true;
    }
    bool parse_inline(std::string t, Node& out) {
        t = trim(t);
        if (t.empty()) {
            out = Node();
            out.kind = Node::Null;
            return true;
        }
        if (t[0] == '[' || t[0] == '{') {
            // flow collections may continue on following lines
            auto balance = [](const std::string& x) {
                int d = 0;
                char q = 0;
                for (char ch : x) {
                    if (q) {
                        if (ch == q) q = 0;
                        continue;
                    }
                    if (ch == '\'' || ch == '"') q = ch;
                    if (ch == '[' || ch == '{') ++d;
                    if (ch == ']' || ch == '}') --d;
                }
                return d;
            };
            while (balance(t) > 0 && cur < lines.size()) t += " " + trim(lines[cur++].text);
            size_t p = 0;
            if (!parse_flow(t, p, out)) return false;
            if (!trim(t.substr(p)).empty()) return fail("trailing characters after flow collection");
            return true;
        }
        if (t[0] == '\'' || t[0] == '"') {
            std::string v;
            if (!unquote(t, v, err)) return fail(err);
            out = make_string(v);
            return true;
        }
        if (t[0] == '&' || t[0] == '*' || t[0] == '!' || t[0] == '|' || t[0] == '>')
            return fail("unsupported YAML feature (anchor/alias/tag/block scalar)");
        out = plain_scalar(t);
        return true;
    }

    // ---- block structure
    bool parse_node(int ind, Node& out) {
        if (cur >= lines.size()) {
            out = Node();
            out.kind = Node::Null;
            return true;
        }
        const Line& L = lines[cur];
        if (is_seq_item(L.text)) return parse_seq(L.indent, out);
        if (map_colon(L.text) >= 0) return parse_map(L.indent, out);
        ++cur;
        return parse_inline(L.text, out);
    }
    bool parse_seq(int ind, Node& out) {
        out = Node();
        out.kind = Node::Array;
        while (cur < lines.size() && lines[cur].indent == ind && is_seq_item(lines[cur].text)) {
            std::string rest = lines[cur].text.substr(1);
            size_t sp = 0;
            while (sp < rest.size() && rest[sp] == ' ') ++sp;
            rest = rest.substr(sp);
            Node item;
            if (rest.empty()) {
                ++cur;
                if (cur < lines.size() && lines[cur].indent > ind) {
                    if (!parse_node(lines[cur].indent, item)) return false;
                } else {
                    item.kind = Node::Null;
                }
            } else {
                // "- x": re-read the remainder as a node at its own column
                lines[cur].indent = ind + 1 + (int)sp;
                lines[cur].text = rest;
                if (!parse_node(lines[cur].indent, item)) return false;
            }
            out.seq.push_back(item);
        }
        if (cur < lines.size() && lines[cur].indent > ind) return fail("bad indentation in sequence");
        return true;
    }
    bool parse_map(int ind, Node& out) {
        out = Node();
        out.kind = Node::Hash;
        while (cur < lines.size() && lines[cur].indent == ind) {
            const std::string t = lines[cur].text;
            int c = map_colon(t);
            if (c < 0) return fail("expected 'key: value'");
            std::string k = trim(t.substr(0, c));
            if (!k.empty() && (k[0] == '\'' || k[0] == '"')) {
                std::string v;
                if (!unquote(k, v, err)) return fail(err);
                k = v;
            }
            std::string rest = t.substr(c + 1);
            ++cur;
            Node val;
            if (trim(rest).empty()) {
                if (cur < lines.size() && lines[cur].indent > ind) {
                    if (!parse_node(lines[cur].indent, val)) return false;
                } else if (cur < lines.size() && lines[cur].indent == ind && is_seq_item(lines[cur].text)) {
                    if (!parse_seq(ind, val)) return false;
                } else {
                    val.kind = Node::Null;
                }
            } else {
                if (!parse_inline(rest, val)) return false;
            }
            bool dup = false;
            for (auto& kv : out.map)
                if (kv.first == k) {
                    kv.second = val;  // later keys win (LinkedHashMap insert)
                    dup = true;
                }
            if (!dup) out.map.emplace_back(k, val);
        }
        if (cur < lines.size() && lines[cur].indent > ind) return fail("bad indentation in mapping");
        return true;
    }
};

}  // namespace

const Node& Node::operator[](const std::string& key) const {
    if (kind != Hash) return kBad;
    for (const auto& kv : map)
        if (kv.first == key) return kv.second;
    return kBad;
}
const Node& Node::operator[](size_t idx) const {
    if (kind != Array || idx >= seq.size()) return kBad;
    return seq[idx];
}

bool rust_parse_f64(const std::string& v, double& out) {
    // [+-]? (inf | infinity | nan | digits[.digits*][e[+-]digits] | .digits[e...]), case-insensitive words
    size_t p = 0;
    if (p < v.size() && (v[p] == '+' || v[p] == '-')) ++p;
    std::string rest = v.substr(p);
    std::string low;
    for (char ch : rest) low += (char)std::tolower((unsigned char)ch);
    if (low == "inf" || low == "infinity" || low == "nan") {
        out = std::strtod(v.c_str(), nullptr);
        return true;
    }
    size_t i = 0, digits = 0;
    while (i < rest.size() && std::isdigit((unsigned char)rest[i])) ++i, ++digits;
    if (i < rest.size() && rest[i] == '.') {
        ++i;
        while (i < rest.size() && std::isdigit((unsigned char)rest[i])) ++i, ++digits;
    }
    if (digits == 0) return false;
    if (i < rest.size() && (rest[i] == 'e' || rest[i] == 'E')) {
        ++i;
        if (i < rest.size() && (rest[i] == '+' || rest[i] == '-')) ++i;
        size_t ed = 0;
        while (i < rest.size() && std::isdigit((unsigned char)rest[i])) ++i, ++ed;
        if (ed == 0) return false;
    }
    if (i != rest.size()) return false;
    out = std::strtod(v.c_str(), nullptr);  // correctly rounded, as Rust's dec2flt
    return true;
}

Node plain_scalar(const std::string& v) {
    Node n;
    auto try_radix = [&](const std::string& digits, int base) {
        if (digits.empty()) return false;
        char* e = nullptr;
        errno = 0;
        long long x = std::strtoll(digits.c_str(), &e, base);
        if (errno || *e || digits[0] == '-' || digits[0] == '+') return false;
        n.kind = Node::Integer;
        n.i = x;
        return true;
    };
    if (v.rfind("0x", 0) == 0 && try_radix(v.substr(2), 16)) return n;
    if (v.rfind("0o", 0) == 0 && try_radix(v.substr(2), 8)) return n;
    if (v == "~" || v == "null") {
        n.kind = Node::Null;
        return n;
    }
    if (v == "true" || v == "false") {
        n.kind = Node::Bool;
        n.b = v == "true";
        return n;
    }
    // i64::from_str: [+-]?digits
    {
        size_t p = (!v.empty() && (v[0] == '+' || v[0] == '-')) ? 1 : 0;
        bool all = p < v.size();
        for (size_t i = p; i < v.size(); ++i)
            if (!std::isdigit((unsigned char)v[i])) all = false;
        if (all) {
            errno = 0;
            long long x = std::strtoll(v.c_str(), nullptr, 10);
            if (!errno) {
                n.kind = Node::Integer;
                n.i = x;
                return n;
            }
        }
    }
    static const char* specials[] = {".inf", ".Inf", ".INF", "+.inf", "+.Inf", "+.INF", "-.inf", "-.Inf",
                                     "-.INF", ".nan", ".NaN", ".NAN"};
    for (const char* sp : specials)
        if (v == sp) {  // Yaml::Real whose later str::parse::<f64> fails (reference panics)
            n.kind = Node::Real;
            n.s = v;
            return n;
        }
    double d;
    if (rust_parse_f64(v, d)) {
        n.kind = Node::Real;
        n.s = v;
        return n;
    }
    return make_string(v);
}

bool load_first(const std::string& text_in, Node& out, std::string& err) {
    std::string text;
    text.reserve(text_in.size());
    for (size_t i = 0; i < text_in.size(); ++i) {
        char ch = text_in[i];
        if (ch == '\r') {
            text += '\n';
            if (i + 1 < text_in.size() && text_in[i + 1] == '\n') ++i;
        } else {
            text += ch;
        }
    }
    Parser P;
    size_t pos = 0;
    int lineno = 0;
    bool started = false;
    while (pos <= text.size()) {
        size_t e = text.find('\n', pos);
        if (e == std::string::npos) e = text.size();
        std::string raw = text.substr(pos, e - pos);
        pos = e + 1;
        ++lineno;
        if (raw.rfind("---", 0) == 0 && (raw.size() == 3 || raw[3] == ' ')) {
            if (started) break;  // second document: stop
            std::string rest = trim(raw.substr(3));
            started = true;
            if (rest.empty()) continue;
            raw = rest;
        }
        if (raw == "..." && started) break;
        std::string t = rtrim(strip_comment(raw));
        int ind = 0;
        while (ind < (int)t.size() && t[ind] == ' ') ++ind;
        if (ind < (int)t.size() && t[ind] == '\t') {
            err = "tab indentation (line " + std::to_string(lineno) + ")";
            return false;
        }
        if (ind == (int)t.size()) continue;
        if (!started && t[0] != '%') started = true;
        if (t[0] == '%') continue;  // directives
        P.lines.push_back({ind, t.substr(ind), lineno});
    }
    if (P.lines.empty()) {
        out = Node();
        out.kind = Node::Null;
        return true;
    }
    if (!P.parse_node(P.lines[0].indent, out)) {
        err = P.err;
        return false;
    }
    if (P.cur < P.lines.size()) {
        err = "unexpected content (line " + std::to_string(P.lines[P.cur].lineno) + ")";
        return false;
    }
    return true;
}

}  // namespace yaml
}  // namespace rr
