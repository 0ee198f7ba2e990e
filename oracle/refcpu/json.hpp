// ORACLE / TEST INFRASTRUCTURE — not product code.
// Minimal JSON value model used by the CPU restatement ("refcpu") of KWOK's Stage
// lifecycle hot path.  It mirrors what `expression.ToJSONStandard`
// (reference: pkg/utils/expression/query.go:72-88) produces in Go: json.Unmarshal into
// interface{}, i.e. nil / bool / float64 / string / []interface{} / map[string]interface{}.
// Numbers are therefore always float64 (pinned by value_int_from_test.go:58-66, where a
// JSON integer reaches the `case float64` branch of int64From.Get).
#pragma once
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace refcpu {

struct JV;
using JVP = std::shared_ptr<const JV>;

struct JV {
  enum Type { NUL, BOOL, NUM, STR, ARR, OBJ } t = NUL;
  bool b = false;
  double n = 0;
  bool gint = false;  // gojq int (value in i)
  long long i = 0;
  std::string s;
  std::vector<JVP> a;
  std::vector<std::pair<std::string, JVP>> o;  // insertion order kept; lookups linear

  static JVP null() { static JVP v = std::make_shared<JV>(); return v; }
  static JVP boolean(bool x) { auto v = std::make_shared<JV>(); v->t = BOOL; v->b = x; return v; }
  static JVP number(double x) { auto v = std::make_shared<JV>(); v->t = NUM; v->n = x; return v; }
  // a gojq int (number literals, length, int arithmetic); JSON input numbers are float64
  static JVP integer(long long x) {
    auto v = std::make_shared<JV>(); v->t = NUM; v->n = (double)x; v->gint = true; v->i = x; return v;
  }
  static JVP str(std::string x) { auto v = std::make_shared<JV>(); v->t = STR; v->s = std::move(x); return v; }

  const JVP* get(const std::string& k) const {
    for (auto& kv : o) if (kv.first == k) return &kv.second;
    return nullptr;
  }
};

struct JsonError : std::runtime_error { using std::runtime_error::runtime_error; };

class JsonParser {
 public:
  explicit JsonParser(const char* p, size_t n) : p_(p), e_(p + n) {}
  JVP parse() {
    JVP v = value();
    ws();
    if (p_ != e_) throw JsonError("trailing characters");
    return v;
  }

 private:
  const char* p_;
  const char* e_;
  void ws() { while (p_ < e_ && (*p_ == ' ' || *p_ == '\t' || *p_ == '\n' || *p_ == '\r')) ++p_; }
  bool lit(const char* s) {
    size_t n = strlen(s);
    if ((size_t)(e_ - p_) >= n && memcmp(p_, s, n) == 0) { p_ += n; return true; }
    return false;
  }
  static void utf8(std::string& out, uint32_t cp) {
    if (cp < 0x80) out += (char)cp;
    else if (cp < 0x800) { out += (char)(0xC0 | (cp >> 6)); out += (char)(0x80 | (cp & 0x3F)); }
    else if (cp < 0x10000) { out += (char)(0xE0 | (cp >> 12)); out += (char)(0x80 | ((cp >> 6) & 0x3F)); out += (char)(0x80 | (cp & 0x3F)); }
    else { out += (char)(0xF0 | (cp >> 18)); out += (char)(0x80 | ((cp >> 12) & 0x3F)); out += (char)(0x80 | ((cp >> 6) & 0x3F)); out += (char)(0x80 | (cp & 0x3F)); }
  }
  uint32_t hex4() {
    if (e_ - p_ < 4) throw JsonError("bad \\u escape");
    uint32_t v = 0;
    for (int i = 0; i < 4; ++i) {
      char c = *p_++;
      v <<= 4;
      if (c >= '0' && c <= '9') v |= c - '0';
      else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
      else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
      else throw JsonError("bad hex digit");
    }
    return v;
  }
  std::string string() {
    if (p_ >= e_ || *p_ != '"') throw JsonError("expected string");
    ++p_;
    std::string out;
    while (true) {
      if (p_ >= e_) throw JsonError("unterminated string");
      char c = *p_++;
      if (c == '"') break;
      if (c != '\\') { out += c; continue; }
      if (p_ >= e_) throw JsonError("bad escape");
      char x = *p_++;
      switch (x) {
        case '"': out += '"'; break;
        case '\\': out += '\\'; break;
        case '/': out += '/'; break;
        case 'b': out += '\b'; break;
        case 'f': out += '\f'; break;
        case 'n': out += '\n'; break;
        case 'r': out += '\r'; break;
        case 't': out += '\t'; break;
        case 'u': {
          uint32_t cp = hex4();
          if (cp >= 0xD800 && cp < 0xDC00 && e_ - p_ >= 6 && p_[0] == '\\' && p_[1] == 'u') {
            p_ += 2;
            uint32_t lo = hex4();
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          }
          utf8(out, cp);
          break;
        }
        default: throw JsonError("bad escape");
      }
    }
    return out;
  }
  JVP value() {
    ws();
    if (p_ >= e_) throw JsonError("unexpected end");
    char c = *p_;
    if (c == '{') {
      ++p_;
      auto v = std::make_shared<JV>();
      v->t = JV::OBJ;
      ws();
      if (p_ < e_ && *p_ == '}') { ++p_; return v; }
      while (true) {
        ws();
        std::string k = string();
        ws();
        if (p_ >= e_ || *p_ != ':') throw JsonError("expected ':'");
        ++p_;
        JVP x = value();
        bool replaced = false;  // Go's json.Unmarshal keeps the last duplicate key
        for (auto& kv : v->o) if (kv.first == k) { kv.second = x; replaced = true; }
        if (!replaced) v->o.emplace_back(std::move(k), x);
        ws();
        if (p_ < e_ && *p_ == ',') { ++p_; continue; }
        if (p_ < e_ && *p_ == '}') { ++p_; return v; }
        throw JsonError("expected ',' or '}'");
      }
    }
    if (c == '[') {
      ++p_;
      auto v = std::make_shared<JV>();
      v->t = JV::ARR;
      ws();
      if (p_ < e_ && *p_ == ']') { ++p_; return v; }
      while (true) {
        v->a.push_back(value());
        ws();
        if (p_ < e_ && *p_ == ',') { ++p_; continue; }
        if (p_ < e_ && *p_ == ']') { ++p_; return v; }
        throw JsonError("expected ',' or ']'");
      }
    }
    if (c == '"') return JV::str(string());
    if (lit("true")) return JV::boolean(true);
    if (lit("false")) return JV::boolean(false);
    if (lit("null")) return JV::null();
    const char* s = p_;
    if (p_ < e_ && (*p_ == '-' || *p_ == '+')) ++p_;
    while (p_ < e_ && ((*p_ >= '0' && *p_ <= '9') || *p_ == '.' || *p_ == 'e' || *p_ == 'E' || *p_ == '-' || *p_ == '+')) ++p_;
    if (p_ == s) throw JsonError("unexpected character");
    std::string num(s, p_);
    char* end = nullptr;
    double d = strtod(num.c_str(), &end);
    if (!end || *end) throw JsonError("bad number");
    return JV::number(d);
  }
};

inline JVP parse_json(const std::string& s) { return JsonParser(s.data(), s.size()).parse(); }

inline void dump_string(std::string& out, const std::string& s) {
  out += '"';
  for (unsigned char c : s) {
    switch (c) {
      case '"': out += "\\\""; break;
      case '\\': out += "\\\\"; break;
      case '\n': out += "\\n"; break;
      case '\r': out += "\\r"; break;
      case '\t': out += "\\t"; break;
      default:
        if (c < 0x20) { char b[8]; snprintf(b, sizeof b, "\\u%04x", c); out += b; }
        else out += (char)c;
    }
  }
  out += '"';
}

inline void dump(std::string& out, const JVP& v) {
  switch (v->t) {
    case JV::NUL: out += "null"; break;
    case JV::BOOL: out += v->b ? "true" : "false"; break;
    case JV::NUM: {
      char b[40];
      if (v->gint) snprintf(b, sizeof b, "%lld", v->i);
      else if (std::floor(v->n) == v->n && std::fabs(v->n) < 1e17) snprintf(b, sizeof b, "%.0f", v->n);
      else snprintf(b, sizeof b, "%.17g", v->n);
      out += b;
      break;
    }
    case JV::STR: dump_string(out, v->s); break;
    case JV::ARR: {
      out += '[';
      for (size_t i = 0; i < v->a.size(); ++i) { if (i) out += ','; dump(out, v->a[i]); }
      out += ']';
      break;
    }
    case JV::OBJ: {
      out += '{';
      for (size_t i = 0; i < v->o.size(); ++i) {
        if (i) out += ',';
        dump_string(out, v->o[i].first);
        out += ':';
        dump(out, v->o[i].second);
      }
      out += '}';
      break;
    }
  }
}

inline std::string dumps(const JVP& v) { std::string s; dump(s, v); return s; }

// jq/gojq structural equality (numbers compare numerically, objects as key sets)
inline bool jv_equal(const JVP& x, const JVP& y) {
  if (x->t != y->t) return false;
  switch (x->t) {
    case JV::NUL: return true;
    case JV::BOOL: return x->b == y->b;
    case JV::NUM: return x->n == y->n;
    case JV::STR: return x->s == y->s;
    case JV::ARR:
      if (x->a.size() != y->a.size()) return false;
      for (size_t i = 0; i < x->a.size(); ++i) if (!jv_equal(x->a[i], y->a[i])) return false;
      return true;
    case JV::OBJ:
      if (x->o.size() != y->o.size()) return false;
      for (auto& kv : x->o) {
        auto* o = y->get(kv.first);
        if (!o || !jv_equal(kv.second, *o)) return false;
      }
      return true;
  }
  return false;
}

inline bool jv_truthy(const JVP& v) { return !(v->t == JV::NUL || (v->t == JV::BOOL && !v->b)); }

}  // namespace refcpu
