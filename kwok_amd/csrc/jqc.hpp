// The jq language subset of Stage selector keys and *From getters, evaluated on the host by the
// native encoder and compiler (libkwok_encoder / libkwok_compiler).
//
// Reference: the Stage CRD's matchExpressions[].key, weightFrom, durationFrom and
// jitterDurationFrom are gojq queries (github.com/itchyny/gojq v0.12.16, go.mod:17),
// compiled by expression.NewQuery and run by Query.Execute (pkg/utils/expression/query.go:33-69)
// on ToJSONStandard(obj) (query.go:72-88).  Restated here:
//   * values as gojq holds them: null, bool, float64 (every JSON number of the input), int (number
//     literals, `length`, int arithmetic; JV::gint), string, array, object (keys sorted, last
//     duplicate wins, as json.Unmarshal into a map);
//   * paths `.`, `.a`, `."a"`, `.[e]`, `.a.[]`, `.[]`, postfix `?`; `|`, `,`, `//`, `and`, `or`,
//     comparisons (gojq's total order), `+ - * / %`, unary `-`, literals, `[...]`, `{...}`,
//     `if-then-elif-else-end`, `try e`, assignment `=`, `|=`, `+=`, `-=`, `*=`, `/=`, `%=`, `//=`;
//   * builtins: empty, error, not, length, keys, keys_unsorted, has(k), type, tostring, tonumber,
//     ascii_downcase, ascii_upcase, startswith(s), endswith(s), ltrimstr(s), rtrimstr(s),
//     contains(x), select(f), map(f), add, any, all, first, last, first(f), values;
//   * Query.Execute: a runtime error makes the whole result nil; null outputs are dropped.
// Anything else (variables, reduce / foreach, def, string interpolation, formats, regexes, `..`)
// is refused at compile time with the construct named (Unsupported); a Go host keeps the
// reference lifecycle for such a resourceRef.
#pragma once
#include <algorithm>
#include <cerrno>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "json_dom.hpp"

namespace kwkjq {

using kwkjson::JV;

struct Error : std::runtime_error {        // a runtime error (Execute -> nil)
  using std::runtime_error::runtime_error;
};
struct Unsupported : std::runtime_error {  // a query outside the subset, or a syntax error
  using std::runtime_error::runtime_error;
};

// ------------------------------------------------------------------ values
// A value is a pointer into the input document (borrowed) or into a value computed by the query
// (held).  null is a static JV.
struct Val {
  const JV* p;
  std::shared_ptr<const JV> hold;
};

inline const JV& null_jv() {
  static const JV n;
  return n;
}
inline Val vnull() { return Val{&null_jv(), nullptr}; }
inline Val own(JV&& v) {
  auto h = std::make_shared<const JV>(std::move(v));
  return Val{h.get(), h};
}
inline Val vbool(bool b) {
  JV v;
  v.t = JV::BOOL;
  v.b = b;
  return own(std::move(v));
}
inline Val vstr(std::string s) {
  JV v;
  v.t = JV::STR;
  v.s = std::move(s);
  return own(std::move(v));
}
inline JV jint(int64_t n) {
  JV v;
  v.t = JV::NUM;
  v.gint = true;
  v.is_int = true;
  v.s = std::to_string(n);
  return v;
}
inline JV jfloat(double d) {
  JV v;
  v.t = JV::NUM;
  char buf[40];
  snprintf(buf, sizeof buf, "%.17g", d);
  v.s = buf;
  return v;
}
inline Val vint(int64_t n) { return own(jint(n)); }
inline Val vfloat(double d) { return own(jfloat(d)); }

inline bool is_gint(const JV& v) { return v.t == JV::NUM && v.gint; }
inline double num(const JV& v) { return strtod(v.s.c_str(), nullptr); }
inline int64_t inum(const JV& v) { return strtoll(v.s.c_str(), nullptr, 10); }
inline bool truthy(const JV& v) { return !(v.t == JV::NUL || (v.t == JV::BOOL && !v.b)); }

inline const char* type_name(const JV& v) {
  switch (v.t) {
    case JV::NUL: return "null";
    case JV::BOOL: return "boolean";
    case JV::NUM: return "number";
    case JV::STR: return "string";
    case JV::ARR: return "array";
    case JV::OBJ: return "object";
  }
  return "?";
}

// an object's entries as gojq's map holds them: unique keys (the last duplicate wins), sorted
// bytewise (gojq iterates, lists and encodes object keys in sorted order)
inline std::vector<std::pair<const std::string*, const JV*>> entries(const JV& o) {
  std::vector<std::pair<const std::string*, const JV*>> e;
  e.reserve(o.k.size());
  for (size_t i = 0; i < o.k.size(); ++i) {
    bool later = false;
    for (size_t j = i + 1; j < o.k.size() && !later; ++j) later = o.k[j] == o.k[i];
    if (!later) e.emplace_back(&o.k[i], &o.a[i]);
  }
  std::sort(e.begin(), e.end(), [](const auto& x, const auto& y) { return *x.first < *y.first; });
  return e;
}

// gojq compare: null < false < true < numbers < strings < arrays < objects; numbers by value
// (int and float alike), strings bytewise, arrays element-wise then by length, objects by their
// sorted key lists, then by the values of those keys
inline int type_rank(const JV& v) {
  switch (v.t) {
    case JV::NUL: return 0;
    case JV::BOOL: return v.b ? 2 : 1;
    case JV::NUM: return 3;
    case JV::STR: return 4;
    case JV::ARR: return 5;
    case JV::OBJ: return 6;
  }
  return 7;
}
inline int compare(const JV& x, const JV& y) {
  const int rx = type_rank(x), ry = type_rank(y);
  if (rx != ry) return rx < ry ? -1 : 1;
  switch (x.t) {
    case JV::NUM: {
      if (is_gint(x) && is_gint(y)) {
        const int64_t a = inum(x), b = inum(y);
        return a < b ? -1 : a > b ? 1 : 0;
      }
      const double a = num(x), b = num(y);
      return a < b ? -1 : a > b ? 1 : 0;
    }
    case JV::STR: return x.s < y.s ? -1 : x.s > y.s ? 1 : 0;
    case JV::ARR: {
      for (size_t i = 0; i < x.a.size() && i < y.a.size(); ++i)
        if (int c = compare(x.a[i], y.a[i])) return c;
      return x.a.size() < y.a.size() ? -1 : x.a.size() > y.a.size() ? 1 : 0;
    }
    case JV::OBJ: {
      const auto ex = entries(x), ey = entries(y);
      for (size_t i = 0; i < ex.size() && i < ey.size(); ++i)
        if (*ex[i].first != *ey[i].first) return *ex[i].first < *ey[i].first ? -1 : 1;
      if (ex.size() != ey.size()) return ex.size() < ey.size() ? -1 : 1;
      for (size_t i = 0; i < ex.size(); ++i)
        if (int c = compare(*ex[i].second, *ey[i].second)) return c;
      return 0;
    }
    default: return 0;
  }
}

// gojq's encoder (tostring, kwk_jq_eval's output): sorted object keys, floats as strconv 'f' with
// the shortest round-trip digits ('e' below 1e-6 or from 1e21), ints as decimal
inline void enc_str(std::string& o, const std::string& s) {
  o += '"';
  for (unsigned char c : s) {
    switch (c) {
      case '"': o += "\\\""; break;
      case '\\': o += "\\\\"; break;
      case '\n': o += "\\n"; break;
      case '\r': o += "\\r"; break;
      case '\t': o += "\\t"; break;
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
inline std::string enc_float(double f) {
  if (f != f) return "null";
  if (f >= 1.7976931348623157e308) f = 1.7976931348623157e308;
  if (f <= -1.7976931348623157e308) f = -1.7976931348623157e308;
  char buf[64];
  int prec = 1;
  for (; prec <= 17; ++prec) {
    snprintf(buf, sizeof buf, "%.*e", prec - 1, f);
    if (strtod(buf, nullptr) == f) break;
  }
  const double x = std::fabs(f);
  if (x != 0 && (x < 1e-6 || x >= 1e21)) {  // 'e' format: mantissa digits, exponent without padding
    std::string m(buf);
    const size_t ep = m.find('e');
    std::string mant = m.substr(0, ep);
    int e10 = atoi(m.c_str() + ep + 1);
    if (mant.find('.') != std::string::npos) {
      while (mant.back() == '0') mant.pop_back();
      if (mant.back() == '.') mant.pop_back();
    }
    return mant + (e10 < 0 ? "e-" : "e+") + std::to_string(e10 < 0 ? -e10 : e10);
  }
  // 'f' format with the same significant digits
  std::string m(buf);
  const size_t ep = m.find('e');
  const int e10 = atoi(m.c_str() + ep + 1);
  std::string digits;
  bool neg = false;
  for (size_t i = 0; i < ep; ++i) {
    if (m[i] == '-') neg = true;
    else if (m[i] >= '0' && m[i] <= '9') digits += m[i];
  }
  while (digits.size() > 1 && digits.back() == '0') digits.pop_back();
  std::string out = neg ? "-" : "";
  if (e10 < 0) {
    out += "0." + std::string((size_t)(-e10 - 1), '0') + digits;
  } else if ((int)digits.size() <= e10 + 1) {
    out += digits + std::string((size_t)(e10 + 1 - (int)digits.size()), '0');
  } else {
    out += digits.substr(0, (size_t)e10 + 1) + "." + digits.substr((size_t)e10 + 1);
  }
  if (out == "-0") out = "-0";
  return out;
}
inline void encode(std::string& o, const JV& v) {
  switch (v.t) {
    case JV::NUL: o += "null"; return;
    case JV::BOOL: o += v.b ? "true" : "false"; return;
    case JV::NUM: o += is_gint(v) ? v.s : enc_float(num(v)); return;
    case JV::STR: enc_str(o, v.s); return;
    case JV::ARR:
      o += '[';
      for (size_t i = 0; i < v.a.size(); ++i) {
        if (i) o += ',';
        encode(o, v.a[i]);
      }
      o += ']';
      return;
    case JV::OBJ: {
      o += '{';
      bool first = true;
      for (const auto& kv : entries(v)) {
        if (!first) o += ',';
        first = false;
        enc_str(o, *kv.first);
        o += ':';
        encode(o, *kv.second);
      }
      o += '}';
      return;
    }
  }
}

// ------------------------------------------------------------------ syntax tree
struct Node {
  enum K {
    IDENT, FIELD, INDEX, ITER, TRY, PIPE, COMMA, ALT, OR, AND, CMP, ARITH, NEG, LIT, ARRAY, OBJECT,
    IF, FUNC, ASSIGN
  } k;
  std::string name;                    // FIELD key, CMP / ARITH / ASSIGN operator, FUNC name
  JV lit;                              // LIT
  std::shared_ptr<Node> a, b;          // operands (a: the sub-expression / left side)
  std::vector<std::shared_ptr<Node>> args;  // FUNC arguments; IF: cond, then, cond, then, ..., [else]
  std::vector<std::pair<std::shared_ptr<Node>, std::shared_ptr<Node>>> obj;  // OBJECT entries
};
using NodeP = std::shared_ptr<Node>;

class Parser {
 public:
  explicit Parser(const std::string& src) : s_(src) {}
  NodeP parse() {
    NodeP n = pipe();
    ws();
    if (i_ != s_.size()) bad("unexpected '" + s_.substr(i_, 8) + "'");
    return n;
  }

 private:
  const std::string& s_;
  size_t i_ = 0;

  [[noreturn]] void bad(const std::string& what) const {
    throw Unsupported("jq construct not supported natively: " + what + " in '" + s_ + "'");
  }
  static NodeP mk(Node::K k) {
    auto n = std::make_shared<Node>();
    n->k = k;
    return n;
  }
  static NodeP mk2(Node::K k, NodeP a, NodeP b, std::string name = "") {
    auto n = mk(k);
    n->a = std::move(a);
    n->b = std::move(b);
    n->name = std::move(name);
    return n;
  }
  static bool idc(char c) { return isalnum((unsigned char)c) || c == '_'; }
  void ws() {
    for (;;) {
      while (i_ < s_.size() && isspace((unsigned char)s_[i_])) ++i_;
      if (i_ < s_.size() && s_[i_] == '#') {  // comment to the end of the line
        while (i_ < s_.size() && s_[i_] != '\n') ++i_;
        continue;
      }
      return;
    }
  }
  bool at(const char* t) {
    ws();
    return s_.compare(i_, strlen(t), t) == 0;
  }
  bool eat(const char* t) {
    if (!at(t)) return false;
    i_ += strlen(t);
    return true;
  }
  // an operator token that is not the prefix of a longer one (`=` but not `==`, `|` but not `|=`)
  bool eat_op(const char* t, std::initializer_list<const char*> longer) {
    if (!at(t)) return false;
    for (const char* l : longer)
      if (s_.compare(i_, strlen(l), l) == 0) return false;
    i_ += strlen(t);
    return true;
  }
  bool at_kw(const char* t) {
    ws();
    const size_t n = strlen(t);
    return s_.compare(i_, n, t) == 0 && !(i_ + n < s_.size() && idc(s_[i_ + n]));
  }
  bool eat_kw(const char* t) {
    if (!at_kw(t)) return false;
    i_ += strlen(t);
    return true;
  }
  void expect(const char* t) {
    if (!eat(t)) bad(std::string("syntax (expected '") + t + "')");
  }
  std::string ident() {
    ws();
    const size_t b = i_;
    if (i_ < s_.size() && (isalpha((unsigned char)s_[i_]) || s_[i_] == '_')) {
      ++i_;
      while (i_ < s_.size() && idc(s_[i_])) ++i_;
    }
    return s_.substr(b, i_ - b);
  }
  std::string string_lit() {
    ws();
    if (i_ >= s_.size() || s_[i_] != '"') bad("syntax (expected a string)");
    const size_t b = i_++;
    while (i_ < s_.size() && s_[i_] != '"') {
      if (s_[i_] == '\\') {
        if (i_ + 1 < s_.size() && s_[i_ + 1] == '(') bad("string interpolation");
        ++i_;
      }
      ++i_;
    }
    if (i_ >= s_.size()) bad("syntax (unterminated string)");
    ++i_;
    JV v;
    kwkjson::Parser P{s_.data() + b, s_.data() + i_};
    if (!P.value(v) || v.t != JV::STR) bad("syntax (bad string literal)");
    return v.s;
  }

  NodeP pipe() {
    NodeP l = comma();
    if (eat_op("|", {"|="})) return mk2(Node::PIPE, l, pipe());
    return l;
  }
  NodeP comma() {
    NodeP l = alt();
    while (eat(",")) l = mk2(Node::COMMA, l, alt());
    return l;
  }
  NodeP alt() {
    NodeP l = assign();
    if (eat_op("//", {"//="})) return mk2(Node::ALT, l, alt());
    return l;
  }
  NodeP assign() {
    NodeP l = orx();
    static const char* ops[] = {"|=", "+=", "-=", "*=", "/=", "%=", "//="};
    for (const char* op : ops)
      if (eat(op)) return mk2(Node::ASSIGN, l, orx(), op);
    if (eat_op("=", {"=="})) return mk2(Node::ASSIGN, l, orx(), "=");
    return l;
  }
  NodeP orx() {
    NodeP l = andx();
    while (eat_kw("or")) l = mk2(Node::OR, l, andx());
    return l;
  }
  NodeP andx() {
    NodeP l = cmp();
    while (eat_kw("and")) l = mk2(Node::AND, l, cmp());
    return l;
  }
  NodeP cmp() {
    NodeP l = additive();
    static const char* ops[] = {"==", "!=", "<=", ">=", "<", ">"};
    for (const char* op : ops)
      if (eat(op)) return mk2(Node::CMP, l, additive(), op);
    return l;
  }
  NodeP additive() {
    NodeP l = multiplicative();
    for (;;) {
      if (eat_op("+", {"+="})) l = mk2(Node::ARITH, l, multiplicative(), "+");
      else if (eat_op("-", {"-="})) l = mk2(Node::ARITH, l, multiplicative(), "-");
      else return l;
    }
  }
  NodeP multiplicative() {
    NodeP l = unary();
    for (;;) {
      if (eat_op("*", {"*="})) l = mk2(Node::ARITH, l, unary(), "*");
      else if (eat_op("/", {"/=", "//"})) l = mk2(Node::ARITH, l, unary(), "/");
      else if (eat_op("%", {"%="})) l = mk2(Node::ARITH, l, unary(), "%");
      else return l;
    }
  }
  NodeP unary() {
    if (eat_op("-", {"-="})) return mk2(Node::NEG, postfix(), nullptr);
    return postfix();
  }
  NodeP postfix() {
    NodeP n = term();
    for (;;) {
      ws();
      if (i_ >= s_.size()) return n;
      if (at_kw("as")) bad("'as'");
      if (s_[i_] == '?') {
        if (s_.compare(i_, 3, "?//") == 0) bad("'?//'");
        ++i_;
        n = mk2(Node::TRY, n, nullptr);
        continue;
      }
      if (s_[i_] == '[') {
        n = bracket(n);
        continue;
      }
      if (s_[i_] == '.' && i_ + 1 < s_.size()) {
        const char c = s_[i_ + 1];
        if (c == '[') {
          ++i_;
          n = bracket(n);
          continue;
        }
        if (c == '"') {
          ++i_;
          auto f = mk2(Node::FIELD, n, nullptr);
          f->name = string_lit();
          n = f;
          continue;
        }
        if (isalpha((unsigned char)c) || c == '_') {
          ++i_;
          auto f = mk2(Node::FIELD, n, nullptr);
          f->name = ident();
          n = f;
          continue;
        }
      }
      return n;
    }
  }
  // [ ]  |  [ e ]  after a term (the '[' at i_)
  NodeP bracket(NodeP base) {
    expect("[");
    if (eat("]")) return mk2(Node::ITER, base, nullptr);
    if (at(":")) bad("slices");
    NodeP key = pipe();
    if (at(":")) bad("slices");
    expect("]");
    return mk2(Node::INDEX, base, key);
  }
  NodeP term() {
    ws();
    if (i_ >= s_.size()) bad("syntax (unexpected end)");
    const char c = s_[i_];
    if (c == '.') {
      if (s_.compare(i_, 2, "..") == 0) bad("'..'");
      const char d = i_ + 1 < s_.size() ? s_[i_ + 1] : '\0';
      if (isalpha((unsigned char)d) || d == '_') {
        ++i_;
        auto f = mk(Node::FIELD);
        f->a = mk(Node::IDENT);
        f->name = ident();
        return f;
      }
      if (d == '"') {
        ++i_;
        auto f = mk(Node::FIELD);
        f->a = mk(Node::IDENT);
        f->name = string_lit();
        return f;
      }
      if (isdigit((unsigned char)d)) return number();
      ++i_;  // `.` (a following `[` is taken by postfix)
      return mk(Node::IDENT);
    }
    if (c == '$') bad("variables");
    if (c == '@') bad("formats");
    if (isdigit((unsigned char)c)) return number();
    if (c == '"') {
      auto n = mk(Node::LIT);
      n->lit.t = JV::STR;
      n->lit.s = string_lit();
      return n;
    }
    if (c == '(') {
      ++i_;
      NodeP n = pipe();
      expect(")");
      return n;
    }
    if (c == '[') {
      ++i_;
      auto n = mk(Node::ARRAY);
      if (!eat("]")) {
        n->a = pipe();
        expect("]");
      }
      return n;
    }
    if (c == '{') return object();
    if (eat_kw("if")) return if_rest();
    if (eat_kw("try")) {
      NodeP body = postfix();
      if (at_kw("catch")) bad("'try ... catch'");
      return mk2(Node::TRY, body, nullptr);
    }
    for (const char* kw : {"reduce", "foreach", "def", "label", "import", "include", "as", "__loc__"})
      if (at_kw(kw)) bad(std::string("'") + kw + "'");
    if (eat_kw("true")) return lit_bool(true);
    if (eat_kw("false")) return lit_bool(false);
    if (eat_kw("null")) return mk(Node::LIT);
    const std::string name = ident();
    if (name.empty()) bad(std::string("syntax ('") + c + "')");
    auto f = mk(Node::FUNC);
    f->name = name;
    if (eat("(")) {
      for (;;) {
        f->args.push_back(pipe());
        if (eat(";")) continue;
        expect(")");
        break;
      }
    }
    check_builtin(*f);
    return f;
  }
  NodeP lit_bool(bool b) {
    auto n = mk(Node::LIT);
    n->lit.t = JV::BOOL;
    n->lit.b = b;
    return n;
  }
  NodeP number() {
    const size_t b = i_;
    while (i_ < s_.size() && isdigit((unsigned char)s_[i_])) ++i_;
    bool frac = false;
    if (i_ < s_.size() && s_[i_] == '.') {
      frac = true;
      ++i_;
      while (i_ < s_.size() && isdigit((unsigned char)s_[i_])) ++i_;
    }
    if (i_ < s_.size() && (s_[i_] == 'e' || s_[i_] == 'E')) {
      size_t j = i_ + 1;
      if (j < s_.size() && (s_[j] == '+' || s_[j] == '-')) ++j;
      if (j < s_.size() && isdigit((unsigned char)s_[j])) {
        frac = true;
        i_ = j;
        while (i_ < s_.size() && isdigit((unsigned char)s_[i_])) ++i_;
      }
    }
    const std::string t = s_.substr(b, i_ - b);
    auto n = mk(Node::LIT);
    // gojq: a literal that parses as an int is an int, anything else a float64
    if (!frac) {
      errno = 0;
      char* end = nullptr;
      const long long v = strtoll(t.c_str(), &end, 10);
      if (errno == 0 && end && *end == '\0') {
        n->lit = jint((int64_t)v);
        return n;
      }
    }
    n->lit = jfloat(strtod(t.c_str(), nullptr));
    return n;
  }
  NodeP object() {
    expect("{");
    auto n = mk(Node::OBJECT);
    if (eat("}")) return n;
    for (;;) {
      ws();
      NodeP key, val;
      if (i_ < s_.size() && s_[i_] == '"') {
        key = mk(Node::LIT);
        key->lit.t = JV::STR;
        key->lit.s = string_lit();
      } else if (i_ < s_.size() && s_[i_] == '(') {
        ++i_;
        key = pipe();
        expect(")");
      } else if (i_ < s_.size() && s_[i_] == '$') {
        bad("variables");
      } else {
        const std::string id = ident();
        if (id.empty()) bad("syntax (object key)");
        key = mk(Node::LIT);
        key->lit.t = JV::STR;
        key->lit.s = id;
      }
      if (eat(":")) {
        val = objval();
      } else {
        if (key->k != Node::LIT) bad("syntax (object key without a value)");
        val = mk(Node::FIELD);
        val->a = mk(Node::IDENT);
        val->name = key->lit.s;
      }
      n->obj.emplace_back(key, val);
      if (eat(",")) continue;
      expect("}");
      return n;
    }
  }
  NodeP objval() {  // a value inside {...}: no top-level ','
    NodeP l = alt();
    if (eat_op("|", {"|="})) return mk2(Node::PIPE, l, objval());
    return l;
  }
  NodeP if_rest() {
    auto n = mk(Node::IF);
    for (;;) {
      n->args.push_back(pipe());
      if (!eat_kw("then")) bad("syntax (expected 'then')");
      n->args.push_back(pipe());
      if (eat_kw("elif")) continue;
      if (eat_kw("else")) {
        n->args.push_back(pipe());
        if (!eat_kw("end")) bad("syntax (expected 'end')");
        return n;
      }
      if (!eat_kw("end")) bad("syntax (expected 'end')");
      return n;
    }
  }
  void check_builtin(const Node& f) const {
    static const char* f0[] = {"empty", "error", "not", "length", "keys", "keys_unsorted", "type", "tostring",
                               "tonumber", "ascii_downcase", "ascii_upcase", "add", "any", "all", "first", "last",
                               "values"};
    static const char* f1[] = {"error", "has", "startswith", "endswith", "ltrimstr", "rtrimstr", "contains",
                               "select", "map", "first"};
    const auto& tab0 = f0;
    const auto& tab1 = f1;
    if (f.args.empty()) {
      for (const char* x : tab0)
        if (f.name == x) return;
    } else if (f.args.size() == 1) {
      for (const char* x : tab1)
        if (f.name == x) return;
    }
    bad("function " + f.name + "/" + std::to_string(f.args.size()));
  }
};

// ------------------------------------------------------------------ evaluation
using Emit = std::function<void(const Val&)>;
using Path = std::vector<Val>;  // string keys / number indices
using EmitPath = std::function<void(const Path&, const Val&)>;

inline Val field_of(const Val& v, const std::string& key) {
  const JV& x = *v.p;
  if (x.t == JV::NUL) return vnull();
  if (x.t != JV::OBJ) throw Error(std::string("expected an object but got: ") + type_name(x));
  const JV* r = x.get(key);
  return r ? Val{r, v.hold} : vnull();
}
inline Val index_of(const Val& v, const JV& key) {
  const JV& x = *v.p;
  if (key.t == JV::STR) return field_of(v, key.s);
  if (key.t == JV::NUM) {
    if (x.t == JV::NUL) return vnull();
    if (x.t != JV::ARR) throw Error(std::string("expected an array but got: ") + type_name(x));
    const double d = num(key);
    if (d != d) return vnull();
    long long i = (long long)std::floor(d);
    if (i < 0) i += (long long)x.a.size();
    if (i < 0 || i >= (long long)x.a.size()) return vnull();
    return Val{&x.a[(size_t)i], v.hold};
  }
  if (key.t == JV::NUL && x.t == JV::NUL) return vnull();
  throw Error(std::string("cannot index ") + type_name(x) + " with " + type_name(key));
}

inline void iterate(const Val& v, const Emit& emit) {
  const JV& x = *v.p;
  if (x.t == JV::ARR) {
    for (const JV& e : x.a) emit(Val{&e, v.hold});
  } else if (x.t == JV::OBJ) {
    for (const auto& kv : entries(x)) emit(Val{kv.second, v.hold});
  } else {
    throw Error(std::string("cannot iterate over: ") + type_name(x));
  }
}

// an object JV from entries (unique keys, in order)
inline JV make_object(std::vector<std::pair<std::string, JV>>&& kv) {
  JV o;
  o.t = JV::OBJ;
  for (auto& e : kv) {
    bool done = false;
    for (size_t i = 0; i < o.k.size() && !done; ++i)
      if (o.k[i] == e.first) {
        o.a[i] = std::move(e.second);
        done = true;
      }
    if (!done) {
      o.k.push_back(e.first);
      o.a.push_back(std::move(e.second));
    }
  }
  return o;
}
inline std::vector<std::pair<std::string, JV>> object_kv(const JV& o) {
  std::vector<std::pair<std::string, JV>> kv;
  for (const auto& e : entries(o)) kv.emplace_back(*e.first, *e.second);
  return kv;
}

inline JV arith(const std::string& op, const JV& l, const JV& r) {
  const bool ints = is_gint(l) && is_gint(r);
  if (op == "+") {
    if (l.t == JV::NUL) return r;
    if (r.t == JV::NUL) return l;
    if (l.t == JV::NUM && r.t == JV::NUM) {
      int64_t z;
      if (ints && !__builtin_add_overflow(inum(l), inum(r), &z)) return jint(z);
      return jfloat(num(l) + num(r));
    }
    if (l.t == JV::STR && r.t == JV::STR) {
      JV v = l;
      v.s += r.s;
      return v;
    }
    if (l.t == JV::ARR && r.t == JV::ARR) {
      JV v = l;
      for (const JV& e : r.a) v.a.push_back(e);
      return v;
    }
    if (l.t == JV::OBJ && r.t == JV::OBJ) {
      auto kv = object_kv(l);
      for (auto& e : object_kv(r)) kv.push_back(std::move(e));
      return make_object(std::move(kv));
    }
  } else if (op == "-") {
    if (l.t == JV::NUM && r.t == JV::NUM) {
      int64_t z;
      if (ints && !__builtin_sub_overflow(inum(l), inum(r), &z)) return jint(z);
      return jfloat(num(l) - num(r));
    }
    if (l.t == JV::ARR && r.t == JV::ARR) {
      JV v;
      v.t = JV::ARR;
      for (const JV& e : l.a) {
        bool drop = false;
        for (const JV& x : r.a) drop |= compare(e, x) == 0;
        if (!drop) v.a.push_back(e);
      }
      return v;
    }
  } else if (op == "*") {
    if (l.t == JV::NUM && r.t == JV::NUM) {
      int64_t z;
      if (ints && !__builtin_mul_overflow(inum(l), inum(r), &z)) return jint(z);
      return jfloat(num(l) * num(r));
    }
    if (l.t == JV::OBJ && r.t == JV::OBJ) {  // deep merge
      auto kv = object_kv(l);
      for (auto& e : object_kv(r)) {
        bool done = false;
        for (auto& x : kv)
          if (x.first == e.first) {
            x.second = x.second.t == JV::OBJ && e.second.t == JV::OBJ ? arith("*", x.second, e.second) : e.second;
            done = true;
          }
        if (!done) kv.push_back(std::move(e));
      }
      return make_object(std::move(kv));
    }
  } else if (op == "/") {
    if (l.t == JV::NUM && r.t == JV::NUM) {
      if (num(r) == 0.0) throw Error("cannot divide by zero");
      if (ints && inum(l) % inum(r) == 0 && !(inum(r) == -1 && inum(l) == INT64_MIN)) return jint(inum(l) / inum(r));
      return jfloat(num(l) / num(r));
    }
    if (l.t == JV::STR && r.t == JV::STR) {  // split
      JV v;
      v.t = JV::ARR;
      if (l.s.empty()) return v;
      size_t p = 0;
      auto next_cp = [&](size_t i) {  // an empty separator splits into UTF-8 sequences
        ++i;
        while (i < l.s.size() && ((unsigned char)l.s[i] & 0xC0) == 0x80) ++i;
        return i < l.s.size() ? i : std::string::npos;
      };
      for (;;) {
        const size_t q = r.s.empty() ? next_cp(p) : l.s.find(r.s, p);
        JV x;
        x.t = JV::STR;
        x.s = l.s.substr(p, q == std::string::npos ? std::string::npos : q - p);
        v.a.push_back(std::move(x));
        if (q == std::string::npos) break;
        p = q + r.s.size();
      }
      return v;
    }
  } else if (op == "%") {
    if (l.t == JV::NUM && r.t == JV::NUM) {
      const double a = num(l), b = num(r);
      if (a != a || b != b) return jfloat(NAN);
      const int64_t x = (int64_t)a, y = (int64_t)b;
      if (y == 0) throw Error("cannot modulo by zero");
      const int64_t ay = y < 0 ? -y : y;
      int64_t z = (x < 0 ? -x : x) % ay;
      if (x < 0) z = -z;
      return jint(z);
    }
  }
  throw Error(std::string("cannot ") + op + ": " + type_name(l) + " and " + type_name(r));
}

inline bool contains(const JV& a, const JV& b) {
  if (a.t != b.t && !(a.t == JV::NUM && b.t == JV::NUM))
    throw Error(std::string(type_name(a)) + " and " + type_name(b) + " cannot have their containment checked");
  switch (a.t) {
    case JV::STR: return a.s.find(b.s) != std::string::npos;
    case JV::ARR:
      for (const JV& y : b.a) {
        bool any = false;
        for (const JV& x : a.a)
          if (x.t == y.t || (x.t == JV::NUM && y.t == JV::NUM)) any = any || contains(x, y);
        if (!any) return false;
      }
      return true;
    case JV::OBJ:
      for (const auto& kv : entries(b)) {
        const JV* x = a.get(*kv.first);
        if (!x) return false;
        if (x->t != kv.second->t && !(x->t == JV::NUM && kv.second->t == JV::NUM))
          throw Error("cannot have their containment checked");
        if (!contains(*x, *kv.second)) return false;
      }
      return true;
    default: return compare(a, b) == 0;
  }
}

inline JV setpath(const JV& root, const Path& p, size_t i, const JV& val) {
  if (i == p.size()) return val;
  const JV& k = *p[i].p;
  if (k.t == JV::STR) {
    if (root.t != JV::NUL && root.t != JV::OBJ) throw Error(std::string("expected an object but got: ") + type_name(root));
    auto kv = root.t == JV::OBJ ? object_kv(root) : std::vector<std::pair<std::string, JV>>{};
    for (auto& e : kv)
      if (e.first == k.s) {
        e.second = setpath(e.second, p, i + 1, val);
        return make_object(std::move(kv));
      }
    kv.emplace_back(k.s, setpath(null_jv(), p, i + 1, val));
    return make_object(std::move(kv));
  }
  if (k.t != JV::NUM) throw Error("invalid path component");
  if (root.t != JV::NUL && root.t != JV::ARR) throw Error(std::string("expected an array but got: ") + type_name(root));
  JV v = root;
  v.t = JV::ARR;
  long long idx = (long long)std::floor(num(k));
  if (idx < 0) idx += (long long)v.a.size();
  if (idx < 0) throw Error("out of bounds negative array index");
  if (idx > 0x7FFFFFF) throw Error("array index too large");
  while ((long long)v.a.size() <= idx) v.a.emplace_back();
  v.a[(size_t)idx] = setpath(v.a[(size_t)idx], p, i + 1, val);
  return v;
}
inline Val getpath(const Val& root, const Path& p) {
  Val cur = root;
  for (const Val& k : p) cur = index_of(cur, *k.p);
  return cur;
}

inline void eval(const Node& n, const Val& in, const Emit& emit);

// An error raised by the consumer of a sub-expression's outputs (the rest of the pipeline, reached
// through the emit callback) is not the sub-expression's: `try` / `?` / `//` / first(f) only catch
// their own.  Downstream errors travel wrapped in this and are unwrapped at the catch site.
struct Downstream {
  Error e;
  const void* owner;  // the guarded() call whose consumer raised it
};
template <class F>
inline void guarded(const Node& n, const Val& in, const Emit& emit, F&& on_error) {
  const char token = 0;
  try {
    eval(n, in, [&](const Val& v) {
      try {
        emit(v);
      } catch (const Error& e) {
        throw Downstream{e, &token};
      }
    });
  } catch (const Error& e) {
    on_error(e);
  } catch (const Downstream& d) {
    if (d.owner == &token) throw d.e;  // the consumer's own error, past this try
    throw;                              // an outer guard's: unchanged
  }
}

// path expressions (the left side of an assignment)
inline void paths(const Node& n, const Val& in, const Path& base, const EmitPath& emit) {
  switch (n.k) {
    case Node::IDENT: emit(base, in); return;
    case Node::FIELD:
      paths(*n.a, in, base, [&](const Path& p, const Val& v) {
        Path q = p;
        q.push_back(vstr(n.name));
        emit(q, index_of(v, *q.back().p));
      });
      return;
    case Node::INDEX:
      paths(*n.a, in, base, [&](const Path& p, const Val& v) {
        eval(*n.b, in, [&](const Val& key) {
          Path q = p;
          q.push_back(key);
          emit(q, index_of(v, *key.p));
        });
      });
      return;
    case Node::ITER:
      paths(*n.a, in, base, [&](const Path& p, const Val& v) {
        const JV& x = *v.p;
        if (x.t == JV::ARR) {
          for (size_t i = 0; i < x.a.size(); ++i) {
            Path q = p;
            q.push_back(vint((int64_t)i));
            emit(q, Val{&x.a[i], v.hold});
          }
        } else if (x.t == JV::OBJ) {
          for (const auto& kv : entries(x)) {
            Path q = p;
            q.push_back(vstr(*kv.first));
            emit(q, Val{kv.second, v.hold});
          }
        } else if (x.t != JV::NUL) {
          throw Error(std::string("cannot iterate over: ") + type_name(x));
        }
      });
      return;
    case Node::PIPE:
      paths(*n.a, in, base, [&](const Path& p, const Val& v) { paths(*n.b, v, p, emit); });
      return;
    case Node::COMMA:
      paths(*n.a, in, base, emit);
      paths(*n.b, in, base, emit);
      return;
    case Node::TRY: {
      std::vector<std::pair<Path, Val>> got;
      try {
        paths(*n.a, in, base, [&](const Path& p, const Val& v) { got.emplace_back(p, v); });
      } catch (const Error&) {
      }
      for (const auto& pv : got) emit(pv.first, pv.second);
      return;
    }
    case Node::FUNC:
      if (n.name == "select") {
        eval(*n.args[0], in, [&](const Val& c) {
          if (truthy(*c.p)) emit(base, in);
        });
        return;
      }
      if (n.name == "empty") return;
      if (n.name == "first" && n.args.size() == 1) {
        struct Stop {};
        std::vector<std::pair<Path, Val>> got;
        try {
          paths(*n.args[0], in, base, [&](const Path& p, const Val& v) {
            got.emplace_back(p, v);
            throw Stop{};
          });
        } catch (const Stop&) {
        }
        for (const auto& pv : got) emit(pv.first, pv.second);
        return;
      }
      break;
    case Node::IF: {
      const size_t nc = n.args.size() / 2;
      std::function<void(size_t)> branch = [&](size_t i) {
        if (i == nc) {
          if (n.args.size() % 2) paths(*n.args.back(), in, base, emit);
          else emit(base, in);
          return;
        }
        eval(*n.args[2 * i], in, [&](const Val& c) {
          if (truthy(*c.p)) paths(*n.args[2 * i + 1], in, base, emit);
          else branch(i + 1);
        });
      };
      branch(0);
      return;
    }
    default: break;
  }
  throw Error("invalid path expression");
}

inline void eval(const Node& n, const Val& in, const Emit& emit) {
  switch (n.k) {
    case Node::IDENT: emit(in); return;
    case Node::FIELD:
      if (n.a->k == Node::IDENT) return emit(field_of(in, n.name));
      eval(*n.a, in, [&](const Val& v) { emit(field_of(v, n.name)); });
      return;
    case Node::INDEX:
      eval(*n.a, in, [&](const Val& v) { eval(*n.b, in, [&](const Val& key) { emit(index_of(v, *key.p)); }); });
      return;
    case Node::ITER: eval(*n.a, in, [&](const Val& v) { iterate(v, emit); }); return;
    case Node::TRY: guarded(*n.a, in, emit, [](const Error&) {}); return;
    case Node::PIPE: eval(*n.a, in, [&](const Val& v) { eval(*n.b, v, emit); }); return;
    case Node::COMMA:
      eval(*n.a, in, emit);
      eval(*n.b, in, emit);
      return;
    case Node::ALT: {  // the left side's truthy outputs (its errors suppressed), or else the right side's
      std::vector<Val> got;
      try {
        eval(*n.a, in, [&](const Val& v) {
          if (truthy(*v.p)) got.push_back(v);
        });
      } catch (const Error&) {
      }
      if (got.empty()) return eval(*n.b, in, emit);
      for (const Val& v : got) emit(v);
      return;
    }
    case Node::OR:
      eval(*n.a, in, [&](const Val& l) {
        if (truthy(*l.p)) return emit(vbool(true));
        eval(*n.b, in, [&](const Val& r) { emit(vbool(truthy(*r.p))); });
      });
      return;
    case Node::AND:
      eval(*n.a, in, [&](const Val& l) {
        if (!truthy(*l.p)) return emit(vbool(false));
        eval(*n.b, in, [&](const Val& r) { emit(vbool(truthy(*r.p))); });
      });
      return;
    case Node::CMP:  // the right operand outermost, as jq's binary operators
      eval(*n.b, in, [&](const Val& r) {
        eval(*n.a, in, [&](const Val& l) {
          const int c = compare(*l.p, *r.p);
          const std::string& op = n.name;
          emit(vbool(op == "==" ? c == 0 : op == "!=" ? c != 0 : op == "<" ? c < 0 : op == "<=" ? c <= 0
                     : op == ">" ? c > 0 : c >= 0));
        });
      });
      return;
    case Node::ARITH:
      eval(*n.b, in, [&](const Val& r) { eval(*n.a, in, [&](const Val& l) { emit(own(arith(n.name, *l.p, *r.p))); }); });
      return;
    case Node::NEG:
      eval(*n.a, in, [&](const Val& v) {
        const JV& x = *v.p;
        if (x.t != JV::NUM) throw Error(std::string("cannot negate: ") + type_name(x));
        if (is_gint(x) && inum(x) != INT64_MIN) return emit(vint(-inum(x)));
        emit(vfloat(-num(x)));
      });
      return;
    case Node::LIT: emit(Val{&n.lit, nullptr}); return;
    case Node::ARRAY: {
      JV v;
      v.t = JV::ARR;
      if (n.a) eval(*n.a, in, [&](const Val& x) { v.a.push_back(*x.p); });
      emit(own(std::move(v)));
      return;
    }
    case Node::OBJECT: {
      std::vector<std::pair<std::string, JV>> cur;
      std::function<void(size_t)> rec = [&](size_t i) {
        if (i == n.obj.size()) {
          auto kv = cur;
          emit(own(make_object(std::move(kv))));
          return;
        }
        eval(*n.obj[i].first, in, [&](const Val& k) {
          if (k.p->t != JV::STR) throw Error(std::string("expected a string for object key but got: ") + type_name(*k.p));
          eval(*n.obj[i].second, in, [&](const Val& v) {
            cur.emplace_back(k.p->s, *v.p);
            rec(i + 1);
            cur.pop_back();
          });
        });
      };
      rec(0);
      return;
    }
    case Node::IF: {
      const size_t nc = n.args.size() / 2;
      std::function<void(size_t)> branch = [&](size_t i) {
        if (i == nc) {
          if (n.args.size() % 2) eval(*n.args.back(), in, emit);
          else emit(in);
          return;
        }
        eval(*n.args[2 * i], in, [&](const Val& c) {
          if (truthy(*c.p)) eval(*n.args[2 * i + 1], in, emit);
          else branch(i + 1);
        });
      };
      branch(0);
      return;
    }
    case Node::ASSIGN: {
      const std::string& op = n.name;
      if (op == "|=") {  // each path's value replaced by the first output of the right side (none: deleted)
        JV out = *in.p;
        Val cur = in;
        std::vector<Path> ps;
        paths(*n.a, in, Path{}, [&](const Path& p, const Val&) { ps.push_back(p); });
        for (const Path& p : ps) {
          Val old = getpath(Val{&out, nullptr}, p);
          bool got = false;
          JV nv;
          eval(*n.b, old, [&](const Val& x) {
            if (!got) {
              got = true;
              nv = *x.p;
            }
          });
          if (!got) throw Error("update-assignment with no output is not supported");
          out = setpath(out, p, 0, nv);
        }
        (void)cur;
        emit(own(std::move(out)));
        return;
      }
      // `p = v` and `p op= v`: the right side is evaluated on the input, once per output
      eval(*n.b, in, [&](const Val& v) {
        JV out = *in.p;
        std::vector<Path> ps;
        paths(*n.a, in, Path{}, [&](const Path& p, const Val&) { ps.push_back(p); });
        for (const Path& p : ps) {
          if (op == "=") {
            out = setpath(out, p, 0, *v.p);
          } else if (op == "//=") {
            const Val old = getpath(Val{&out, nullptr}, p);
            out = setpath(out, p, 0, truthy(*old.p) ? JV(*old.p) : *v.p);
          } else {
            const Val old = getpath(Val{&out, nullptr}, p);
            out = setpath(out, p, 0, arith(op.substr(0, 1), *old.p, *v.p));
          }
        }
        emit(own(std::move(out)));
      });
      return;
    }
    case Node::FUNC: break;
  }
  // builtins
  const std::string& f = n.name;
  const JV& x = *in.p;
  if (n.args.empty()) {
    if (f == "empty") return;
    if (f == "error") throw Error(x.t == JV::STR ? x.s : "error");
    if (f == "not") return emit(vbool(!truthy(x)));
    if (f == "length") {
      switch (x.t) {
        case JV::NUL: return emit(vint(0));
        case JV::BOOL: throw Error("length cannot be applied to: boolean");
        case JV::NUM:
          if (is_gint(x) && inum(x) == INT64_MIN) return emit(vfloat(9223372036854775808.0));
          if (is_gint(x)) return emit(vint(inum(x) < 0 ? -inum(x) : inum(x)));
          return emit(vfloat(std::fabs(num(x))));
        case JV::STR: {
          int64_t cps = 0;
          for (unsigned char c : x.s) cps += (c & 0xC0) != 0x80;
          return emit(vint(cps));
        }
        case JV::ARR: return emit(vint((int64_t)x.a.size()));
        case JV::OBJ: return emit(vint((int64_t)entries(x).size()));
      }
    }
    if (f == "keys" || f == "keys_unsorted") {
      JV v;
      v.t = JV::ARR;
      if (x.t == JV::OBJ) {
        for (const auto& kv : entries(x)) {
          JV s;
          s.t = JV::STR;
          s.s = *kv.first;
          v.a.push_back(std::move(s));
        }
      } else if (x.t == JV::ARR) {
        for (size_t i = 0; i < x.a.size(); ++i) v.a.push_back(jint((int64_t)i));
      } else {
        throw Error(std::string(f) + " cannot be applied to: " + type_name(x));
      }
      return emit(own(std::move(v)));
    }
    if (f == "type") return emit(vstr(type_name(x)));
    if (f == "tostring") {
      if (x.t == JV::STR) return emit(in);
      std::string s;
      encode(s, x);
      return emit(vstr(std::move(s)));
    }
    if (f == "tonumber") {
      if (x.t == JV::NUM) return emit(in);
      if (x.t != JV::STR) throw Error(std::string("tonumber cannot be applied to: ") + type_name(x));
      errno = 0;
      char* end = nullptr;
      const long long iv = strtoll(x.s.c_str(), &end, 10);
      if (!x.s.empty() && errno == 0 && end && *end == '\0') return emit(vint((int64_t)iv));
      JV probe;
      kwkjson::Parser P{x.s.data(), x.s.data() + x.s.size()};
      if (!P.value(probe) || probe.t != JV::NUM || P.p != P.e) throw Error("cannot parse '" + x.s + "' as number");
      return emit(vfloat(strtod(x.s.c_str(), nullptr)));
    }
    if (f == "ascii_downcase" || f == "ascii_upcase") {
      if (x.t != JV::STR) throw Error(f + " cannot be applied to: " + type_name(x));
      std::string s = x.s;
      for (char& c : s)
        if (f == "ascii_downcase" ? (c >= 'A' && c <= 'Z') : (c >= 'a' && c <= 'z')) c ^= 0x20;
      return emit(vstr(std::move(s)));
    }
    if (f == "add") {
      JV acc;
      bool first = true;
      iterate(in, [&](const Val& e) {
        acc = first ? JV(*e.p) : arith("+", acc, *e.p);
        first = false;
      });
      return emit(own(std::move(acc)));
    }
    if (f == "any" || f == "all") {
      bool r = f == "all";
      iterate(in, [&](const Val& e) {
        if (f == "any") r = r || truthy(*e.p);
        else r = r && truthy(*e.p);
      });
      return emit(vbool(r));
    }
    if (f == "first" || f == "last") {
      JV k = jint(f == "first" ? 0 : -1);
      return emit(index_of(in, k));
    }
    if (f == "values") {
      if (x.t != JV::NUL) emit(in);
      return;
    }
  } else {
    const Node& a0 = *n.args[0];
    if (f == "select") {
      eval(a0, in, [&](const Val& c) {
        if (truthy(*c.p)) emit(in);
      });
      return;
    }
    if (f == "map") {
      JV v;
      v.t = JV::ARR;
      iterate(in, [&](const Val& e) { eval(a0, e, [&](const Val& y) { v.a.push_back(*y.p); }); });
      return emit(own(std::move(v)));
    }
    if (f == "first") {  // first(f): the first output (an error after it is not reached)
      struct Stop {};
      Val first{nullptr, nullptr};
      try {
        eval(a0, in, [&](const Val& y) {
          first = y;
          throw Stop{};
        });
      } catch (const Stop&) {
      }
      if (first.p) emit(first);
      return;
    }
    eval(a0, in, [&](const Val& av) {
      const JV& y = *av.p;
      if (f == "error") throw Error(y.t == JV::STR ? y.s : "error");
      if (f == "has") {
        if (x.t == JV::OBJ && y.t == JV::STR) return emit(vbool(x.get(y.s) != nullptr));
        if (x.t == JV::ARR && y.t == JV::NUM) {  // gojq toInt: truncation
          const double d = num(y);
          if (d != d) return emit(vbool(false));
          const long long i = d >= 9.2e18 ? LLONG_MAX : d <= -9.2e18 ? LLONG_MIN : (long long)d;
          return emit(vbool(i >= 0 && i < (long long)x.a.size()));
        }
        throw Error(std::string("has(") + type_name(y) + ") cannot be applied to: " + type_name(x));
      }
      if (f == "startswith" || f == "endswith") {
        if (x.t != JV::STR || y.t != JV::STR) throw Error(f + "() cannot be applied to: " + type_name(x));
        const bool r = f == "startswith" ? x.s.compare(0, y.s.size(), y.s) == 0
                                         : x.s.size() >= y.s.size() && x.s.compare(x.s.size() - y.s.size(), y.s.size(), y.s) == 0;
        return emit(vbool(r));
      }
      if (f == "ltrimstr" || f == "rtrimstr") {
        if (x.t == JV::STR && y.t == JV::STR) {
          if (f == "ltrimstr" && x.s.compare(0, y.s.size(), y.s) == 0) return emit(vstr(x.s.substr(y.s.size())));
          if (f == "rtrimstr" && x.s.size() >= y.s.size() && x.s.compare(x.s.size() - y.s.size(), y.s.size(), y.s) == 0)
            return emit(vstr(x.s.substr(0, x.s.size() - y.s.size())));
        }
        return emit(in);
      }
      if (f == "contains") return emit(vbool(contains(x, y)));
      throw Error("unknown function " + f);
    });
    return;
  }
  throw Error("unknown function " + f);
}

// ------------------------------------------------------------------ queries
// expression.NewQuery (query.go:33-45): parse + compile (Unsupported outside the subset)
struct Query {
  NodeP root;
  std::string src;
  explicit Query(const std::string& s) : src(s) { root = Parser(src).parse(); }
  // Query.Execute (query.go:48-69): false for the nil result (a runtime error), else the non-null
  // outputs (pointers into `doc` or held values)
  bool execute(const JV& doc, std::vector<Val>& out) const {
    out.clear();
    try {
      eval(*root, Val{&doc, nullptr}, [&](const Val& v) {
        if (v.p->t != JV::NUL) out.push_back(v);
      });
    } catch (const Error&) {
      out.clear();
      return false;
    } catch (const Downstream&) {
      out.clear();
      return false;
    } catch (const std::bad_alloc&) {
      out.clear();
      return false;
    }
    return true;
  }
};

// selector.go:101-111 hasValue: strings, bools (FormatBool) and gojq ints (FormatInt); float64
// JSON numbers never match
inline bool has_value(const JV& d, const std::string& lit) {
  switch (d.t) {
    case JV::STR: return d.s == lit;
    case JV::BOOL: return (d.b ? "true" : "false") == lit;
    case JV::NUM: return is_gint(d) && d.s == lit;
    default: return false;
  }
}

}  // namespace kwkjq
