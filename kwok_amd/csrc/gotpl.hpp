// Go text/template subset for Stage `next` patches, native form of the host compiler's mirror
// (kwok_amd/host/gotpl.py) — what libkwok_compiler renders while it derives the device's
// next-state deltas (exploration) and "patch already applied" bits.
//
// Reference: pkg/utils/gotpl/renderer.go:59-124 (Renderer.ToJSON: JSON round trip of the object
// with UseNumber, template Execute, sigs.k8s.io/yaml.YAMLToJSON), pkg/utils/gotpl/funcs.go:42-116
// (Quote, Now, StartTime, YAML, Version, NodeConditions), text/template's builtins and the sprig
// helpers KWOK's stages use.  Supported, as the Python mirror: text / actions with {{- -}} trimming
// and comments, pipelines, variables ($, $x :=, $x =, $i, $e := range), field chains on dot /
// variables / parenthesised pipelines, string / raw / number / bool / nil literals,
// if / else if / else / range / with / end.
//
// The YAML side (YAMLToJSON) is a block-YAML subset loader with YAML 1.1 (PyYAML SafeLoader)
// scalar resolution minus timestamps — block mappings and sequences, plain / single / double
// quoted scalars, flow collections, comments; anchors, tags, block scalars and multi-line plain
// scalars are rejected (TplError), never guessed.  The YAML template function writes its value
// as a JSON flow collection on one line (the structure YAMLToJSON reads back equals PyYAML's
// block dump read back).
#pragma once
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "host_common.hpp"

namespace kwktpl {

using kwkjson::JV;

struct TplError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// ------------------------------------------------------------------ UTF-8
inline bool utf8_next(const std::string& s, size_t& i, uint32_t& cp) {
  const unsigned char c = (unsigned char)s[i];
  int n;
  if (c < 0x80) { cp = c; n = 1; }
  else if ((c >> 5) == 6) { cp = c & 0x1F; n = 2; }
  else if ((c >> 4) == 14) { cp = c & 0x0F; n = 3; }
  else if ((c >> 3) == 30) { cp = c & 0x07; n = 4; }
  else { cp = c; ++i; return false; }
  if (i + n > s.size()) { cp = c; ++i; return false; }
  for (int k = 1; k < n; ++k) cp = (cp << 6) | ((unsigned char)s[i + k] & 0x3F);
  i += n;
  return true;
}

inline void utf8_put(std::string& o, uint32_t c) { kwkjson::Parser::utf8(o, c); }

// ------------------------------------------------------------------ Go JSON encoding
// gotpl.go_json_string: encoding/json string encoding with escapeHTML (Go 1.22)
inline std::string go_json_string(const std::string& s) {
  std::string o = "\"";
  size_t i = 0;
  while (i < s.size()) {
    const size_t at = i;
    uint32_t cp;
    if (!utf8_next(s, i, cp)) { o.append(s, at, i - at); continue; }
    char buf[8];
    switch (cp) {
      case '"': o += "\\\""; continue;
      case '\\': o += "\\\\"; continue;
      case '\n': o += "\\n"; continue;
      case '\r': o += "\\r"; continue;
      case '\t': o += "\\t"; continue;
      case '\b': o += "\\b"; continue;
      case '\f': o += "\\f"; continue;
      default: break;
    }
    if (cp < 0x20 || cp == '<' || cp == '>' || cp == '&' || cp == 0x2028 || cp == 0x2029) {
      snprintf(buf, sizeof buf, "\\u%04x", cp);
      o += buf;
    } else {
      o.append(s, at, i - at);
    }
  }
  o += '"';
  return o;
}

// shortest round-trip digits of |d| and the decimal point position (digits "d1d2.." x 10^(point-len))
inline void shortest_digits(double a, std::string& digits, int& point) {
  char buf[40];
  int prec = 1;
  for (; prec <= 17; ++prec) {
    snprintf(buf, sizeof buf, "%.*e", prec - 1, a);
    if (strtod(buf, nullptr) == a) break;
  }
  std::string m(buf);
  const size_t ep = m.find('e');
  const int exp10 = atoi(m.c_str() + ep + 1);
  digits.clear();
  for (size_t i = 0; i < ep; ++i)
    if (m[i] >= '0' && m[i] <= '9') digits += m[i];
  while (digits.size() > 1 && digits.back() == '0') digits.pop_back();
  point = exp10 + 1;
}

// gotpl.go_json_float: encoding/json float64 ('f' unless |f| < 1e-6 or >= 1e21, then 'e' with
// the exponent's leading zero dropped for negative two-digit exponents)
inline std::string go_json_float(double f) {
  if (std::isnan(f) || std::isinf(f)) throw TplError("json: unsupported value");
  if (f == 0) return std::signbit(f) ? "-0" : "0";
  const double a = std::fabs(f);
  std::string s;
  int point;
  shortest_digits(a, s, point);
  std::string out;
  if (a < 1e-6 || a >= 1e21) {
    const int e = point - 1;
    out = s.substr(0, 1) + (s.size() > 1 ? "." + s.substr(1) : "");
    char buf[16];
    snprintf(buf, sizeof buf, "e%c%02d", e < 0 ? '-' : '+', e < 0 ? -e : e);
    out += buf;
    if (e < 0 && out[out.size() - 2] == '0') out.erase(out.size() - 2, 1);
  } else if (point <= 0) {
    out = "0." + std::string((size_t)(-point), '0') + s;
  } else if (point >= (int)s.size()) {
    out = s + std::string((size_t)(point - (int)s.size()), '0');
  } else {
    out = s.substr(0, (size_t)point) + "." + s.substr((size_t)point);
  }
  return (f < 0 ? "-" : "") + out;
}

// gotpl.go_json_bytes of a decoded YAML / JSON value (JV: numbers with is_int are Python ints,
// the others Python floats)
inline void go_json_bytes(std::string& o, const JV& v) {
  switch (v.t) {
    case JV::NUL: o += "null"; return;
    case JV::BOOL: o += v.b ? "true" : "false"; return;
    case JV::NUM:
      if (v.is_int) o += v.s;
      else o += go_json_float(strtod(v.s.c_str(), nullptr));
      return;
    case JV::STR: o += go_json_string(v.s); return;
    case JV::ARR:
      o += '[';
      for (size_t i = 0; i < v.a.size(); ++i) {
        if (i) o += ',';
        go_json_bytes(o, v.a[i]);
      }
      o += ']';
      return;
    case JV::OBJ: {
      std::map<std::string, const JV*> m;
      for (size_t i = 0; i < v.k.size(); ++i) m[v.k[i]] = &v.a[i];
      o += '{';
      bool first = true;
      for (const auto& kv : m) {
        if (!first) o += ',';
        first = false;
        o += go_json_string(kv.first);
        o += ':';
        go_json_bytes(o, *kv.second);
      }
      o += '}';
      return;
    }
  }
}

// Python's int() of a JSON integer literal as text (JSON has no '+' or leading zeros)
inline std::string py_int_text(const std::string& s) { return s == "-0" ? "0" : s; }

// a JV number's text as Python json.dumps writes the value json.loads gave
inline std::string py_num_text(const JV& v) {
  return v.is_int ? py_int_text(v.s) : kwkhost::py_float_repr(strtod(v.s.c_str(), nullptr));
}

// ------------------------------------------------------------------ template values
// gotpl's Go data: MISSING (an invalid reflect.Value: a missing map key), nil, bool, json.Number
// (NUM, its text), string, []interface{}, map[string]interface{} (keys sorted, unique)
struct TV {
  enum K : uint8_t { MISSING, NIL, BOOL, NUM, STR, ARR, OBJ } k = NIL;
  bool b = false;
  bool pyint = false;  // NUM produced as a Python int by a function (NodePort): truthy iff != 0
  std::string s;
  std::shared_ptr<const std::vector<TV>> arr;
  std::shared_ptr<const std::vector<std::pair<std::string, TV>>> obj;

  static TV missing() { TV t; t.k = MISSING; return t; }
  static TV nil() { return TV(); }
  static TV boolean(bool x) { TV t; t.k = BOOL; t.b = x; return t; }
  static TV num(std::string x) { TV t; t.k = NUM; t.s = std::move(x); return t; }
  static TV str(std::string x) { TV t; t.k = STR; t.s = std::move(x); return t; }
  static TV list(std::vector<TV> xs) {
    TV t;
    t.k = ARR;
    t.arr = std::make_shared<const std::vector<TV>>(std::move(xs));
    return t;
  }
  static TV dict(std::map<std::string, TV> m) {
    TV t;
    t.k = OBJ;
    std::vector<std::pair<std::string, TV>> v(m.begin(), m.end());
    t.obj = std::make_shared<const std::vector<std::pair<std::string, TV>>>(std::move(v));
    return t;
  }
  const TV* get(const std::string& key) const {
    if (k != OBJ) return nullptr;
    size_t lo = 0, hi = obj->size();
    while (lo < hi) {
      const size_t mid = (lo + hi) / 2;
      const int c = (*obj)[mid].first.compare(key);
      if (c == 0) return &(*obj)[mid].second;
      if (c < 0) lo = mid + 1;
      else hi = mid;
    }
    return nullptr;
  }
  size_t size() const { return k == ARR ? arr->size() : k == OBJ ? obj->size() : s.size(); }
};

// _to_go_data(json.loads(json.dumps(data))): numbers become json.Number of Python's text
inline TV from_jv(const JV& v) {
  switch (v.t) {
    case JV::NUL: return TV::nil();
    case JV::BOOL: return TV::boolean(v.b);
    case JV::NUM: return TV::num(py_num_text(v));
    case JV::STR: return TV::str(v.s);
    case JV::ARR: {
      std::vector<TV> xs;
      xs.reserve(v.a.size());
      for (const JV& x : v.a) xs.push_back(from_jv(x));
      return TV::list(std::move(xs));
    }
    case JV::OBJ: {
      std::map<std::string, TV> m;
      for (size_t i = 0; i < v.k.size(); ++i) m[v.k[i]] = from_jv(v.a[i]);  // the last duplicate wins
      return TV::dict(std::move(m));
    }
  }
  return TV::nil();
}

// _from_go_data: json.Number -> json.loads(text) (int or float), MISSING -> None
inline JV to_jv(const TV& v) {
  JV j;
  switch (v.k) {
    case TV::MISSING:
    case TV::NIL: j.t = JV::NUL; break;
    case TV::BOOL: j.t = JV::BOOL; j.b = v.b; break;
    case TV::NUM: {
      j.t = JV::NUM;
      kwkjson::Parser P{v.s.data(), v.s.data() + v.s.size()};
      JV n;
      if (!P.value(n) || n.t != JV::NUM) throw TplError("invalid number " + v.s);
      j.is_int = n.is_int;
      j.s = n.is_int ? py_int_text(n.s) : kwkhost::py_float_repr(strtod(n.s.c_str(), nullptr));
      break;
    }
    case TV::STR: j.t = JV::STR; j.s = v.s; break;
    case TV::ARR:
      j.t = JV::ARR;
      for (const TV& x : *v.arr) j.a.push_back(to_jv(x));
      break;
    case TV::OBJ:
      j.t = JV::OBJ;
      for (const auto& kv : *v.obj) {
        j.k.push_back(kv.first);
        j.a.push_back(to_jv(kv.second));
      }
      break;
  }
  return j;
}

inline bool truth(const TV& v) {
  switch (v.k) {
    case TV::MISSING:
    case TV::NIL: return false;
    case TV::BOOL: return v.b;
    case TV::NUM: return v.pyint ? strtod(v.s.c_str(), nullptr) != 0 : !v.s.empty();
    case TV::STR: return !v.s.empty();
    case TV::ARR: return !v.arr->empty();
    case TV::OBJ: return !v.obj->empty();
  }
  return true;
}

// fmt.Sprint of a template value (gotpl.go_sprint)
inline std::string go_sprint(const TV& v) {
  switch (v.k) {
    case TV::MISSING: return "<no value>";
    case TV::NIL: return "<nil>";
    case TV::BOOL: return v.b ? "true" : "false";
    case TV::NUM:
    case TV::STR: return v.s;
    case TV::ARR: {
      std::string o = "[";
      for (size_t i = 0; i < v.arr->size(); ++i) {
        if (i) o += ' ';
        o += go_sprint((*v.arr)[i]);
      }
      return o + "]";
    }
    case TV::OBJ: {
      std::string o = "map[";
      bool first = true;
      for (const auto& kv : *v.obj) {
        if (!first) o += ' ';
        first = false;
        o += kv.first + ":" + go_sprint(kv.second);
      }
      return o + "]";
    }
  }
  return "";
}

// go_json_marshal of a template value (json.Number keeps its text, maps sorted)
inline void tv_json(std::string& o, const TV& v) {
  switch (v.k) {
    case TV::MISSING:
    case TV::NIL: o += "null"; return;
    case TV::BOOL: o += v.b ? "true" : "false"; return;
    case TV::NUM: o += v.s; return;
    case TV::STR: o += go_json_string(v.s); return;
    case TV::ARR:
      o += '[';
      for (size_t i = 0; i < v.arr->size(); ++i) {
        if (i) o += ',';
        tv_json(o, (*v.arr)[i]);
      }
      o += ']';
      return;
    case TV::OBJ: {
      o += '{';
      bool first = true;
      for (const auto& kv : *v.obj) {
        if (!first) o += ',';
        first = false;
        o += go_json_string(kv.first) + ":";
        tv_json(o, kv.second);
      }
      o += '}';
      return;
    }
  }
}

// Python json.dumps of a str (ensure_ascii), as gotpl.quote uses for a non-string JSON text
inline std::string py_json_string(const std::string& s) {
  std::string o;
  kwkhost::esc(o, s);
  return o;
}

// gotpl.rfc3339nano: time.Time.Format(time.RFC3339Nano) in UTC
inline std::string rfc3339nano(int64_t ns) {
  int64_t sec = ns / 1000000000, frac = ns % 1000000000;
  if (frac < 0) { frac += 1000000000; --sec; }
  int64_t days = sec / 86400, rem = sec % 86400;
  if (rem < 0) { rem += 86400; --days; }
  // civil from days (Howard Hinnant)
  days += 719468;
  const int64_t era = (days >= 0 ? days : days - 146096) / 146097;
  const int64_t doe = days - era * 146097;
  const int64_t yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
  int64_t y = yoe + era * 400;
  const int64_t doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
  const int64_t mp = (5 * doy + 2) / 153;
  const int64_t d = doy - (153 * mp + 2) / 5 + 1;
  const int64_t m = mp < 10 ? mp + 3 : mp - 9;
  if (m <= 2) ++y;
  char buf[64];
  snprintf(buf, sizeof buf, "%04lld-%02lld-%02lldT%02lld:%02lld:%02lld", (long long)y, (long long)m, (long long)d,
           (long long)(rem / 3600), (long long)(rem % 3600 / 60), (long long)(rem % 60));
  std::string o(buf);
  if (frac) {
    snprintf(buf, sizeof buf, "%09lld", (long long)frac);
    std::string f(buf);
    while (!f.empty() && f.back() == '0') f.pop_back();
    o += "." + f;
  }
  return o + "Z";
}

// ------------------------------------------------------------------ parse tree
struct Pipe;
struct Operand {
  enum K : uint8_t { LIT, DOT, VAR, FIELD, PAREN, IDENT } k = LIT;
  TV lit;                              // LIT (a raw / double-quoted string, json.Number, bool, nil)
  bool lit_str = false;                // LIT of a string literal
  std::string name;                    // VAR ($name) / IDENT
  std::shared_ptr<Operand> base;       // FIELD: the operand the chain starts from
  std::vector<std::string> path;       // FIELD
  std::shared_ptr<Pipe> pipe;          // PAREN
};
using Cmd = std::vector<Operand>;
struct Pipe {
  bool has_decl = false;
  std::vector<std::string> names;      // $x := / $i, $e := / $x =
  bool decl = true;                    // ":=" (else "=")
  std::vector<Cmd> cmds;
};
struct Node {
  enum K : uint8_t { TEXT, ACTION, IF, RANGE, WITH } k = TEXT;
  std::string text;
  Pipe pipe;
  std::vector<Node> body;
  bool has_else = false;
  std::vector<Node> els;
};

// ---- lexer (gotpl._TOKEN, tried in the same order)
struct Tok {
  enum K : uint8_t { STR, RAW, NUM, DECL, ASSIGN, PIPE, LP, RP, COMMA, VAR, FIELD, DOT, IDENT, END } k;
  std::string v;
};

inline bool is_alpha_(char c) { return (c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z') || c == '_'; }
inline bool is_digit(char c) { return c >= '0' && c <= '9'; }
inline bool is_alnum_(char c) { return is_alpha_(c) || is_digit(c); }
inline bool is_space(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\f' || c == '\v'; }

inline std::vector<Tok> tokenize(const std::string& src) {
  std::vector<Tok> out;
  size_t i = 0;
  const size_t n = src.size();
  while (i < n) {
    const char c = src[i];
    if (is_space(c)) { ++i; continue; }
    if (c == '"') {
      size_t j = i + 1;
      while (j < n && src[j] != '"') j += src[j] == '\\' ? 2 : 1;
      if (j >= n) throw TplError("bad token at " + src.substr(i, 20));
      out.push_back({Tok::STR, src.substr(i, j + 1 - i)});
      i = j + 1;
      continue;
    }
    if (c == '`') {
      const size_t j = src.find('`', i + 1);
      if (j == std::string::npos) throw TplError("bad token at " + src.substr(i, 20));
      out.push_back({Tok::RAW, src.substr(i, j + 1 - i)});
      i = j + 1;
      continue;
    }
    if (is_digit(c) || (c == '-' && i + 1 < n && is_digit(src[i + 1]))) {
      size_t j = i + (c == '-' ? 1 : 0);
      while (j < n && is_digit(src[j])) ++j;
      if (j + 1 < n && src[j] == '.' && is_digit(src[j + 1])) {
        ++j;
        while (j < n && is_digit(src[j])) ++j;
      }
      out.push_back({Tok::NUM, src.substr(i, j - i)});
      i = j;
      continue;
    }
    if (c == ':' && i + 1 < n && src[i + 1] == '=') { out.push_back({Tok::DECL, ":="}); i += 2; continue; }
    if (c == '=') { out.push_back({Tok::ASSIGN, "="}); ++i; continue; }
    if (c == '|') { out.push_back({Tok::PIPE, "|"}); ++i; continue; }
    if (c == '(') { out.push_back({Tok::LP, "("}); ++i; continue; }
    if (c == ')') { out.push_back({Tok::RP, ")"}); ++i; continue; }
    if (c == ',') { out.push_back({Tok::COMMA, ","}); ++i; continue; }
    if (c == '$') {
      size_t j = i + 1;
      while (j < n && is_alnum_(src[j])) ++j;
      out.push_back({Tok::VAR, src.substr(i, j - i)});
      i = j;
      continue;
    }
    if (c == '.') {
      size_t j = i;
      while (j + 1 < n && src[j] == '.' && is_alpha_(src[j + 1])) {
        j += 2;
        while (j < n && is_alnum_(src[j])) ++j;
      }
      if (j > i) {
        out.push_back({Tok::FIELD, src.substr(i, j - i)});
        i = j;
      } else {
        out.push_back({Tok::DOT, "."});
        ++i;
      }
      continue;
    }
    if (is_alpha_(c)) {
      size_t j = i;
      while (j < n && is_alnum_(src[j])) ++j;
      out.push_back({Tok::IDENT, src.substr(i, j - i)});
      i = j;
      continue;
    }
    throw TplError("bad token at " + src.substr(i, 20));
  }
  return out;
}

inline std::vector<std::string> split_fields(const std::string& f) {  // ".a.b" -> {a, b}
  std::vector<std::string> out;
  size_t i = 1;
  while (i <= f.size()) {
    const size_t j = f.find('.', i);
    out.push_back(f.substr(i, j == std::string::npos ? std::string::npos : j - i));
    if (j == std::string::npos) break;
    i = j + 1;
  }
  return out;
}

struct PipeParser {
  std::vector<Tok> t;
  size_t i = 0;
  Tok::K peek(size_t k = 0) const { return i + k < t.size() ? t[i + k].k : Tok::END; }
  Tok take() { return i < t.size() ? t[i++] : Tok{Tok::END, ""}; }

  Pipe pipeline() {
    Pipe p;
    if (peek() == Tok::VAR) {
      if (peek(1) == Tok::DECL || peek(1) == Tok::ASSIGN) {
        p.has_decl = true;
        p.names.push_back(take().v);
        p.decl = take().k == Tok::DECL;
      } else if (peek(1) == Tok::COMMA && peek(2) == Tok::VAR && peek(3) == Tok::DECL) {
        p.has_decl = true;
        p.names.push_back(take().v);
        take();
        p.names.push_back(take().v);
        take();
        p.decl = true;
      }
    }
    p.cmds.push_back(command());
    while (peek() == Tok::PIPE) {
      take();
      p.cmds.push_back(command());
    }
    return p;
  }
  Cmd command() {
    Cmd args;
    while (peek() != Tok::END && peek() != Tok::PIPE && peek() != Tok::RP) args.push_back(operand());
    if (args.empty()) throw TplError("empty command");
    return args;
  }
  Operand field_on(Operand base) {
    Operand f;
    f.k = Operand::FIELD;
    f.base = std::make_shared<Operand>(std::move(base));
    f.path = split_fields(take().v);
    return f;
  }
  Operand operand() {
    const Tok tk = take();
    Operand o;
    switch (tk.k) {
      case Tok::FIELD: {
        Operand d;
        d.k = Operand::DOT;
        o.k = Operand::FIELD;
        o.base = std::make_shared<Operand>(d);
        o.path = split_fields(tk.v);
        return o;
      }
      case Tok::DOT: o.k = Operand::DOT; return o;
      case Tok::VAR:
        o.k = Operand::VAR;
        o.name = tk.v;
        if (peek() == Tok::FIELD) return field_on(std::move(o));
        return o;
      case Tok::STR: {
        JV s;
        kwkjson::Parser P{tk.v.data(), tk.v.data() + tk.v.size()};
        if (!P.value(s) || s.t != JV::STR) throw TplError("bad string literal " + tk.v);
        o.lit = TV::str(s.s);
        o.lit_str = true;
        return o;
      }
      case Tok::RAW:
        o.lit = TV::str(tk.v.substr(1, tk.v.size() - 2));
        o.lit_str = true;
        return o;
      case Tok::NUM: o.lit = TV::num(tk.v); return o;
      case Tok::LP: {
        o.k = Operand::PAREN;
        o.pipe = std::make_shared<Pipe>(pipeline());
        if (take().k != Tok::RP) throw TplError("missing )");
        if (peek() == Tok::FIELD) return field_on(std::move(o));
        return o;
      }
      case Tok::IDENT:
        if (tk.v == "true" || tk.v == "false") { o.lit = TV::boolean(tk.v == "true"); return o; }
        if (tk.v == "nil") { o.lit = TV::nil(); return o; }
        o.k = Operand::IDENT;
        o.name = tk.v;
        return o;
      default: throw TplError("unexpected token " + tk.v);
    }
  }
};

inline Pipe parse_pipe(const std::string& src) {
  PipeParser P;
  P.t = tokenize(src);
  return P.pipeline();  // as the mirror: a trailing ')' after the pipeline is not looked at
}

inline std::string py_strip(const std::string& s) {
  size_t a = 0, b = s.size();
  while (a < b && is_space(s[a])) ++a;
  while (b > a && is_space(s[b - 1])) --b;
  return s.substr(a, b - a);
}
inline std::string py_rstrip(const std::string& s) {
  size_t b = s.size();
  while (b > 0 && is_space(s[b - 1])) --b;
  return s.substr(0, b);
}
inline std::string py_lstrip(const std::string& s) {
  size_t a = 0;
  while (a < s.size() && is_space(s[a])) ++a;
  return s.substr(a);
}

// gotpl._parse: text / actions, {{- -}} trimming, control blocks
struct TemplateParser {
  struct Item {
    bool act = false;
    std::string s;
    bool ltrim = false, rtrim = false;
  };
  std::vector<Item> items;

  explicit TemplateParser(const std::string& text) {
    size_t pos = 0;
    for (;;) {
      const size_t a = text.find("{{", pos);
      if (a == std::string::npos) break;
      const size_t e = text.find("}}", a + 2);
      if (e == std::string::npos) break;
      items.push_back({false, text.substr(pos, a - pos)});
      Item it;
      it.act = true;
      size_t b = a + 2;
      if (b + 1 < e && text[b] == '-' && is_space(text[b + 1])) {  // (-\s)?
        it.ltrim = true;
        b += 2;
      }
      size_t end = e;
      if (end >= b + 2 && text[end - 1] == '-' && is_space(text[end - 2])) {
        it.rtrim = true;
        end -= 2;
      }
      it.s = text.substr(b, end - b);
      items.push_back(it);
      pos = e + 2;
    }
    items.push_back({false, text.substr(pos)});
    for (size_t k = 0; k < items.size(); ++k) {
      if (!items[k].act) continue;
      if (items[k].ltrim && k > 0 && !items[k - 1].act) items[k - 1].s = py_rstrip(items[k - 1].s);
      if (items[k].rtrim && k + 1 < items.size() && !items[k + 1].act) items[k + 1].s = py_lstrip(items[k + 1].s);
    }
  }

  static void word_rest(const std::string& src, std::string& word, std::string& rest) {
    size_t i = 0;
    while (i < src.size() && !is_space(src[i])) ++i;
    word = src.substr(0, i);
    rest = py_strip(src.substr(i));
  }

  // -> nodes; i advanced; term = the {{end}} / {{else...}} source that stopped the block
  std::vector<Node> block(size_t& i, bool stop_else, bool stop_end, std::string& term) {
    std::vector<Node> nodes;
    while (i < items.size()) {
      const Item& it = items[i];
      if (!it.act) {
        if (!it.s.empty()) {
          Node n;
          n.k = Node::TEXT;
          n.text = it.s;
          nodes.push_back(std::move(n));
        }
        ++i;
        continue;
      }
      const std::string src = py_strip(it.s);
      if (src.rfind("/*", 0) == 0) { ++i; continue; }
      std::string word, rest;
      word_rest(src, word, rest);
      if (word == "end" || word == "else") {
        if ((word == "end" && stop_end) || (word == "else" && stop_else)) {
          term = src;
          return nodes;
        }
        throw TplError("unexpected {{" + src + "}}");
      }
      if (word == "if" || word == "range" || word == "with") {
        ++i;
        nodes.push_back(control(word, rest, i));
        continue;
      }
      Node n;
      n.k = Node::ACTION;
      n.pipe = parse_pipe(src);
      nodes.push_back(std::move(n));
      ++i;
    }
    if (stop_end) throw TplError("missing {{end}}");
    term.clear();
    return nodes;
  }

  Node control(const std::string& word, const std::string& rest, size_t& i) {
    Node n;
    n.k = word == "if" ? Node::IF : word == "range" ? Node::RANGE : Node::WITH;
    n.pipe = parse_pipe(rest);
    std::string term;
    n.body = block(i, true, true, term);
    if (term.rfind("else", 0) == 0) {
      const std::string rest2 = py_strip(term.substr(4));
      n.has_else = true;
      if (rest2.rfind("if ", 0) == 0 || rest2.rfind("with ", 0) == 0) {
        std::string w2, r2;
        word_rest(rest2, w2, r2);
        ++i;
        n.els.push_back(control(w2, r2, i));
        return n;
      }
      ++i;
      std::string t2;
      n.els = block(i, false, true, t2);
    }
    ++i;
    return n;
  }

  std::vector<Node> parse() {
    size_t i = 0;
    std::string term;
    return block(i, false, false, term);
  }
};

inline std::vector<Node> parse_template(const std::string& text) { return TemplateParser(text).parse(); }

// ------------------------------------------------------------------ execution
using Func = std::function<TV(std::vector<TV>&)>;

// NODE_CONDITIONS (funcs.go:85-116: k8s.io/api NodeCondition JSON, zero times null), as JSON text
// in the Python mirror's key order
inline const char* node_conditions_json() {
  return "[{\"type\": \"Ready\", \"status\": \"True\", \"lastHeartbeatTime\": null, \"lastTransitionTime\": null, "
         "\"reason\": \"KubeletReady\", \"message\": \"kubelet is posting ready status\"}, "
         "{\"type\": \"MemoryPressure\", \"status\": \"False\", \"lastHeartbeatTime\": null, \"lastTransitionTime\": null, "
         "\"reason\": \"KubeletHasSufficientMemory\", \"message\": \"kubelet has sufficient memory available\"}, "
         "{\"type\": \"DiskPressure\", \"status\": \"False\", \"lastHeartbeatTime\": null, \"lastTransitionTime\": null, "
         "\"reason\": \"KubeletHasNoDiskPressure\", \"message\": \"kubelet has no disk pressure\"}, "
         "{\"type\": \"PIDPressure\", \"status\": \"False\", \"lastHeartbeatTime\": null, \"lastTransitionTime\": null, "
         "\"reason\": \"KubeletHasSufficientPID\", \"message\": \"kubelet has sufficient PID available\"}, "
         "{\"type\": \"NetworkUnavailable\", \"status\": \"False\", \"lastHeartbeatTime\": null, \"lastTransitionTime\": null, "
         "\"reason\": \"RouteCreated\", \"message\": \"RouteController created a route\"}]";
}

inline JV parse_json_text(const std::string& s) {
  JV v;
  kwkjson::Parser P{s.data(), s.data() + s.size()};
  if (!P.value(v)) throw TplError("invalid JSON");
  return v;
}

// _basic: the comparison class of a value
inline int basic_kind(const TV& v) {  // 0 invalid, 1 bool, 2 string (str and json.Number), 3 other
  switch (v.k) {
    case TV::MISSING:
    case TV::NIL: return 0;
    case TV::BOOL: return 1;
    case TV::NUM:
    case TV::STR: return 2;
    default: return 3;
  }
}

inline bool tpl_eq(const TV& a, const std::vector<TV>& bs, size_t from) {
  const int ka = basic_kind(a);
  for (size_t i = from; i < bs.size(); ++i) {
    const int kb = basic_kind(bs[i]);
    if (ka != kb) {
      if (ka != 0 && kb != 0) throw TplError("incompatible types for comparison");
      continue;
    }
    if (ka == 3) throw TplError("non-comparable type");
    if (ka == 0) return true;
    if (ka == 1 ? a.b == bs[i].b : a.s == bs[i].s) return true;
  }
  return false;
}

struct Renderer {
  std::map<std::string, Func> funcs;
  std::map<std::string, std::vector<Node>> cache;

  // gotpl.default_funcs(now_ns, version)
  explicit Renderer(int64_t now_ns = 0, const std::string& version = "v0.6.0") {
    funcs["Quote"] = [](std::vector<TV>& a) {
      if (a.size() != 1) throw TplError("Quote: wrong number of args");
      std::string d;
      tv_json(d, a[0]);
      if (d.empty()) return TV::str("\"\"");
      if (d[0] == '"') return TV::str(d);
      return TV::str(py_json_string(d));
    };
    set_now(now_ns);
    const std::string st = rfc3339nano(now_ns);
    funcs["StartTime"] = [st](std::vector<TV>&) { return TV::str(st); };
    funcs["YAML"] = [](std::vector<TV>& a) {
      if (a.empty()) throw TplError("YAML: wrong number of args");
      // written as a JSON flow collection (see the header); indent as gotpl.yaml_func
      std::string data;
      go_json_bytes(data, to_jv(a[0]));
      data += "\n";
      if (a.size() == 2) {
        const long ind = strtol(go_sprint(a[1]).c_str(), nullptr, 10);
        if (ind > 0) {
          const std::string pad((size_t)ind * 2, ' ');
          std::string d2 = "\n" + data, out;
          for (char c : d2) {
            out += c;
            if (c == '\n') out += pad;
          }
          data = out;
        }
      }
      return TV::str(data);
    };
    funcs["Version"] = [version](std::vector<TV>&) { return TV::str(version); };
    funcs["NodeConditions"] = [](std::vector<TV>&) { return from_jv(parse_json_text(node_conditions_json())); };
  }
  void set_now(int64_t now_ns) {
    const std::string t = rfc3339nano(now_ns);
    funcs["Now"] = [t](std::vector<TV>&) { return TV::str(t); };
  }
  // compiler.exploration_funcs: deterministic stand-ins for the controllers' functions
  void exploration_funcs() {
    funcs["NodeIP"] = [](std::vector<TV>&) { return TV::str("10.0.0.1"); };
    funcs["NodeName"] = [](std::vector<TV>&) { return TV::str("node"); };
    funcs["NodePort"] = [](std::vector<TV>&) { TV t = TV::num("10250"); t.pyint = true; return t; };
    funcs["PodIP"] = [](std::vector<TV>&) { return TV::str("10.0.0.2"); };
    funcs["NodeIPWith"] = [](std::vector<TV>&) { return TV::str("10.0.0.1"); };
    funcs["PodIPWith"] = [](std::vector<TV>&) { return TV::str("10.0.0.2"); };
  }

  const std::vector<Node>& tree(const std::string& text) {
    const std::string t = py_strip(text);  // renderer.go:60
    auto it = cache.find(t);
    if (it == cache.end()) it = cache.emplace(t, parse_template(t)).first;
    return it->second;
  }

  using Scopes = std::vector<std::map<std::string, TV>>;

  std::string to_text(const std::string& text, const JV& data) {
    const TV root = from_jv(data);
    Scopes sc(1);
    sc[0]["$"] = root;
    std::string out;
    exec(tree(text), root, sc, out);
    return out;
  }

  void exec(const std::vector<Node>& nodes, const TV& dot, Scopes& sc, std::string& out) {
    for (const Node& n : nodes) {
      switch (n.k) {
        case Node::TEXT: out += n.text; break;
        case Node::ACTION: {
          TV v = pipe(n.pipe, dot, sc);
          if (!n.pipe.has_decl) out += go_sprint(v);
          break;
        }
        case Node::IF: {
          sc.emplace_back();
          const TV v = pipe(n.pipe, dot, sc);
          if (truth(v)) exec(n.body, dot, sc, out);
          else if (n.has_else) exec(n.els, dot, sc, out);
          sc.pop_back();
          break;
        }
        case Node::WITH: {
          sc.emplace_back();
          const TV v = pipe(n.pipe, dot, sc);
          if (truth(v)) exec(n.body, v, sc, out);
          else if (n.has_else) exec(n.els, dot, sc, out);
          sc.pop_back();
          break;
        }
        case Node::RANGE: {
          sc.emplace_back();
          Pipe p = n.pipe;
          p.has_decl = false;
          const TV v = pipe(p, dot, sc);
          std::vector<std::pair<TV, TV>> items;
          if (v.k == TV::NIL) throw TplError("range can't iterate over <nil>");
          if (v.k == TV::ARR) {
            for (size_t i = 0; i < v.arr->size(); ++i) items.emplace_back(TV::num(std::to_string(i)), (*v.arr)[i]);
          } else if (v.k == TV::OBJ) {
            for (const auto& kv : *v.obj) items.emplace_back(TV::str(kv.first), kv.second);
          } else if (v.k == TV::NUM) {
            const long cnt = strtol(v.s.c_str(), nullptr, 10);
            for (long i = 0; i < cnt; ++i) items.emplace_back(TV::num(std::to_string(i)), TV::num(std::to_string(i)));
          } else if (v.k != TV::MISSING) {
            throw TplError("range can't iterate over " + go_sprint(v));
          }
          if (items.empty() && n.has_else) exec(n.els, dot, sc, out);
          for (const auto& kv : items) {
            sc.emplace_back();
            if (n.pipe.has_decl) {
              if (n.pipe.names.size() == 1) sc.back()[n.pipe.names[0]] = kv.second;
              else {
                sc.back()[n.pipe.names[0]] = kv.first;
                sc.back()[n.pipe.names[1]] = kv.second;
              }
            }
            exec(n.body, kv.second, sc, out);
            sc.pop_back();
          }
          sc.pop_back();
          break;
        }
      }
    }
  }

  TV lookup(const std::string& name, Scopes& sc) {
    for (size_t i = sc.size(); i-- > 0;) {
      auto it = sc[i].find(name);
      if (it != sc[i].end()) return it->second;
    }
    throw TplError("undefined variable " + name);
  }

  TV pipe(const Pipe& p, const TV& dot, Scopes& sc) {
    TV val;
    bool first = true;
    for (const Cmd& c : p.cmds) {
      val = command(c, dot, sc, first ? nullptr : &val);
      first = false;
    }
    if (p.has_decl) {
      if (p.decl) {
        sc.back()[p.names[0]] = val;
      } else {
        bool set = false;
        for (size_t i = sc.size(); i-- > 0 && !set;) {
          auto it = sc[i].find(p.names[0]);
          if (it != sc[i].end()) { it->second = val; set = true; }
        }
        if (!set) throw TplError("undefined variable " + p.names[0]);
      }
    }
    return val;
  }

  static TV field(const TV& v, const std::string& name) {
    if (v.k == TV::MISSING) return v;
    if (v.k == TV::NIL) throw TplError("nil pointer evaluating interface {}." + name);
    if (v.k == TV::OBJ) {
      const TV* x = v.get(name);
      return x ? *x : TV::missing();
    }
    throw TplError("can't evaluate field " + name);
  }

  TV arg(const Operand& o, const TV& dot, Scopes& sc) {
    switch (o.k) {
      case Operand::LIT: return o.lit;
      case Operand::DOT: return dot;
      case Operand::VAR: return lookup(o.name, sc);
      case Operand::FIELD: {
        TV v = arg(*o.base, dot, sc);
        for (const std::string& f : o.path) v = field(v, f);
        return v;
      }
      case Operand::PAREN: return pipe(*o.pipe, dot, sc);
      case Operand::IDENT: return call(o.name, nullptr, 0, dot, sc, nullptr);
    }
    return TV();
  }

  TV call(const std::string& name, const Cmd* c, size_t from, const TV& dot, Scopes& sc, const TV* extra) {
    if (name == "and" || name == "or") {
      const bool is_or = name == "or";
      TV v;
      const size_t n = c ? c->size() : 0;
      for (size_t i = from; i < n; ++i) {
        v = arg((*c)[i], dot, sc);
        if (is_or == truth(v)) return v;
      }
      if (extra) {
        v = *extra;
        if (is_or == truth(v)) return v;
      }
      return v;
    }
    std::vector<TV> a;
    if (c)
      for (size_t i = from; i < c->size(); ++i) a.push_back(arg((*c)[i], dot, sc));
    if (extra) a.push_back(*extra);
    auto f = funcs.find(name);
    if (f != funcs.end()) return f->second(a);
    return builtin(name, a);
  }

  TV command(const Cmd& c, const TV& dot, Scopes& sc, const TV* prev) {
    const Operand& head = c[0];
    if (head.k == Operand::IDENT) return call(head.name, &c, 1, dot, sc, prev);
    if (c.size() > 1 || prev) throw TplError("can't give argument to non-function");
    return arg(head, dot, sc);
  }

  static TV builtin(const std::string& name, std::vector<TV>& a) {
    if (name == "not") {
      if (a.size() != 1) throw TplError("not: wrong number of args");
      return TV::boolean(!truth(a[0]));
    }
    if (name == "len") {
      if (a.size() != 1 || !(a[0].k == TV::STR || a[0].k == TV::NUM || a[0].k == TV::ARR || a[0].k == TV::OBJ))
        throw TplError("len of an unsupported value");
      return TV::num(std::to_string(a[0].k == TV::STR || a[0].k == TV::NUM ? utf8_len(a[0].s) : a[0].size()));
    }
    if (name == "index") {
      if (a.empty()) throw TplError("index: wrong number of args");
      TV x = a[0];
      for (size_t i = 1; i < a.size(); ++i) {
        if (x.k == TV::MISSING || x.k == TV::NIL) throw TplError("index of untyped nil");
        if (x.k == TV::OBJ) {
          const TV* y = x.get(go_sprint(a[i]));
          x = y ? *y : TV::nil();
        } else if (x.k == TV::ARR) {
          const long k = strtol(go_sprint(a[i]).c_str(), nullptr, 10);
          if (k < 0 || (size_t)k >= x.arr->size()) throw TplError("index out of range");
          x = (*x.arr)[(size_t)k];
        } else {
          throw TplError("can't index item");
        }
      }
      return x;
    }
    if (name == "eq") {
      if (a.size() < 2) throw TplError("eq: missing argument");
      return TV::boolean(tpl_eq(a[0], a, 1));
    }
    if (name == "ne") {
      if (a.size() != 2) throw TplError("ne: wrong number of args");
      return TV::boolean(!tpl_eq(a[0], a, 1));
    }
    if (name == "lt" || name == "le" || name == "gt" || name == "ge") {
      if (a.size() != 2) throw TplError(name + ": wrong number of args");
      const int ka = basic_kind(a[0]), kb = basic_kind(a[1]);
      if (ka != kb || ka != 2) throw TplError("incompatible types for comparison");
      const int c = a[0].s.compare(a[1].s);
      return TV::boolean(name == "lt" ? c < 0 : name == "le" ? c <= 0 : name == "gt" ? c > 0 : c >= 0);
    }
    if (name == "print") {
      std::string o;
      for (const TV& x : a) o += go_sprint(x);
      return TV::str(o);
    }
    if (name == "printf") {
      if (a.empty()) throw TplError("printf: missing format");
      const std::string fmt = go_sprint(a[0]);
      std::string o;
      size_t next = 1;
      for (size_t i = 0; i < fmt.size(); ++i) {
        if (fmt[i] == '%' && i + 1 < fmt.size() && strchr("%svdq", fmt[i + 1])) {
          const char verb = fmt[++i];
          if (verb == '%') { o += '%'; continue; }
          const TV x = next < a.size() ? a[next++] : TV::missing();
          if (verb == 'q') o += py_json_string(go_sprint(x));
          else o += go_sprint(x);
        } else {
          o += fmt[i];
        }
      }
      return TV::str(o);
    }
    if (name == "dict") {
      std::map<std::string, TV> m;
      for (size_t i = 0; i < a.size(); i += 2) m[go_sprint(a[i])] = i + 1 < a.size() ? a[i + 1] : TV::str("");
      return TV::dict(std::move(m));
    }
    if (name == "list") return TV::list(a);
    if (name == "default") {
      if (a.empty()) throw TplError("default: missing argument");
      const TV v = a.size() > 1 ? a[1] : TV::missing();
      return truth(v) ? v : a[0];
    }
    if (name == "hasKey") {
      if (a.size() != 2) throw TplError("hasKey: wrong number of args");
      return TV::boolean(a[0].k == TV::OBJ && a[0].get(go_sprint(a[1])) != nullptr);
    }
    throw TplError("function \"" + name + "\" not defined");
  }

  static size_t utf8_len(const std::string& s) {
    size_t n = 0, i = 0;
    uint32_t cp;
    while (i < s.size()) {
      utf8_next(s, i, cp);
      ++n;
    }
    return n;
  }
};

// ------------------------------------------------------------------ YAML subset (YAMLToJSON)
// PyYAML SafeLoader implicit resolvers (YAML 1.1), timestamps removed (gotpl._YamlLoader)
inline bool yaml_is_bool(const std::string& s, bool& v) {
  static const char* t[] = {"yes", "Yes", "YES", "true", "True", "TRUE", "on", "On", "ON"};
  static const char* f[] = {"no", "No", "NO", "false", "False", "FALSE", "off", "Off", "OFF"};
  for (const char* x : t)
    if (s == x) { v = true; return true; }
  for (const char* x : f)
    if (s == x) { v = false; return true; }
  return false;
}

inline bool all_of(const std::string& s, size_t a, size_t b, const char* set) {
  if (a >= b) return false;
  for (size_t i = a; i < b; ++i)
    if (!strchr(set, s[i])) return false;
  return true;
}

// [-+]?[1-9][0-9_]*(:[0-5]?[0-9])+ (sexagesimal tail after the first group)
inline bool sexa_tail(const std::string& s, size_t i, size_t end) {
  bool any = false;
  while (i < end) {
    if (s[i] != ':') return false;
    ++i;
    size_t j = i;
    while (j < end && is_digit(s[j]) && j - i < 2) ++j;
    if (j == i) return false;
    if (j - i == 2 && s[i] > '5') return false;
    i = j;
    any = true;
  }
  return any;
}

inline bool yaml_int_text(const std::string& s0, std::string& out) {
  // ^(?:[-+]?0b[0-1_]+|[-+]?0[0-7_]+|[-+]?(?:0|[1-9][0-9_]*)|[-+]?0x[0-9a-fA-F_]+|[-+]?[1-9][0-9_]*(?::[0-5]?[0-9])+)$
  if (s0.empty()) return false;
  size_t i = 0;
  bool neg = false;
  if (s0[0] == '-' || s0[0] == '+') { neg = s0[0] == '-'; i = 1; }
  const size_t n = s0.size();
  int base = 0;
  size_t body = i;
  if (n - i >= 3 && s0[i] == '0' && s0[i + 1] == 'b' && all_of(s0, i + 2, n, "01_")) { base = 2; body = i + 2; }
  else if (n - i >= 3 && s0[i] == '0' && s0[i + 1] == 'x' && all_of(s0, i + 2, n, "0123456789abcdefABCDEF_")) { base = 16; body = i + 2; }
  else if (n - i >= 2 && s0[i] == '0' && all_of(s0, i + 1, n, "01234567_")) { base = 8; body = i + 1; }
  else if (n - i == 1 && s0[i] == '0') { base = 10; }
  else if (n > i && s0[i] >= '1' && s0[i] <= '9') {
    size_t j = i + 1;
    while (j < n && (is_digit(s0[j]) || s0[j] == '_')) ++j;
    if (j == n) base = 10;
    else if (sexa_tail(s0, j, n)) base = 60;
    else return false;
  } else {
    return false;
  }
  // construct_yaml_int: '_' removed; sexagesimal digits base 60
  unsigned __int128 v = 0;
  if (base == 60) {
    std::vector<long> parts;
    std::string cur;
    for (size_t k = i; k <= n; ++k) {
      if (k == n || s0[k] == ':') { parts.push_back(strtol(cur.c_str(), nullptr, 10)); cur.clear(); }
      else if (s0[k] != '_') cur += s0[k];
    }
    for (long p : parts) v = v * 60 + (unsigned long)p;
  } else {
    for (size_t k = body; k < n; ++k) {
      if (s0[k] == '_') continue;
      const char c = s0[k];
      const int d = is_digit(c) ? c - '0' : (c | 32) - 'a' + 10;
      v = v * (unsigned)base + (unsigned)d;
      if (v > ((unsigned __int128)1 << 64)) throw TplError("YAML integer out of range: " + s0);
    }
  }
  if (v > ((unsigned __int128)1 << 63) || (!neg && v == ((unsigned __int128)1 << 63)))
    throw TplError("YAML integer out of int64 range: " + s0);
  char buf[32];
  snprintf(buf, sizeof buf, "%llu", (unsigned long long)v);
  out = (neg && v != 0 ? "-" : "") + std::string(buf);
  return true;
}

inline bool yaml_float(const std::string& s, double& out) {
  // ^(?:[-+]?(?:[0-9][0-9_]*)\.[0-9_]*(?:[eE][-+][0-9]+)?|\.[0-9][0-9_]*(?:[eE][-+][0-9]+)?
  //   |[-+]?[0-9][0-9_]*(?::[0-5]?[0-9])+\.[0-9_]*|[-+]?\.(?:inf|Inf|INF)|\.(?:nan|NaN|NAN))$
  const size_t n = s.size();
  if (!n) return false;
  size_t i = 0;
  bool sign = false, neg = false;
  if (s[0] == '-' || s[0] == '+') { sign = true; neg = s[0] == '-'; i = 1; }
  const std::string r = s.substr(i);
  if (r == ".inf" || r == ".Inf" || r == ".INF") { out = neg ? -INFINITY : INFINITY; return true; }
  if (!sign && (r == ".nan" || r == ".NaN" || r == ".NAN")) { out = NAN; return true; }
  auto exp_ok = [&](size_t j) {  // (?:[eE][-+][0-9]+)?$ from j
    if (j == n) return true;
    if (!(s[j] == 'e' || s[j] == 'E') || j + 2 >= n + 0 || !(s[j + 1] == '-' || s[j + 1] == '+')) return false;
    return all_of(s, j + 2, n, "0123456789");
  };
  std::string clean;
  for (char c : s)
    if (c != '_') clean += c;
  if (i < n && is_digit(s[i])) {
    size_t j = i + 1;
    while (j < n && (is_digit(s[j]) || s[j] == '_')) ++j;
    if (j < n && s[j] == '.') {
      size_t k = j + 1;
      while (k < n && (is_digit(s[k]) || s[k] == '_')) ++k;
      if (!exp_ok(k)) return false;
      out = strtod(clean.c_str(), nullptr);
      return true;
    }
    if (j < n && s[j] == ':') {  // sexagesimal float
      size_t k = j;
      while (k < n && s[k] != '.') ++k;
      if (k == n || !sexa_tail(s, j, k) || !(k + 1 == n || all_of(s, k + 1, n, "0123456789_"))) return false;
      std::vector<std::string> parts;
      std::string cur;
      for (size_t q = i; q < n; ++q) {
        if (s[q] == ':') { parts.push_back(cur); cur.clear(); }
        else if (s[q] != '_') cur += s[q];
      }
      parts.push_back(cur);
      double v = 0;
      for (const std::string& p : parts) v = v * 60 + strtod(p.c_str(), nullptr);
      out = neg ? -v : v;
      return true;
    }
    return false;
  }
  if (!sign && i < n && s[i] == '.' && i + 1 < n && is_digit(s[i + 1])) {
    size_t k = i + 2;
    while (k < n && (is_digit(s[k]) || s[k] == '_')) ++k;
    if (!exp_ok(k)) return false;
    out = strtod(clean.c_str(), nullptr);
    return true;
  }
  return false;
}

inline JV yaml_plain(const std::string& s) {
  JV v;
  bool b;
  double f;
  std::string it;
  if (s.empty() || s == "~" || s == "null" || s == "Null" || s == "NULL") { v.t = JV::NUL; return v; }
  if (yaml_is_bool(s, b)) { v.t = JV::BOOL; v.b = b; return v; }
  if (yaml_int_text(s, it)) { v.t = JV::NUM; v.is_int = true; v.s = it; return v; }
  if (yaml_float(s, f)) {
    v.t = JV::NUM;
    v.is_int = false;
    if (std::isnan(f) || std::isinf(f)) v.s = std::isnan(f) ? "NaN" : (f > 0 ? "Infinity" : "-Infinity");
    else v.s = kwkhost::py_float_repr(f);
    return v;
  }
  v.t = JV::STR;
  v.s = s;
  return v;
}

struct YamlLoader {
  struct Line {
    int indent;
    std::string c;  // content without indentation, trailing blanks or a comment
  };
  std::vector<Line> L;
  size_t i = 0;

  // a '#' starting a comment: at the content's start or after a blank, outside quotes
  static std::string strip_comment(const std::string& s) {
    char q = 0;
    for (size_t k = 0; k < s.size(); ++k) {
      const char c = s[k];
      if (q) {
        if (q == '"' && c == '\\') { ++k; continue; }
        if (c == q) {
          if (q == '\'' && k + 1 < s.size() && s[k + 1] == '\'') { ++k; continue; }
          q = 0;
        }
        continue;
      }
      if ((c == '"' || c == '\'') && (k == 0 || s[k - 1] == ' ' || s[k - 1] == '[' || s[k - 1] == '{' ||
                                      s[k - 1] == ',' || s[k - 1] == ':' || s[k - 1] == '-')) {
        q = c;
        continue;
      }
      if (c == '#' && (k == 0 || s[k - 1] == ' ' || s[k - 1] == '\t')) return s.substr(0, k);
    }
    return s;
  }

  explicit YamlLoader(const std::string& text) {
    size_t p = 0;
    while (p <= text.size()) {
      size_t e = text.find('\n', p);
      if (e == std::string::npos) e = text.size();
      std::string line = text.substr(p, e - p);
      if (!line.empty() && line.back() == '\r') line.pop_back();
      int ind = 0;
      while ((size_t)ind < line.size() && line[(size_t)ind] == ' ') ++ind;
      std::string c = line.substr((size_t)ind);
      if (!c.empty() && c[0] == '\t') throw TplError("YAML: tab indentation");
      c = py_rstrip(strip_comment(c));
      if (!c.empty()) {
        if (c == "---" || c == "..." || c.rfind("--- ", 0) == 0 || c[0] == '%')
          throw TplError("YAML: document markers / directives are not supported");
        L.push_back({ind, c});
      }
      p = e + 1;
    }
  }

  static bool is_seq(const std::string& c) { return c == "-" || c.rfind("- ", 0) == 0; }

  // the key of a mapping line ("key: ..." / "key:"): returns the position after ':' or npos
  static size_t key_end(const std::string& c, std::string& key) {
    if (c.empty()) return std::string::npos;
    if (c[0] == '"' || c[0] == '\'') {
      size_t k = 1;
      const char q = c[0];
      for (; k < c.size(); ++k) {
        if (q == '"' && c[k] == '\\') { ++k; continue; }
        if (c[k] == q) {
          if (q == '\'' && k + 1 < c.size() && c[k + 1] == '\'') { ++k; continue; }
          break;
        }
      }
      if (k >= c.size()) return std::string::npos;
      size_t j = k + 1;
      while (j < c.size() && c[j] == ' ') ++j;
      if (j < c.size() && c[j] == ':' && (j + 1 == c.size() || c[j + 1] == ' ')) {
        key = quoted(c.substr(0, k + 1));
        return j + 1;
      }
      return std::string::npos;
    }
    if (strchr("-?:,[]{}#&*!|>'\"%@`", c[0]) && !(c[0] == '-' && c.size() > 1 && c[1] != ' ')) return std::string::npos;
    for (size_t k = 0; k < c.size(); ++k) {
      if (c[k] == ':' && (k + 1 == c.size() || c[k + 1] == ' ')) {
        key = py_rstrip(c.substr(0, k));
        return k + 1;
      }
    }
    return std::string::npos;
  }

  static std::string quoted(const std::string& s) {
    std::string o;
    if (s[0] == '\'') {
      for (size_t k = 1; k + 1 < s.size(); ++k) {
        if (s[k] == '\'' && s[k + 1] == '\'') { o += '\''; ++k; }
        else o += s[k];
      }
      return o;
    }
    for (size_t k = 1; k + 1 < s.size(); ++k) {
      if (s[k] != '\\') { o += s[k]; continue; }
      const char x = s[++k];
      uint32_t cp = 0;
      int hex = 0;
      switch (x) {
        case '0': o += '\0'; break;
        case 'a': o += '\a'; break;
        case 'b': o += '\b'; break;
        case 't': case '\t': o += '\t'; break;
        case 'n': o += '\n'; break;
        case 'v': o += '\v'; break;
        case 'f': o += '\f'; break;
        case 'r': o += '\r'; break;
        case 'e': o += '\x1b'; break;
        case ' ': o += ' '; break;
        case '"': o += '"'; break;
        case '/': o += '/'; break;
        case '\\': o += '\\'; break;
        case 'N': utf8_put(o, 0x85); break;
        case '_': utf8_put(o, 0xA0); break;
        case 'L': utf8_put(o, 0x2028); break;
        case 'P': utf8_put(o, 0x2029); break;
        case 'x': hex = 2; break;
        case 'u': hex = 4; break;
        case 'U': hex = 8; break;
        default: throw TplError("YAML: unknown escape");
      }
      if (hex) {
        for (int h = 0; h < hex; ++h) {
          const char d = s[++k];
          cp = cp * 16 + (uint32_t)(is_digit(d) ? d - '0' : (d | 32) - 'a' + 10);
        }
        utf8_put(o, cp);
      }
    }
    return o;
  }

  // a complete scalar / flow value on one line
  static JV scalar(const std::string& c) {
    JV v;
    if (c.empty()) { v.t = JV::NUL; return v; }
    if (c[0] == '"' || c[0] == '\'') {
      std::string key;
      // the quote must close at the end of the content
      size_t k = 1;
      const char q = c[0];
      for (; k < c.size(); ++k) {
        if (q == '"' && c[k] == '\\') { ++k; continue; }
        if (c[k] == q) {
          if (q == '\'' && k + 1 < c.size() && c[k + 1] == '\'') { ++k; continue; }
          break;
        }
      }
      if (k != c.size() - 1) throw TplError("YAML: content after a quoted scalar");
      v.t = JV::STR;
      v.s = quoted(c);
      return v;
    }
    if (c[0] == '[' || c[0] == '{') {
      size_t p = 0;
      v = flow(c, p);
      while (p < c.size() && c[p] == ' ') ++p;
      if (p != c.size()) throw TplError("YAML: content after a flow collection");
      return v;
    }
    if (strchr("&*!|>%@`", c[0])) throw TplError("YAML: anchors, tags and block scalars are not supported");
    if (c.find(": ") != std::string::npos || c.back() == ':') throw TplError("YAML: mapping values are not allowed here");
    return yaml_plain(c);
  }

  // flow collections ([a, "b", {k: v}]) on one line
  static JV flow(const std::string& c, size_t& p) {
    auto ws = [&]() { while (p < c.size() && c[p] == ' ') ++p; };
    JV v;
    const char open = c[p];
    if (open == '[' || open == '{') {
      const char close = open == '[' ? ']' : '}';
      v.t = open == '[' ? JV::ARR : JV::OBJ;
      ++p;
      ws();
      if (p < c.size() && c[p] == close) { ++p; return v; }
      for (;;) {
        ws();
        if (v.t == JV::OBJ) {
          JV k = flow_item(c, p, true);
          ws();
          if (p >= c.size() || c[p] != ':') throw TplError("YAML: flow mapping without ':'");
          ++p;
          ws();
          JV val = (p < c.size() && (c[p] == ',' || c[p] == '}')) ? JV() : flow(c, p);
          if (k.t != JV::STR) {  // keys are strings in JSON (sigs.k8s.io/yaml)
            std::string t;
            go_json_bytes(t, k);
            k.t = JV::STR;
            k.s = t;
          }
          v.k.push_back(k.s);
          v.a.push_back(std::move(val));
        } else {
          v.a.push_back(flow(c, p));
        }
        ws();
        if (p < c.size() && c[p] == ',') { ++p; ws(); if (p < c.size() && c[p] == close) { ++p; return v; } continue; }
        if (p < c.size() && c[p] == close) { ++p; return v; }
        throw TplError("YAML: bad flow collection");
      }
    }
    return flow_item(c, p, false);
  }
  static JV flow_item(const std::string& c, size_t& p, bool key) {
    if (p < c.size() && (c[p] == '[' || c[p] == '{')) return flow(c, p);
    if (p < c.size() && (c[p] == '"' || c[p] == '\'')) {
      const char q = c[p];
      size_t k = p + 1;
      for (; k < c.size(); ++k) {
        if (q == '"' && c[k] == '\\') { ++k; continue; }
        if (c[k] == q) {
          if (q == '\'' && k + 1 < c.size() && c[k + 1] == '\'') { ++k; continue; }
          break;
        }
      }
      if (k >= c.size()) throw TplError("YAML: unterminated quoted scalar");
      JV v;
      v.t = JV::STR;
      v.s = quoted(c.substr(p, k + 1 - p));
      p = k + 1;
      return v;
    }
    size_t e = p;
    while (e < c.size() && c[e] != ',' && c[e] != ']' && c[e] != '}' && !(c[e] == ':' && (e + 1 == c.size() || c[e + 1] == ' ' || key)))
      ++e;
    const std::string s = py_rstrip(c.substr(p, e - p));
    p = e;
    return yaml_plain(s);
  }

  JV node(int indent) {
    if (i >= L.size()) { JV v; return v; }
    Line& ln = L[i];
    if (ln.indent < indent) { JV v; return v; }
    if (is_seq(ln.c)) return seq(ln.indent);
    std::string key;
    if (key_end(ln.c, key) != std::string::npos) return map(ln.indent);
    ++i;
    if (i < L.size() && L[i].indent > ln.indent) throw TplError("YAML: multi-line scalars are not supported");
    return scalar(ln.c);
  }

  JV value_after_key(int indent, const std::string& rest) {
    if (!rest.empty()) {
      ++i;
      if (i < L.size() && L[i].indent > indent) throw TplError("YAML: multi-line scalars are not supported");
      return scalar(rest);
    }
    ++i;
    if (i < L.size() && L[i].indent > indent) return node(L[i].indent);
    if (i < L.size() && L[i].indent == indent && is_seq(L[i].c)) return seq(indent);
    JV v;
    return v;
  }

  JV map(int indent) {
    JV v;
    v.t = JV::OBJ;
    while (i < L.size() && L[i].indent == indent && !is_seq(L[i].c)) {
      std::string key;
      const size_t e = key_end(L[i].c, key);
      if (e == std::string::npos) throw TplError("YAML: expected a mapping entry: " + L[i].c);
      const std::string rest = py_strip(L[i].c.substr(e));
      JV val = value_after_key(indent, rest);
      bool dup = false;
      for (size_t k = 0; k < v.k.size(); ++k)
        if (v.k[k] == key) { v.a[k] = val; dup = true; }
      if (!dup) {
        v.k.push_back(key);
        v.a.push_back(std::move(val));
      }
    }
    if (i < L.size() && L[i].indent > indent) throw TplError("YAML: bad indentation of a mapping entry");
    return v;
  }

  JV seq(int indent) {
    JV v;
    v.t = JV::ARR;
    while (i < L.size() && L[i].indent == indent && is_seq(L[i].c)) {
      const std::string rest = L[i].c.size() > 1 ? L[i].c.substr(2) : "";
      size_t sp = 0;
      while (sp < rest.size() && rest[sp] == ' ') ++sp;
      const std::string r = rest.substr(sp);
      if (r.empty()) {
        ++i;
        if (i < L.size() && L[i].indent > indent) v.a.push_back(node(L[i].indent));
        else v.a.emplace_back();
        continue;
      }
      std::string key;
      if (is_seq(r) || key_end(r, key) != std::string::npos) {
        // the item's block starts on this line, at the column after "- "
        L[i].indent = indent + 2 + (int)sp;
        L[i].c = r;
        v.a.push_back(node(L[i].indent));
        continue;
      }
      ++i;
      if (i < L.size() && L[i].indent > indent) throw TplError("YAML: multi-line scalars are not supported");
      v.a.push_back(scalar(r));
    }
    if (i < L.size() && L[i].indent > indent) throw TplError("YAML: bad indentation of a sequence entry");
    return v;
  }

  JV load() {
    if (L.empty()) { JV v; return v; }
    JV v = node(L[0].indent);
    if (i != L.size()) throw TplError("YAML: content after the document's root node");
    return v;
  }
};

inline JV yaml_to_json(const std::string& text) { return YamlLoader(text).load(); }

}  // namespace kwktpl
