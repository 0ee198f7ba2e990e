// CEL subset of kwok's Metric values, natively: parser, constant folding and the lowering of a
// value expression to the postfix device program metrics_kernel / histogram_kernel run
// (include/kwok_engine.h: kwk_metric_op).  The C++ restatement of kwok_amd/host/cel.py (parse,
// Evaluator over constants, lower), byte-equal to it on every expression the tests feed both
// (tests/test_metric_compiler.py).
//
// Reference: pkg/kwok/metrics/evaluator.go:51-144 (the environment: node / pod / container
// variables, Usage / CumulativeUsage / StartedContainersTotal methods bound to the usage
// callbacks), pkg/utils/cel/environment.go:98-138 (Compile, AsFloat64), funcs.go (Now,
// SinceSecond, UnixSecond, Quantity), quantity.go:48-201 (Quantity arithmetic incl. the
// Quantity x double rule newQuantityFromFloat64: int64(v * 10e9) nano).  cel-go v0.17.8 itself
// is a dependency absent from /root/reference: its typing rules (no implicit int <-> double
// arithmetic, checked int64 / uint64 overflow, heterogeneous numeric equality, error-absorbing
// && / ||) are restated as cel.py states them.
//
// What lowers: double arithmetic (+ - * / and unary -) over the per-series inputs KWK_MIN_*
// (usage / cumulative usage of the series' node, pod or container, SinceSecond, UnixSecond of
// Now() or a creationTimestamp, StartedContainersTotal) and constants; a sub-expression that does
// not depend on the series is folded on the host with CEL's semantics.  Anything else has no
// device form (LowerError): the host evaluates that metric per series.
//
// Quantities hold int64Amount-style {value, scale} in __int128 (cel.py uses unbounded Python
// ints): a constant whose exact value leaves the 128-bit range is a compile error here.
#pragma once
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace kwkcel {

typedef __int128 i128;

struct SyntaxError : std::runtime_error { using std::runtime_error::runtime_error; };
struct CELError : std::runtime_error { using std::runtime_error::runtime_error; };
struct LowerError : std::runtime_error { using std::runtime_error::runtime_error; };

constexpr int64_t kI64Min = INT64_MIN, kI64Max = INT64_MAX;

// ------------------------------------------------------------------ Go math.Pow10 (quantity.py)
inline double go_pow10(int64_t n) {
  static double tab[32], pos32[10], neg32[11];
  static bool init = false;
  if (!init) {
    char b[16];
    for (int i = 0; i < 32; ++i) { snprintf(b, sizeof b, "1e%d", i); tab[i] = strtod(b, nullptr); }
    for (int i = 0; i < 10; ++i) { snprintf(b, sizeof b, "1e%d", 32 * i); pos32[i] = strtod(b, nullptr); }
    for (int i = 0; i < 11; ++i) { snprintf(b, sizeof b, "1e-%d", 32 * i); neg32[i] = strtod(b, nullptr); }
    init = true;
  }
  if (0 <= n && n <= 308) return pos32[n / 32] * tab[n % 32];
  if (-323 <= n && n <= 0) return neg32[(-n) / 32] / tab[(-n) % 32];
  return n > 0 ? HUGE_VAL : 0.0;
}

// ------------------------------------------------------------------ 128-bit helpers
inline i128 pow10_128(int k) {
  if (k < 0 || k > 38) throw CELError("quantity out of the 128-bit range");
  i128 r = 1;
  for (int i = 0; i < k; ++i) r *= 10;
  return r;
}
inline i128 mul_chk(i128 a, i128 b) {
  i128 r;
  if (__builtin_mul_overflow(a, b, &r)) throw CELError("quantity out of the 128-bit range");
  return r;
}
inline i128 add_chk(i128 a, i128 b) {
  i128 r;
  if (__builtin_add_overflow(a, b, &r)) throw CELError("quantity out of the 128-bit range");
  return r;
}
inline i128 ceil_div(i128 a, i128 d) {  // d > 0: Python -((-a) // d)
  i128 q = a / d;
  if (a % d != 0 && a > 0) ++q;
  return q;
}
inline double i128_to_double(i128 v) { return (double)v; }  // round to nearest even (libgcc __floattidf)
inline std::string i128_str(i128 v) {
  if (v == 0) return "0";
  bool neg = v < 0;
  unsigned __int128 u = neg ? (unsigned __int128)(-(v + 1)) + 1 : (unsigned __int128)v;
  std::string s;
  while (u) { s += (char)('0' + (int)(u % 10)); u /= 10; }
  if (neg) s += '-';
  return std::string(s.rbegin(), s.rend());
}

// ------------------------------------------------------------------ Quantity (cel.py Quantity)
struct Quantity {
  i128 value = 0;
  int64_t scale = 0;
  static Quantity nano(i128 v) { return Quantity{v, -9}; }
  i128 scaled_nano() const {  // ScaledValue(Nano): ceil(q / 1e-9)
    if (scale >= -9) return mul_chk(value, pow10_128((int)(scale + 9)));
    return ceil_div(value, pow10_128((int)(-9 - scale)));
  }
  double approx() const {  // AsApproximateFloat64
    if (scale == 0) return i128_to_double(value);
    return i128_to_double(value) * go_pow10(scale);
  }
  void aligned(const Quantity& o, i128& a, i128& b, int64_t& s) const {
    s = std::min(scale, o.scale);
    a = mul_chk(value, pow10_128((int)(scale - s)));
    b = mul_chk(o.value, pow10_128((int)(o.scale - s)));
  }
  int cmp(const Quantity& o) const {
    i128 a, b;
    int64_t s;
    aligned(o, a, b, s);
    return (a > b) - (a < b);
  }
};

// apimachinery ParseQuantity's grammar (quantity.py parse_quantity_f64: which strings fail)
struct QtyParts { bool positive = true; std::string value, num, denom, suffix; };
inline bool isdig(char c) { return c >= '0' && c <= '9'; }

inline QtyParts parse_quantity_string(const std::string& s) {
  QtyParts r;
  size_t pos = 0, end = s.size();
  if (pos < end) {
    if (s[0] == '-') { r.positive = false; ++pos; }
    else if (s[0] == '+') ++pos;
  }
  size_t i = pos;
  for (;;) {  // leading zeros
    if (i >= end) { r.value = "0"; r.num = "0"; return r; }
    if (s[i] == '0') { ++pos; ++i; } else break;
  }
  i = pos;
  for (;;) {
    if (i >= end) { r.value = s.substr(0, end); r.num = s.substr(pos, end - pos); return r; }
    if (isdig(s[i])) { ++i; continue; }
    r.num = s.substr(pos, i - pos);
    pos = i;
    break;
  }
  if (r.num.empty()) r.num = "0";
  if (pos < end && s[pos] == '.') {
    ++pos;
    i = pos;
    for (;;) {
      if (i >= end) { r.value = s.substr(0, end); r.denom = s.substr(pos, end - pos); return r; }
      if (isdig(s[i])) { ++i; continue; }
      r.denom = s.substr(pos, i - pos);
      pos = i;
      break;
    }
  }
  r.value = s.substr(0, pos);
  const size_t suffix_start = pos;
  i = pos;
  for (;;) {
    if (i >= end) { r.suffix = s.substr(suffix_start); return r; }
    if (!strchr("eEinumkKMGTP", s[i])) { pos = i; break; }
    ++i;
  }
  if (pos < end && (s[pos] == '-' || s[pos] == '+')) ++pos;
  i = pos;
  for (;;) {
    if (i >= end) { r.suffix = s.substr(suffix_start); return r; }
    if (isdig(s[i])) { ++i; continue; }
    throw CELError("quantities must match the regular expression");
  }
}

struct Suffix { int base; int64_t exp; int fmt; };  // fmt 0 DecimalSI, 1 BinarySI, 2 DecimalExponent
inline Suffix interpret_suffix(const std::string& suf) {
  static const char* dec[] = {"n", "u", "m", "", "k", "M", "G", "T", "P", "E"};
  static const int dexp[] = {-9, -6, -3, 0, 3, 6, 9, 12, 15, 18};
  static const char* bin[] = {"Ki", "Mi", "Gi", "Ti", "Pi", "Ei"};
  for (int i = 0; i < 10; ++i) if (suf == dec[i]) return {10, dexp[i], 0};
  for (int i = 0; i < 6; ++i) if (suf == bin[i]) return {2, 10 * (i + 1), 1};
  if (suf.size() > 1 && (suf[0] == 'e' || suf[0] == 'E')) {
    const std::string body = suf.substr(1);
    bool ok = !body.empty();
    for (size_t k = 0; k < body.size() && ok; ++k) {
      const char c = body[k];
      if (!(isdig(c) || c == '+' || c == '-')) ok = false;
      if (k > 0 && (c == '+' || c == '-')) ok = false;
    }
    if (ok && (body == "+" || body == "-")) ok = false;
    if (!ok) throw CELError("unable to parse quantity's suffix");
    // int(body) within int64, then int32(parsed)
    i128 e = 0;
    size_t k = (body[0] == '+' || body[0] == '-') ? 1 : 0;
    for (; k < body.size(); ++k) {
      e = e * 10 + (body[k] - '0');
      if (e > ((i128)1 << 64)) throw CELError("unable to parse quantity's suffix");
    }
    if (body[0] == '-') e = -e;
    if (e < (i128)kI64Min || e > (i128)kI64Max) throw CELError("unable to parse quantity's suffix");
    const int64_t w = (int64_t)(int32_t)(uint32_t)(uint64_t)(int64_t)e;
    return {10, w, 2};
  }
  throw CELError("unable to parse quantity's suffix");
}

// Python Fraction(value) acceptance for the inf.Dec path's value text ([sign] digits [. digits])
inline bool fraction_ok(const std::string& v) {
  size_t i = 0;
  if (i < v.size() && (v[i] == '+' || v[i] == '-')) ++i;
  if (i >= v.size()) return false;
  if (!(isdig(v[i]) || (v[i] == '.' && i + 1 < v.size() && isdig(v[i + 1])))) return false;
  return true;
}

// ParseQuantity's failures (parse_quantity_f64 raising), nothing else
inline void validate_quantity(const std::string& s) {
  if (s.empty()) throw CELError("quantities must match the regular expression");
  if (s == "0") return;
  const QtyParts p = parse_quantity_string(s);
  const Suffix sf = interpret_suffix(p.suffix);
  int64_t precision = 0, scale = 0;
  if (sf.fmt == 2 || sf.fmt == 0) {
    scale = sf.exp;
    precision = 18 - (int64_t)(p.num.size() + p.denom.size());
  } else {
    if (sf.exp >= 0 && p.denom.empty()) {
      const float e32 = (float)sf.exp;
      precision = 15 - (int64_t)p.num.size() - (int64_t)(int32_t)(e32 * 3.0f / 10.0f) - 1;
    } else {
      precision = -1;
    }
  }
  if (precision >= 0) {
    scale -= (int64_t)p.denom.size();
    if (scale >= -9) return;  // int64Amount: at most 18 digits, never above INT64_MAX
  }
  if (p.value.empty() || p.value == "+" || p.value == "-" || !fraction_ok(p.value))
    throw CELError("quantities must match the regular expression");
}

inline Quantity quantity_parse(const std::string& s) {
  validate_quantity(s);
  // Quantity._exact: ([+-]?)(\d*)(?:\.(\d*))?(.*)
  size_t i = 0;
  bool neg = false;
  if (i < s.size() && (s[i] == '+' || s[i] == '-')) { neg = s[i] == '-'; ++i; }
  const size_t n0 = i;
  while (i < s.size() && isdig(s[i])) ++i;
  std::string num = s.substr(n0, i - n0);
  std::string frac;
  if (i < s.size() && s[i] == '.') {
    const size_t f0 = ++i;
    while (i < s.size() && isdig(s[i])) ++i;
    frac = s.substr(f0, i - f0);
  }
  const Suffix sf = interpret_suffix(s.substr(i));
  const std::string digits = num + frac;
  i128 v = 0;
  for (char c : digits) v = add_chk(mul_chk(v, 10), c - '0');
  if (neg) v = -v;
  Quantity q;
  if (sf.base == 10) {
    q = Quantity{v, sf.exp - (int64_t)frac.size()};
  } else {
    // Fraction(v, 10^len(frac)) * 2^exp: integral -> {x, 0}, else ceil(x * 1e9) nano
    const i128 den = pow10_128((int)frac.size());
    if (sf.exp > 100) throw CELError("quantity out of the 128-bit range");
    const i128 numr = mul_chk(v, (i128)1 << sf.exp);
    if (numr % den == 0) q = Quantity{numr / den, 0};
    else q = Quantity{ceil_div(mul_chk(numr, pow10_128(9)), den), -9};
  }
  if (q.scale < -9) q = Quantity{ceil_div(q.value, pow10_128((int)(-9 - q.scale))), -9};
  return q;
}

// newQuantityFromFloat64 (quantity.go:69-72): int64(v * 10e9) nano
inline Quantity quantity_from_float(double v) {
  const double x = v * 10e9;
  if (!(x >= -9.223372036854776e18 && x < 9.223372036854776e18)) return Quantity::nano(kI64Min);
  return Quantity::nano((i128)(int64_t)x);
}

// ------------------------------------------------------------------ values (constants only)
struct Value;
typedef std::shared_ptr<const Value> VP;
struct Value {
  enum T { NUL, BOOL, INT, UINT, DBL, STR, LIST, MAP, QTY } t = NUL;
  bool b = false;
  int64_t i = 0;
  uint64_t u = 0;
  double d = 0;
  std::string s;
  std::vector<Value> list;                      // LIST items
  std::vector<std::pair<Value, Value>> map;     // MAP entries (insertion order, Python dict)
  Quantity q;
};
inline Value vnull() { return Value(); }
inline Value vbool(bool x) { Value v; v.t = Value::BOOL; v.b = x; return v; }
inline Value vint(int64_t x) { Value v; v.t = Value::INT; v.i = x; return v; }
inline Value vuint(uint64_t x) { Value v; v.t = Value::UINT; v.u = x; return v; }
inline Value vdbl(double x) { Value v; v.t = Value::DBL; v.d = x; return v; }
inline Value vstr(std::string x) { Value v; v.t = Value::STR; v.s = std::move(x); return v; }
inline Value vqty(Quantity x) { Value v; v.t = Value::QTY; v.q = x; return v; }

inline const char* type_name(const Value& v) {
  switch (v.t) {
    case Value::NUL: return "null_type";
    case Value::BOOL: return "bool";
    case Value::INT: return "int";
    case Value::UINT: return "uint";
    case Value::DBL: return "double";
    case Value::STR: return "string";
    case Value::LIST: return "list";
    case Value::MAP: return "map";
    case Value::QTY: return "kubernetes.Quantity";
  }
  return "?";
}
inline bool is_intlike(const Value& v) { return v.t == Value::INT || v.t == Value::UINT; }  // Python int (not bool)
inline bool is_pynum(const Value& v) { return v.t == Value::BOOL || is_intlike(v) || v.t == Value::DBL; }
inline i128 as_i128(const Value& v) {
  return v.t == Value::BOOL ? (i128)v.b : v.t == Value::INT ? (i128)v.i : (i128)v.u;
}
inline double as_dbl(const Value& v) {
  return v.t == Value::DBL ? v.d : v.t == Value::INT ? (double)v.i : v.t == Value::UINT ? (double)v.u : (v.b ? 1.0 : 0.0);
}

// Python's == (dict keys, list / dict equality): bool / int / float numerically, str, None,
// lists and dicts structurally, Quantity only with Quantity (Quantity.__eq__)
inline bool py_eq(const Value& a, const Value& b) {
  if (is_pynum(a) && is_pynum(b)) {
    if (a.t == Value::DBL || b.t == Value::DBL) {
      if (a.t == Value::DBL && b.t == Value::DBL) return a.d == b.d;
      const Value& f = a.t == Value::DBL ? a : b;
      const Value& n = a.t == Value::DBL ? b : a;
      if (std::isnan(f.d) || std::isinf(f.d)) return false;
      if (f.d != std::floor(f.d)) return false;
      if (std::fabs(f.d) >= 1.7e38) return false;
      return (i128)f.d == as_i128(n);  // Python compares int / float exactly
    }
    return as_i128(a) == as_i128(b);
  }
  if (a.t != b.t) return false;
  switch (a.t) {
    case Value::NUL: return true;
    case Value::STR: return a.s == b.s;
    case Value::QTY: return a.q.cmp(b.q) == 0;
    case Value::LIST:
      if (a.list.size() != b.list.size()) return false;
      for (size_t k = 0; k < a.list.size(); ++k) if (!py_eq(a.list[k], b.list[k])) return false;
      return true;
    case Value::MAP: {
      if (a.map.size() != b.map.size()) return false;
      for (const auto& e : a.map) {
        bool found = false;
        for (const auto& f : b.map)
          if (py_eq(e.first, f.first)) { found = py_eq(e.second, f.second); break; }
        if (!found) return false;
      }
      return true;
    }
    default: return false;
  }
}
inline void check_hashable(const Value& k) {
  if (k.t == Value::LIST || k.t == Value::MAP) throw CELError("unhashable map key");
}
inline const Value* map_find(const Value& m, const Value& k) {
  check_hashable(k);
  for (const auto& e : m.map) if (py_eq(e.first, k)) return &e.second;
  return nullptr;
}

// ------------------------------------------------------------------ lexer (cel.py _TOK order)
enum TokKind { TK_FLOAT, TK_HEX, TK_INT, TK_STR, TK_OP, TK_IDENT, TK_EOF };
struct Tok { TokKind k; std::string s; };

inline bool isws(unsigned char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\f' || c == '\v'; }
inline bool isident0(char c) { return (c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z') || c == '_'; }
inline bool ishex(char c) { return isdig(c) || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F'); }

inline size_t match_float(const std::string& s, size_t i) {
  const size_t n = s.size();
  size_t j = i;
  // (?:\d+\.\d*|\.\d+)(?:[eE][+-]?\d+)?
  size_t k = j;
  while (k < n && isdig(s[k])) ++k;
  bool mant = false;
  if (k > j && k < n && s[k] == '.') {
    ++k;
    while (k < n && isdig(s[k])) ++k;
    mant = true;
  } else if (k == j && k < n && s[k] == '.' && k + 1 < n && isdig(s[k + 1])) {
    ++k;
    while (k < n && isdig(s[k])) ++k;
    mant = true;
  }
  auto expo = [&](size_t p) -> size_t {  // [eE][+-]?\d+ at p, or 0 chars
    if (p < n && (s[p] == 'e' || s[p] == 'E')) {
      size_t q = p + 1;
      if (q < n && (s[q] == '+' || s[q] == '-')) ++q;
      const size_t d0 = q;
      while (q < n && isdig(s[q])) ++q;
      if (q > d0) return q - p;
    }
    return 0;
  };
  if (mant) return k + expo(k) - i;
  // \d+[eE][+-]?\d+
  k = j;
  while (k < n && isdig(s[k])) ++k;
  if (k > j) {
    const size_t e = expo(k);
    if (e) return k + e - i;
  }
  return 0;
}

inline std::vector<Tok> lex(const std::string& src) {
  std::vector<Tok> out;
  size_t i = 0;
  const size_t n = src.size();
  static const char* two[] = {"==", "!=", "<=", ">=", "&&", "||"};
  while (i < n) {
    const char c = src[i];
    if (isws((unsigned char)c)) { ++i; continue; }
    if (size_t m = match_float(src, i)) { out.push_back({TK_FLOAT, src.substr(i, m)}); i += m; continue; }
    if (c == '0' && i + 2 < n + 1 && i + 1 < n && (src[i + 1] == 'x' || src[i + 1] == 'X') && i + 2 < n && ishex(src[i + 2])) {
      size_t k = i + 2;
      while (k < n && ishex(src[k])) ++k;
      if (k < n && (src[k] == 'u' || src[k] == 'U')) ++k;
      out.push_back({TK_HEX, src.substr(i, k - i)});
      i = k;
      continue;
    }
    if (isdig(c)) {
      size_t k = i;
      while (k < n && isdig(src[k])) ++k;
      if (k < n && (src[k] == 'u' || src[k] == 'U')) ++k;
      out.push_back({TK_INT, src.substr(i, k - i)});
      i = k;
      continue;
    }
    {  // [rR]?("..."|'...'), no raw newline, backslash escapes any char but newline
      size_t k = i;
      if ((src[k] == 'r' || src[k] == 'R') && k + 1 < n && (src[k + 1] == '"' || src[k + 1] == '\'')) ++k;
      if (k < n && (src[k] == '"' || src[k] == '\'')) {
        const char q = src[k];
        size_t p = k + 1;
        bool ok = false;
        while (p < n) {
          if (src[p] == q) { ok = true; break; }
          if (src[p] == '\n') break;
          if (src[p] == '\\') {
            if (p + 1 >= n || src[p + 1] == '\n') break;
            p += 2;
            continue;
          }
          ++p;
        }
        if (ok) {
          out.push_back({TK_STR, src.substr(i, p + 1 - i)});
          i = p + 1;
          continue;
        }
        if (k == i) throw SyntaxError(std::string("unexpected character '") + c + "' at " + std::to_string(i));
        // r / R followed by an unterminated string: the ident alternative takes the r
      }
    }
    bool two_op = false;
    for (const char* t : two)
      if (i + 1 < n && src[i] == t[0] && src[i + 1] == t[1]) {
        out.push_back({TK_OP, std::string(t)});
        i += 2;
        two_op = true;
        break;
      }
    if (two_op) continue;
    if (strchr("-+*/%!<>?:.,[](){}", c) && c != '\0') {
      out.push_back({TK_OP, std::string(1, c)});
      ++i;
      continue;
    }
    if (isident0(c)) {
      size_t k = i;
      while (k < n && (isident0(src[k]) || isdig(src[k]))) ++k;
      out.push_back({TK_IDENT, src.substr(i, k - i)});
      i = k;
      continue;
    }
    throw SyntaxError(std::string("unexpected character at ") + std::to_string(i));
  }
  out.push_back({TK_EOF, ""});
  return out;
}

inline void utf8_append(std::string& o, uint32_t c) {
  if (c < 0x80) o += (char)c;
  else if (c < 0x800) { o += (char)(0xC0 | (c >> 6)); o += (char)(0x80 | (c & 0x3F)); }
  else if (c < 0x10000) { o += (char)(0xE0 | (c >> 12)); o += (char)(0x80 | ((c >> 6) & 0x3F)); o += (char)(0x80 | (c & 0x3F)); }
  else { o += (char)(0xF0 | (c >> 18)); o += (char)(0x80 | ((c >> 12) & 0x3F)); o += (char)(0x80 | ((c >> 6) & 0x3F)); o += (char)(0x80 | (c & 0x3F)); }
}

inline std::string unescape(const std::string& tok) {
  const bool raw = tok[0] == 'r' || tok[0] == 'R';
  const std::string body = raw ? tok.substr(2, tok.size() - 3) : tok.substr(1, tok.size() - 2);
  if (raw) return body;
  std::string out;
  size_t i = 0;
  auto hexval = [&](size_t a, size_t len, int base) -> uint32_t {
    if (a + len > body.size()) throw SyntaxError("bad escape");
    uint32_t v = 0;
    for (size_t k = a; k < a + len; ++k) {
      const char c = body[k];
      int d = isdig(c) ? c - '0' : (c >= 'a' && c <= 'f') ? c - 'a' + 10 : (c >= 'A' && c <= 'F') ? c - 'A' + 10 : 99;
      if (d >= base) throw SyntaxError("bad escape");
      v = v * base + d;
    }
    return v;
  };
  while (i < body.size()) {
    const char c = body[i];
    if (c != '\\') { out += c; ++i; continue; }
    const char x = body[i + 1];
    switch (x) {
      case 'n': out += '\n'; i += 2; continue;
      case 't': out += '\t'; i += 2; continue;
      case 'r': out += '\r'; i += 2; continue;
      case '\\': out += '\\'; i += 2; continue;
      case '"': out += '"'; i += 2; continue;
      case '\'': out += '\''; i += 2; continue;
      case 'a': out += '\a'; i += 2; continue;
      case 'b': out += '\b'; i += 2; continue;
      case 'f': out += '\f'; i += 2; continue;
      case 'v': out += '\v'; i += 2; continue;
      case '`': out += '`'; i += 2; continue;
      case '?': out += '?'; i += 2; continue;
      case 'x': case 'X': utf8_append(out, hexval(i + 2, 2, 16)); i += 4; continue;
      case 'u': utf8_append(out, hexval(i + 2, 4, 16)); i += 6; continue;
      case 'U': {
        const uint32_t v = hexval(i + 2, 8, 16);
        if (v > 0x10FFFF) throw SyntaxError("bad escape");
        utf8_append(out, v);
        i += 10;
        continue;
      }
      default: utf8_append(out, hexval(i + 1, 3, 8)); i += 4; continue;
    }
  }
  return out;
}

// ------------------------------------------------------------------ AST and parser (cel.py _Parser)
struct Node;
typedef std::shared_ptr<Node> NP;
struct Node {
  enum K { LIT, IDENT, SELECT, INDEX, CALL, METHOD, UNARY, BINARY, COND, LIST, MAP } k;
  Value lit;                 // LIT
  std::string name;          // IDENT name, SELECT field, CALL / METHOD name, UNARY / BINARY op
  std::vector<NP> kids;      // SELECT/INDEX/METHOD target first, then args / operands / items
  std::vector<std::pair<NP, NP>> entries;  // MAP
};
inline NP mk(Node::K k) { auto n = std::make_shared<Node>(); n->k = k; return n; }

struct Parser {
  std::vector<Tok> t;
  size_t i = 0;
  explicit Parser(const std::string& src) : t(lex(src)) {}
  const Tok& cur() const {
    if (i >= t.size()) throw SyntaxError("unexpected end of expression");
    return t[i];
  }
  bool peek_is(const char* v) const {
    const Tok& x = cur();
    return x.s == v && (x.k == TK_OP || x.k == TK_IDENT);
  }
  bool peek_op(const char* v) const { const Tok& x = cur(); return x.s == v && x.k == TK_OP; }
  Tok eat() { Tok x = cur(); ++i; return x; }
  Tok eat(const char* v) {
    const Tok& x = cur();
    if (x.s != v) throw SyntaxError(std::string("expected '") + v + "', got '" + x.s + "'");
    ++i;
    return x;
  }
  NP parse() {
    NP e = expr();
    if (cur().k != TK_EOF) throw SyntaxError("unexpected '" + cur().s + "'");
    return e;
  }
  NP expr() {
    NP c = or_();
    if (peek_is("?")) {
      eat("?");
      NP a = or_();
      eat(":");
      NP b = expr();
      NP n = mk(Node::COND);
      n->kids = {c, a, b};
      return n;
    }
    return c;
  }
  NP bin(const std::string& op, NP l, NP r) {
    NP n = mk(Node::BINARY);
    n->name = op;
    n->kids = {l, r};
    return n;
  }
  NP or_() {
    NP e = and_();
    while (peek_is("||")) { eat(); e = bin("||", e, and_()); }
    return e;
  }
  NP and_() {
    NP e = rel();
    while (peek_is("&&")) { eat(); e = bin("&&", e, rel()); }
    return e;
  }
  NP rel() {
    NP e = add();
    for (;;) {
      const Tok& x = cur();
      const bool isrel = x.s == "==" || x.s == "!=" || x.s == "<" || x.s == "<=" || x.s == ">" || x.s == ">=" || x.s == "in";
      if (!(isrel && (x.k == TK_OP || x.k == TK_IDENT))) break;
      const std::string op = eat().s;
      e = bin(op, e, add());
    }
    return e;
  }
  NP add() {
    NP e = mul();
    while ((cur().s == "+" || cur().s == "-") && cur().k == TK_OP) {
      const std::string op = eat().s;
      e = bin(op, e, mul());
    }
    return e;
  }
  NP mul() {
    NP e = unary();
    while ((cur().s == "*" || cur().s == "/" || cur().s == "%") && cur().k == TK_OP) {
      const std::string op = eat().s;
      e = bin(op, e, unary());
    }
    return e;
  }
  bool postfix_follows() const {
    if (i + 1 >= t.size()) throw SyntaxError("unexpected end of expression");
    return (t[i + 1].s == "." || t[i + 1].s == "[") && t[i + 1].k == TK_OP;
  }
  NP unary() {
    if ((cur().s == "!" || cur().s == "-") && cur().k == TK_OP) {
      const std::string op = eat().s;
      const Tok& x = cur();
      if (op == "-" && (x.k == TK_INT || x.k == TK_FLOAT || x.k == TK_HEX) && !postfix_follows()) {
        const Tok num = eat();
        NP n = mk(Node::LIT);
        n->lit = number(num, true);
        return n;
      }
      NP n = mk(Node::UNARY);
      n->name = op;
      n->kids = {unary()};
      return n;
    }
    return member();
  }
  static Value number(const Tok& x, bool neg) {
    if (x.k == TK_FLOAT) {
      const double v = strtod(x.s.c_str(), nullptr);
      return vdbl(neg ? -v : v);
    }
    const bool u = x.s.back() == 'u' || x.s.back() == 'U';
    std::string body = u ? x.s.substr(0, x.s.size() - 1) : x.s;
    unsigned __int128 v = 0;
    const bool hex = x.k == TK_HEX;
    for (size_t k = hex ? 2 : 0; k < body.size(); ++k) {
      const char c = body[k];
      const int d = isdig(c) ? c - '0' : (c >= 'a' && c <= 'f') ? c - 'a' + 10 : c - 'A' + 10;
      v = v * (hex ? 16 : 10) + d;
      if (v > ((unsigned __int128)1 << 66)) {
        if (u) throw SyntaxError("uint literal out of range");
        throw SyntaxError("int literal out of range");
      }
    }
    if (u) {
      if (neg || v > (unsigned __int128)UINT64_MAX) throw SyntaxError("uint literal out of range");
      return vuint((uint64_t)v);
    }
    const i128 sv = neg ? -(i128)v : (i128)v;
    if (sv < (i128)kI64Min || sv > (i128)kI64Max) throw SyntaxError("int literal out of range");
    return vint((int64_t)sv);
  }
  std::vector<NP> args() {
    eat("(");
    std::vector<NP> out;
    if (!peek_is(")")) {
      out.push_back(expr());
      while (peek_is(",")) { eat(); out.push_back(expr()); }
    }
    eat(")");
    return out;
  }
  NP member() {
    NP e = primary();
    for (;;) {
      if (peek_op(".")) {
        eat();
        const std::string name = eat().s;
        if (peek_op("(")) {
          NP n = mk(Node::METHOD);
          n->name = name;
          n->kids.push_back(e);
          for (NP& a : args()) n->kids.push_back(a);
          e = n;
        } else {
          NP n = mk(Node::SELECT);
          n->name = name;
          n->kids = {e};
          e = n;
        }
      } else if (peek_op("[")) {
        eat();
        NP idx = expr();
        eat("]");
        NP n = mk(Node::INDEX);
        n->kids = {e, idx};
        e = n;
      } else {
        return e;
      }
    }
  }
  NP primary() {
    const Tok x = cur();
    if (x.k == TK_INT || x.k == TK_FLOAT || x.k == TK_HEX) {
      eat();
      NP n = mk(Node::LIT);
      n->lit = number(x, false);
      return n;
    }
    if (x.k == TK_STR) {
      eat();
      NP n = mk(Node::LIT);
      n->lit = vstr(unescape(x.s));
      return n;
    }
    if (x.k == TK_IDENT) {
      eat();
      NP n = mk(Node::LIT);
      if (x.s == "true") { n->lit = vbool(true); return n; }
      if (x.s == "false") { n->lit = vbool(false); return n; }
      if (x.s == "null") { n->lit = vnull(); return n; }
      if (peek_op("(")) {
        NP c = mk(Node::CALL);
        c->name = x.s;
        c->kids = args();
        return c;
      }
      NP id = mk(Node::IDENT);
      id->name = x.s;
      return id;
    }
    if (x.s == "(") {
      eat();
      NP e = expr();
      eat(")");
      return e;
    }
    if (x.s == "[") {
      eat();
      NP n = mk(Node::LIST);
      if (!peek_is("]")) {
        n->kids.push_back(expr());
        while (peek_is(",")) {
          eat();
          if (peek_is("]")) break;
          n->kids.push_back(expr());
        }
      }
      eat("]");
      return n;
    }
    if (x.s == "{") {
      eat();
      NP n = mk(Node::MAP);
      if (!peek_is("}")) {
        for (;;) {
          NP key = expr();
          eat(":");
          NP val = expr();
          n->entries.emplace_back(key, val);
          if (!peek_is(",")) break;
          eat();
          if (peek_is("}")) break;
        }
      }
      eat("}");
      return n;
    }
    throw SyntaxError("unexpected '" + x.s + "'");
  }
};

inline NP parse(const std::string& src) { return Parser(src).parse(); }

// ------------------------------------------------------------------ constant evaluation (cel.py Evaluator, Env())
inline int64_t checked_int(i128 v) {
  if (v < (i128)kI64Min || v > (i128)kI64Max) throw CELError("integer overflow");
  return (int64_t)v;
}
inline uint64_t checked_uint(i128 v) {
  if (v < 0 || v > (i128)UINT64_MAX) throw CELError("unsigned integer overflow");
  return (uint64_t)v;
}

inline bool num_eq(const Value& a, const Value& b) {  // _num_eq
  if (a.t == Value::BOOL || b.t == Value::BOOL) return a.t == b.t && a.b == b.b;
  const bool an = is_intlike(a) || a.t == Value::DBL, bn = is_intlike(b) || b.t == Value::DBL;
  if (an && bn) {
    if (a.t == Value::DBL || b.t == Value::DBL) return as_dbl(a) == as_dbl(b);
    return as_i128(a) == as_i128(b);
  }
  if (a.t == Value::QTY || b.t == Value::QTY) {
    if (a.t == Value::QTY && b.t == Value::QTY) return a.q.cmp(b.q) == 0;
    throw CELError("no such overload: ==");
  }
  if (strcmp(type_name(a), type_name(b)) != 0) return false;
  return py_eq(a, b);
}

inline Value arith(const std::string& op, const Value& a, const Value& b) {
  if (a.t == Value::QTY) {
    if (op == "+" || op == "-") {
      if (b.t != Value::QTY) throw CELError("no such overload: Quantity " + op);
      i128 x, y;
      int64_t s;
      a.q.aligned(b.q, x, y, s);
      return vqty(Quantity{op == "+" ? add_chk(x, y) : add_chk(x, -y), s});
    }
    if (op == "*" || op == "/") {
      if (b.t == Value::BOOL) throw CELError("no such overload");
      if (is_intlike(b)) {  // nano arithmetic, Go int64 wrap-around for *
        const i128 n = a.q.scaled_nano();
        const i128 m = as_i128(b);
        if (op == "*") {
          const uint64_t r = (uint64_t)(unsigned __int128)n * (uint64_t)(unsigned __int128)m;
          return vqty(Quantity::nano((i128)(int64_t)r));
        }
        if (m == 0) throw CELError("integer divide by zero");
        const i128 q = (n < 0 ? -n : n) / (m < 0 ? -m : m);
        return vqty(Quantity::nano((n >= 0) == (m >= 0) ? q : -q));
      }
      if (b.t == Value::DBL) {
        if (op == "/" && b.d == 0.0) throw CELError("float division by zero");
        return vqty(quantity_from_float(op == "*" ? a.q.approx() * b.d : a.q.approx() / b.d));
      }
    }
    throw CELError(std::string("no such overload: Quantity ") + op + " " + type_name(b));
  }
  if (a.t == Value::BOOL || b.t == Value::BOOL || a.t != b.t)
    throw CELError(std::string("no such overload: ") + type_name(a) + " " + op + " " + type_name(b));
  switch (a.t) {
    case Value::DBL:
      if (op == "+") return vdbl(a.d + b.d);
      if (op == "-") return vdbl(a.d - b.d);
      if (op == "*") return vdbl(a.d * b.d);
      if (op == "/") {
        if (b.d == 0.0) {
          if (a.d != 0 && a.d == a.d) return vdbl(std::copysign(HUGE_VAL, a.d) * std::copysign(1.0, b.d));
          return vdbl(NAN);
        }
        return vdbl(a.d / b.d);
      }
      throw CELError("no such overload: double %");
    case Value::UINT: {
      const i128 x = a.u, y = b.u;
      if (op == "+") return vuint(checked_uint(x + y));
      if (op == "-") return vuint(checked_uint(x - y));
      if (op == "*") return vuint(checked_uint(mul_chk(x, y)));
      if (y == 0) throw CELError(op == "/" ? "divide by zero" : "modulus by zero");
      return vuint((uint64_t)(op == "/" ? x / y : x % y));
    }
    case Value::INT: {
      const i128 x = a.i, y = b.i;
      if (op == "+") return vint(checked_int(x + y));
      if (op == "-") return vint(checked_int(x - y));
      if (op == "*") return vint(checked_int(x * y));
      if (y == 0) throw CELError(op == "/" ? "divide by zero" : "modulus by zero");
      if (op == "/") {
        if (x == kI64Min && y == -1) throw CELError("integer overflow");
        return vint((int64_t)(x / y));  // truncation toward zero
      }
      return vint((int64_t)(x % y));    // sign of the dividend
    }
    case Value::STR:
      if (op == "+") return vstr(a.s + b.s);
      break;
    case Value::LIST:
      if (op == "+") {
        Value r = a;
        r.list.insert(r.list.end(), b.list.begin(), b.list.end());
        return r;
      }
      break;
    default: break;
  }
  throw CELError(std::string("no such overload: ") + type_name(a) + " " + op + " " + type_name(b));
}

inline bool order(const std::string& op, const Value& a, const Value& b) {
  int c;
  if (a.t == Value::QTY && b.t == Value::QTY) {
    c = a.q.cmp(b.q);
  } else if (a.t == b.t && (a.t == Value::INT || a.t == Value::UINT || a.t == Value::DBL || a.t == Value::STR)) {
    if (a.t == Value::STR) c = (a.s > b.s) - (a.s < b.s);  // UTF-8 byte order = code point order
    else if (a.t == Value::DBL) c = (a.d > b.d) - (a.d < b.d);
    else c = (as_i128(a) > as_i128(b)) - (as_i128(a) < as_i128(b));
  } else if (a.t == Value::BOOL && b.t == Value::BOOL) {
    c = (a.b > b.b) - (a.b < b.b);
  } else {
    throw CELError(std::string("no such overload: ") + type_name(a) + " " + op + " " + type_name(b));
  }
  if (op == "<") return c < 0;
  if (op == "<=") return c <= 0;
  if (op == ">") return c > 0;
  return c >= 0;
}

inline size_t utf8_len(const std::string& s) {
  size_t n = 0;
  for (unsigned char c : s) n += (c & 0xC0) != 0x80;
  return n;
}

// Python float(str) for the ASCII forms double() meets in practice (strtod over the stripped text)
inline double py_float_of(const std::string& s) {
  size_t a = 0, b = s.size();
  while (a < b && isws((unsigned char)s[a])) ++a;
  while (b > a && isws((unsigned char)s[b - 1])) --b;
  const std::string t = s.substr(a, b - a);
  if (t.empty()) throw CELError("double conversion error");
  for (char c : t)
    if (!(isdig(c) || c == '.' || c == 'e' || c == 'E' || c == '+' || c == '-' || isident0(c)))
      throw CELError("double conversion error");
  std::string low;
  for (char c : t) low += (char)tolower((unsigned char)c);
  const std::string body = (low[0] == '+' || low[0] == '-') ? low.substr(1) : low;
  if (body == "inf" || body == "infinity") return low[0] == '-' ? -HUGE_VAL : HUGE_VAL;
  if (body == "nan") return NAN;
  for (char c : body) if (isident0(c) && c != 'e') throw CELError("double conversion error");
  char* end = nullptr;
  const double v = strtod(t.c_str(), &end);
  if (end != t.c_str() + t.size() || !(isdig(body[0]) || (body[0] == '.' && body.size() > 1 && isdig(body[1]))))
    throw CELError("double conversion error");
  return v;
}

struct Evaluator {
  Value ev(const NP& n) {
    switch (n->k) {
      case Node::LIT: return n->lit;
      case Node::IDENT: throw CELError("undeclared reference to '" + n->name + "'");
      case Node::SELECT: {
        const Value v = ev(n->kids[0]);
        if (v.t == Value::MAP) {
          const Value* x = map_find(v, vstr(n->name));
          if (!x) throw CELError("no such key: " + n->name);
          return *x;
        }
        throw CELError(std::string("type ") + type_name(v) + " has no field '" + n->name + "'");
      }
      case Node::INDEX: {
        const Value v = ev(n->kids[0]);
        const Value i = ev(n->kids[1]);
        if (v.t == Value::MAP) {
          const Value* x = map_find(v, i);
          if (!x) throw CELError("no such key");
          return *x;
        }
        if (v.t == Value::LIST) {
          i128 k;
          if (is_intlike(i)) k = as_i128(i);
          else if (i.t == Value::DBL && i.d == std::floor(i.d) && std::fabs(i.d) < 1e30) k = (i128)i.d;
          else throw CELError("invalid list index");
          if (k < 0 || k >= (i128)v.list.size()) throw CELError("index out of range");
          return v.list[(size_t)k];
        }
        throw CELError(std::string("no such overload: index ") + type_name(v));
      }
      case Node::COND: {
        const Value c = ev(n->kids[0]);
        if (c.t != Value::BOOL) throw CELError("no such overload: ternary condition");
        return ev(c.b ? n->kids[1] : n->kids[2]);
      }
      case Node::UNARY: {
        const Value v = ev(n->kids[0]);
        if (n->name == "!") {
          if (v.t != Value::BOOL) throw CELError("no such overload: !");
          return vbool(!v.b);
        }
        if (v.t == Value::QTY) return vqty(Quantity{-v.q.value, v.q.scale});
        if (v.t == Value::INT) return vint(checked_int(-(i128)v.i));
        if (v.t == Value::DBL) return vdbl(-v.d);
        throw CELError(std::string("no such overload: -") + type_name(v));
      }
      case Node::BINARY: return binary(n);
      case Node::LIST: {
        Value r;
        r.t = Value::LIST;
        for (const NP& x : n->kids) r.list.push_back(ev(x));
        return r;
      }
      case Node::MAP: {
        Value r;
        r.t = Value::MAP;
        for (const auto& e : n->entries) {
          Value k = ev(e.first);
          Value v = ev(e.second);
          check_hashable(k);
          bool set = false;
          for (auto& f : r.map)
            if (py_eq(f.first, k)) { f.second = v; set = true; break; }  // first key kept, value replaced
          if (!set) r.map.emplace_back(std::move(k), std::move(v));
        }
        return r;
      }
      case Node::CALL: {
        std::vector<Value> full;
        for (const NP& x : n->kids) full.push_back(ev(x));
        return call(n->name, false, full);
      }
      case Node::METHOD: {
        std::vector<Value> full;
        for (const NP& x : n->kids) full.push_back(ev(x));  // target first, then the args
        return call(n->name, true, full);
      }
    }
    throw CELError("bad node");
  }

  Value binary(const NP& n) {
    const std::string& op = n->name;
    if (op == "&&" || op == "||") {
      bool have_err = false;
      std::string err;
      for (int side = 0; side < 2; ++side) {
        bool v;
        try {
          const Value x = ev(n->kids[side]);
          if (x.t != Value::BOOL) throw CELError("no such overload: " + op);
          v = x.b;
        } catch (const CELError& e) {
          have_err = true;
          err = e.what();
          continue;
        }
        if (op == "&&" && !v) return vbool(false);
        if (op == "||" && v) return vbool(true);
      }
      if (have_err) throw CELError(err);
      return vbool(op == "&&");
    }
    const Value a = ev(n->kids[0]);
    const Value b = ev(n->kids[1]);
    if (op == "==") return vbool(num_eq(a, b));
    if (op == "!=") return vbool(!num_eq(a, b));
    if (op == "<" || op == "<=" || op == ">" || op == ">=") return vbool(order(op, a, b));
    if (op == "in") {
      if (b.t == Value::MAP) return vbool(map_find(b, a) != nullptr);
      if (b.t == Value::LIST) {
        for (const Value& x : b.list) {
          const bool comparable = strcmp(type_name(x), type_name(a)) == 0 || (is_pynum(x) && is_pynum(a));
          if (comparable && num_eq(a, x)) return vbool(true);
        }
        return vbool(false);
      }
      throw CELError("no such overload: in");
    }
    return arith(op, a, b);
  }

  Value call(const std::string& name, bool method, const std::vector<Value>& full) {
    if ((name == "Now" || name == "now") && full.empty()) throw CELError("Now is not bound");
    if (name == "Rand" && full.empty()) throw CELError("Rand is not bound");
    if (name == "Quantity" && full.size() == 1 && full[0].t == Value::STR) return vqty(quantity_parse(full[0].s));
    if (!method && full.size() == 1) {  // standard conversions
      const Value& v = full[0];
      if (name == "double") {
        if (v.t == Value::QTY) return vdbl(v.q.approx());
        if (is_intlike(v) || v.t == Value::DBL) return vdbl(as_dbl(v));
        if (v.t == Value::STR) return vdbl(py_float_of(v.s));
      }
      if (name == "int" && (is_intlike(v) || v.t == Value::DBL)) {
        if (v.t == Value::DBL) {
          if (!(v.d > -9.223372036854776e18 && v.d < 9.223372036854776e18)) throw CELError("int conversion range error");
          return vint((int64_t)v.d);
        }
        return vint(checked_int(as_i128(v)));
      }
      if (name == "string") {
        if (v.t == Value::STR) return v;
        if (v.t == Value::BOOL) return vstr(v.b ? "true" : "false");
        if (is_intlike(v)) return vstr(i128_str(as_i128(v)));
      }
    }
    if (name == "size" && full.size() == 1) {
      const Value& v = full[0];
      if (v.t == Value::STR) return vint((int64_t)utf8_len(v.s));
      if (v.t == Value::LIST) return vint((int64_t)v.list.size());
      if (v.t == Value::MAP) return vint((int64_t)v.map.size());
    }
    throw CELError("found no matching overload for '" + name + "'");
  }
};

// AsFloat64 (environment.go:117-138)
inline double as_float64(const Value& v) {
  if (v.t == Value::BOOL) return v.b ? 1.0 : 0.0;
  if (is_intlike(v) || v.t == Value::DBL) return as_dbl(v);
  if (v.t == Value::QTY) return v.q.approx();
  throw CELError(std::string("unsupported type: ") + type_name(v));
}

// ------------------------------------------------------------------ lowering (cel.py lower)
enum { OP_CONST = 1, OP_LOAD = 2, OP_ADD = 3, OP_SUB = 4, OP_MUL = 5, OP_DIV = 6, OP_NEG = 7 };
enum {
  IN_NOW_S = 0, IN_CONTAINER_CPU = 1, IN_CONTAINER_CUM_CPU = 3, IN_POD_CPU = 5, IN_POD_CUM_CPU = 7, IN_NODE_CPU = 9,
  IN_NODE_CUM_CPU = 11, IN_POD_SINCE = 13, IN_NODE_SINCE = 14, IN_POD_CREATED = 15, IN_NODE_CREATED = 16,
  IN_STARTED_CONTAINERS = 17
};
enum Dim { DIM_NODE = 0, DIM_POD = 1, DIM_CONTAINER = 2, DIM_OTHER = 3 };

struct Op { uint32_t op; uint32_t arg; double value; };

inline bool dyn(const NP& n) {  // depends on the series: a variable, the clock, a callback
  switch (n->k) {
    case Node::IDENT: return true;
    case Node::LIT: return false;
    case Node::CALL:
      if (n->name == "Now" || n->name == "now" || n->name == "Rand" || n->name == "StartedContainersTotal" ||
          n->name == "startedContainersTotal")
        return true;
      break;
    case Node::MAP:
      for (const auto& e : n->entries) if (dyn(e.first) || dyn(e.second)) return true;
      return false;
    default: break;
  }
  for (const NP& x : n->kids) if (dyn(x)) return true;
  return false;
}

inline bool is_ident(const NP& n, const char* name) { return n->k == Node::IDENT && n->name == name; }
inline bool is_creation(const NP& t, const char* who) {  // who.metadata.creationTimestamp
  return t->k == Node::SELECT && t->name == "creationTimestamp" && t->kids[0]->k == Node::SELECT &&
         t->kids[0]->name == "metadata" && is_ident(t->kids[0]->kids[0], who);
}
inline bool is_now_call(const NP& t) {
  return t->k == Node::CALL && (t->name == "Now" || t->name == "now") && t->kids.empty();
}

struct Lowering {
  Dim dim;
  std::vector<Op> prog;
  enum Ty { DOUBLE, INTT, QTYT };

  Ty emit(const NP& n) {
    if (!dyn(n)) {
      const Value v = Evaluator().ev(n);
      if (v.t == Value::DBL) { prog.push_back({OP_CONST, 0, v.d}); return DOUBLE; }
      if (is_intlike(v)) { prog.push_back({OP_CONST, 0, as_dbl(v)}); return INTT; }
      if (v.t == Value::QTY) { prog.push_back({OP_CONST, 0, v.q.approx()}); return QTYT; }
      throw LowerError(std::string("constant of type ") + type_name(v));
    }
    if (n->k == Node::METHOD && (n->name == "Usage" || n->name == "CumulativeUsage")) {
      const NP& tgt = n->kids[0];
      const size_t na = n->kids.size() - 1;
      const bool cum = n->name == "CumulativeUsage";
      if (!is_ident(tgt, "pod") && !is_ident(tgt, "node")) throw LowerError("Usage on something other than pod / node");
      if (na == 0 || n->kids[1]->k != Node::LIT || n->kids[1]->lit.t != Value::STR ||
          (n->kids[1]->lit.s != "cpu" && n->kids[1]->lit.s != "memory"))
        throw LowerError("Usage resource must be a literal cpu / memory");
      const uint32_t r = n->kids[1]->lit.s == "cpu" ? 0 : 1;
      if (is_ident(tgt, "node") && na == 1) {
        if (dim == DIM_OTHER) throw LowerError("unknown dimension");
        prog.push_back({OP_LOAD, (cum ? IN_NODE_CUM_CPU : IN_NODE_CPU) + r, 0.0});
      } else if (is_ident(tgt, "pod") && na == 1) {
        if (dim != DIM_POD && dim != DIM_CONTAINER) throw LowerError("pod usage needs the pod dimension");
        prog.push_back({OP_LOAD, (cum ? IN_POD_CUM_CPU : IN_POD_CPU) + r, 0.0});
      } else if (is_ident(tgt, "pod") && na == 2 && n->kids[2]->k == Node::SELECT && n->kids[2]->name == "name" &&
                 is_ident(n->kids[2]->kids[0], "container")) {
        if (dim != DIM_CONTAINER) throw LowerError("container usage needs the container dimension");
        prog.push_back({OP_LOAD, (cum ? IN_CONTAINER_CUM_CPU : IN_CONTAINER_CPU) + r, 0.0});
      } else {
        throw LowerError("unsupported Usage arguments");
      }
      return DOUBLE;
    }
    if (n->k == Node::METHOD && n->name == "SinceSecond" && n->kids.size() == 1 &&
        (is_ident(n->kids[0], "pod") || is_ident(n->kids[0], "node"))) {
      prog.push_back({OP_LOAD, is_ident(n->kids[0], "pod") ? (uint32_t)IN_POD_SINCE : (uint32_t)IN_NODE_SINCE, 0.0});
      return DOUBLE;
    }
    if (n->k == Node::CALL && n->name == "SinceSecond" && n->kids.size() == 1 &&
        (is_ident(n->kids[0], "pod") || is_ident(n->kids[0], "node"))) {
      prog.push_back({OP_LOAD, is_ident(n->kids[0], "pod") ? (uint32_t)IN_POD_SINCE : (uint32_t)IN_NODE_SINCE, 0.0});
      return DOUBLE;
    }
    if (n->k == Node::METHOD && (n->name == "StartedContainersTotal" || n->name == "startedContainersTotal") &&
        is_ident(n->kids[0], "node") && n->kids.size() == 1) {
      prog.push_back({OP_LOAD, IN_STARTED_CONTAINERS, 0.0});
      return DOUBLE;
    }
    if ((n->k == Node::METHOD && n->name == "UnixSecond" && n->kids.size() == 1) ||
        (n->k == Node::CALL && n->name == "UnixSecond" && n->kids.size() == 1)) {
      const NP& t = n->kids[0];
      if (is_now_call(t)) { prog.push_back({OP_LOAD, IN_NOW_S, 0.0}); return DOUBLE; }
      if (is_creation(t, "pod")) { prog.push_back({OP_LOAD, IN_POD_CREATED, 0.0}); return DOUBLE; }
      if (is_creation(t, "node")) { prog.push_back({OP_LOAD, IN_NODE_CREATED, 0.0}); return DOUBLE; }
      throw LowerError("UnixSecond of an unsupported timestamp");
    }
    if (n->k == Node::UNARY && n->name == "-") {
      if (emit(n->kids[0]) != DOUBLE) throw LowerError("negation of a non-double");
      prog.push_back({OP_NEG, 0, 0.0});
      return DOUBLE;
    }
    if (n->k == Node::BINARY && (n->name == "+" || n->name == "-" || n->name == "*" || n->name == "/")) {
      const Ty ta = emit(n->kids[0]);
      const Ty tb = emit(n->kids[1]);
      if (ta != DOUBLE || tb != DOUBLE) throw LowerError("mixed-type arithmetic " + n->name);  // CEL: no int <-> double
      const char c = n->name[0];
      prog.push_back({(uint32_t)(c == '+' ? OP_ADD : c == '-' ? OP_SUB : c == '*' ? OP_MUL : OP_DIV), 0, 0.0});
      return DOUBLE;
    }
    throw LowerError("no device form for this expression");
  }
};

// value expression -> postfix program; throws SyntaxError / CELError (the expression is wrong:
// a compile error) or LowerError (valid, but the host must evaluate it per series)
inline std::vector<Op> lower(const std::string& src, Dim dim) {
  const NP ast = parse(src);
  if (!dyn(ast)) return {{OP_CONST, 0, as_float64(Evaluator().ev(ast))}};
  Lowering L{dim, {}};
  if (L.emit(ast) != Lowering::DOUBLE) throw LowerError("the value is not a double");
  return L.prog;
}

}  // namespace kwkcel
