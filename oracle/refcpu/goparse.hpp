// ORACLE / TEST INFRASTRUCTURE — not product code.
// Restatements of the Go standard-library parsers KWOK's value getters call
// (Go 1.22.3, .dependencies.yaml / go.mod:3; the Go toolchain is absent from this image):
//   strconv.ParseInt(s, 0, 0)     — expression/value_int_from.go:69
//   time.ParseDuration(s)         — expression/value_duration_from.go:73
//   time.Parse(time.RFC3339Nano)  — expression/value_duration_from.go:68 (fast RFC3339 path
//                                   plus the lenient generic-layout fallbacks)
//   time.Time.Sub (saturating)    — expression/value_duration_from.go:70
#pragma once
#include <cstdint>
#include <string>

namespace refcpu {

inline char go_lower(char c) { return (char)(c | ('x' - 'X')); }

inline bool go_underscore_ok(std::string s) {
  char saw = '^';
  size_t i = 0;
  if (!s.empty() && (s[0] == '-' || s[0] == '+')) s = s.substr(1);
  bool hex = false;
  if (s.size() >= 2 && s[0] == '0' && (go_lower(s[1]) == 'b' || go_lower(s[1]) == 'o' || go_lower(s[1]) == 'x')) {
    i = 2;
    saw = '0';
    hex = go_lower(s[1]) == 'x';
  }
  for (; i < s.size(); ++i) {
    if ((s[i] >= '0' && s[i] <= '9') || (hex && go_lower(s[i]) >= 'a' && go_lower(s[i]) <= 'f')) { saw = '0'; continue; }
    if (s[i] == '_') { if (saw != '0') return false; saw = '_'; continue; }
    if (saw == '_') return false;
    saw = '!';
  }
  return saw != '_';
}

// strconv.ParseUint(s, 0, 64); returns 0 ok, 1 syntax error, 2 range error
inline int go_parse_uint0(const std::string& s0, uint64_t& out) {
  out = 0;
  if (s0.empty()) return 1;
  std::string s = s0;
  int base = 10;
  if (s[0] == '0') {
    if (s.size() >= 3 && go_lower(s[1]) == 'b') { base = 2; s = s.substr(2); }
    else if (s.size() >= 3 && go_lower(s[1]) == 'o') { base = 8; s = s.substr(2); }
    else if (s.size() >= 3 && go_lower(s[1]) == 'x') { base = 16; s = s.substr(2); }
    else { base = 8; s = s.substr(1); }
  }
  const uint64_t maxv = ~0ull;
  const uint64_t cutoff = maxv / (uint64_t)base + 1;
  bool underscores = false;
  uint64_t n = 0;
  for (char c : s) {
    unsigned d;
    if (c == '_') { underscores = true; continue; }
    else if (c >= '0' && c <= '9') d = (unsigned)(c - '0');
    else if (go_lower(c) >= 'a' && go_lower(c) <= 'z') d = (unsigned)(go_lower(c) - 'a' + 10);
    else return 1;
    if (d >= (unsigned)base) return 1;
    if (n >= cutoff) { out = maxv; return 2; }
    n *= (uint64_t)base;
    uint64_t n1 = n + d;
    if (n1 < n) { out = maxv; return 2; }
    n = n1;
  }
  if (underscores && !go_underscore_ok(s0)) return 1;
  out = n;
  return 0;
}

// strconv.ParseInt(s, 0, 0) on a 64-bit platform; returns true iff err == nil
inline bool go_parse_int(const std::string& s0, int64_t& out) {
  out = 0;
  if (s0.empty()) return false;
  std::string s = s0;
  bool neg = false;
  if (s[0] == '+') s = s.substr(1);
  else if (s[0] == '-') { neg = true; s = s.substr(1); }
  uint64_t un;
  int e = go_parse_uint0(s, un);
  if (e == 1) return false;
  const uint64_t cutoff = 1ull << 63;
  if (e == 2) return false;
  if (!neg && un >= cutoff) return false;
  if (neg && un > cutoff) return false;
  out = neg ? (int64_t)(0 - un) : (int64_t)un;
  return true;
}

// time.ParseDuration; returns true iff err == nil
inline bool go_parse_duration(const std::string& orig, int64_t& out) {
  out = 0;
  std::string s = orig;
  uint64_t d = 0;
  bool neg = false;
  if (!s.empty() && (s[0] == '-' || s[0] == '+')) { neg = s[0] == '-'; s = s.substr(1); }
  if (s == "0") { out = 0; return true; }
  if (s.empty()) return false;
  const uint64_t LIM = 1ull << 63;
  while (!s.empty()) {
    uint64_t v = 0, f = 0;
    double scale = 1;
    if (!(s[0] == '.' || (s[0] >= '0' && s[0] <= '9'))) return false;
    size_t pl = s.size();
    size_t i = 0;
    for (; i < s.size(); ++i) {  // leadingInt
      char c = s[i];
      if (c < '0' || c > '9') break;
      if (v > LIM / 10) return false;
      v = v * 10 + (uint64_t)(c - '0');
      if (v > LIM) return false;
    }
    s = s.substr(i);
    bool pre = pl != s.size();
    bool post = false;
    if (!s.empty() && s[0] == '.') {
      s = s.substr(1);
      size_t pl2 = s.size();
      size_t j = 0;
      bool overflow = false;
      for (; j < s.size(); ++j) {  // leadingFraction
        char c = s[j];
        if (c < '0' || c > '9') break;
        if (overflow) continue;
        if (f > (LIM - 1) / 10) { overflow = true; continue; }
        uint64_t y = f * 10 + (uint64_t)(c - '0');
        if (y > LIM) { overflow = true; continue; }
        f = y;
        scale *= 10;
      }
      s = s.substr(j);
      post = pl2 != s.size();
    }
    if (!pre && !post) return false;
    size_t k = 0;
    for (; k < s.size(); ++k) { char c = s[k]; if (c == '.' || (c >= '0' && c <= '9')) break; }
    if (k == 0) return false;  // missing unit
    std::string u = s.substr(0, k);
    s = s.substr(k);
    uint64_t unit;
    if (u == "ns") unit = 1;
    else if (u == "us" || u == "\xC2\xB5s" || u == "\xCE\xBCs") unit = 1000ull;
    else if (u == "ms") unit = 1000000ull;
    else if (u == "s") unit = 1000000000ull;
    else if (u == "m") unit = 60ull * 1000000000ull;
    else if (u == "h") unit = 3600ull * 1000000000ull;
    else return false;
    if (v > LIM / unit) return false;
    v *= unit;
    if (f > 0) {
      v += (uint64_t)((double)f * ((double)unit / scale));
      if (v > LIM) return false;
    }
    d += v;
    if (d > LIM) return false;
  }
  if (neg) { out = (int64_t)(0 - d); return true; }
  if (d > LIM - 1) return false;
  out = (int64_t)d;
  return true;
}

inline bool go_is_leap(int64_t y) { return y % 4 == 0 && (y % 100 != 0 || y % 400 == 0); }
inline int go_days_in(int m, int64_t y) {
  static const int d[] = {31, 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
  if (m == 2 && go_is_leap(y)) return 29;
  return d[m - 1];
}
// days from 1970-01-01 to y-m-d (proleptic Gregorian)
inline int64_t days_from_civil(int64_t y, unsigned m, unsigned d) {
  y -= m <= 2;
  const int64_t era = (y >= 0 ? y : y - 399) / 400;
  const unsigned yoe = (unsigned)(y - era * 400);
  const unsigned doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
  const unsigned doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
  return era * 146097 + (int64_t)doe - 719468;
}

struct GoTime { int64_t sec; int32_t nsec; };  // unix seconds + [0,1e9) nanoseconds

inline bool go_digits(const std::string& s, size_t pos, size_t n, int& out) {
  if (pos + n > s.size()) return false;
  int x = 0;
  for (size_t i = 0; i < n; ++i) {
    char c = s[pos + i];
    if (c < '0' || c > '9') return false;
    x = x * 10 + (c - '0');
  }
  out = x;
  return true;
}

// parseNanoseconds(value, nbytes): value[0] is '.' or ','
inline int go_parse_nanos(const std::string& frac_with_sep, size_t nbytes) {
  if (nbytes > 10) nbytes = 10;
  int ns = 0;
  for (size_t i = 1; i < nbytes; ++i) ns = ns * 10 + (frac_with_sep[i] - '0');
  for (size_t i = 0; i < 10 - nbytes; ++i) ns *= 10;
  return ns;
}

inline GoTime go_make_time(int64_t y, int mo, int d, int h, int mi, int se, int ns, int64_t zone_sec) {
  int64_t days = days_from_civil(y, (unsigned)mo, (unsigned)d);
  return GoTime{days * 86400 + h * 3600 + mi * 60 + se - zone_sec, ns};
}

// time/format_rfc3339.go parseRFC3339 (the fast path)
inline bool go_parse_rfc3339_fast(const std::string& s0, GoTime& out) {
  std::string s = s0;
  if (s.size() < 19) return false;
  int year, month, day, hour, mi, sec;
  bool ok = go_digits(s, 0, 4, year) && go_digits(s, 5, 2, month) && go_digits(s, 8, 2, day) &&
            go_digits(s, 11, 2, hour) && go_digits(s, 14, 2, mi) && go_digits(s, 17, 2, sec);
  if (!ok) return false;
  if (month < 1 || month > 12) return false;
  if (day < 1 || day > go_days_in(month, year)) return false;
  if (hour > 23 || mi > 59 || sec > 59) return false;
  if (!(s[4] == '-' && s[7] == '-' && s[10] == 'T' && s[13] == ':' && s[16] == ':')) return false;
  s = s.substr(19);
  int nsec = 0;
  if (s.size() >= 2 && s[0] == '.' && s[1] >= '0' && s[1] <= '9') {
    size_t n = 2;
    while (n < s.size() && s[n] >= '0' && s[n] <= '9') ++n;
    nsec = go_parse_nanos(s, n);
    s = s.substr(n);
  }
  int64_t zone = 0;
  if (!(s.size() == 1 && s[0] == 'Z')) {
    if (s.size() != 6) return false;
    int hr, mm;
    if (!go_digits(s, 1, 2, hr) || !go_digits(s, 4, 2, mm)) return false;
    if (hr > 23 || mm > 59) return false;
    if (!((s[0] == '-' || s[0] == '+') && s[3] == ':')) return false;
    zone = (hr * 60 + mm) * 60;
    if (s[0] == '-') zone = -zone;
  }
  out = go_make_time(year, month, day, hour, mi, sec, nsec, zone);
  return true;
}

// time.Parse's generic layout walk for "2006-01-02T15:04:05.999999999Z07:00" (format.go
// `parse`): differs from the fast path by accepting a 1-digit hour, a ',' fraction separator
// and zone offsets up to 24h/60m.
inline bool go_parse_rfc3339_generic(const std::string& v, GoTime& out) {
  size_t p = 0;
  int year, month, day, hour, mi, sec;
  if (!go_digits(v, p, 4, year)) return false;
  p += 4;
  if (p >= v.size() || v[p] != '-') return false;
  ++p;
  if (!go_digits(v, p, 2, month)) return false;
  p += 2;
  if (p >= v.size() || v[p] != '-') return false;
  ++p;
  if (!go_digits(v, p, 2, day)) return false;
  p += 2;
  if (p >= v.size() || v[p] != 'T') return false;
  ++p;
  // stdHour: getnum(value, false) — one or two digits
  if (p >= v.size() || v[p] < '0' || v[p] > '9') return false;
  hour = v[p] - '0';
  ++p;
  if (p < v.size() && v[p] >= '0' && v[p] <= '9') { hour = hour * 10 + (v[p] - '0'); ++p; }
  if (p >= v.size() || v[p] != ':') return false;
  ++p;
  if (!go_digits(v, p, 2, mi)) return false;
  p += 2;
  if (p >= v.size() || v[p] != ':') return false;
  ++p;
  if (!go_digits(v, p, 2, sec)) return false;
  p += 2;
  int nsec = 0;
  if (p + 1 < v.size() && (v[p] == '.' || v[p] == ',') && v[p + 1] >= '0' && v[p + 1] <= '9') {
    size_t i = 0;
    while (p + i + 1 < v.size() && v[p + i + 1] >= '0' && v[p + i + 1] <= '9') ++i;
    nsec = go_parse_nanos(v.substr(p), 1 + i);
    p += 1 + i;
  }
  int64_t zone = 0;
  if (p < v.size() && v[p] == 'Z') {
    ++p;
  } else {
    if (v.size() - p < 6) return false;
    if (v[p + 3] != ':') return false;
    int hr, mm;
    if (!go_digits(v, p + 1, 2, hr) || !go_digits(v, p + 4, 2, mm)) return false;
    if (hr > 24 || mm > 60) return false;
    zone = (hr * 60 + mm) * 60;
    if (v[p] == '-') zone = -zone;
    else if (v[p] != '+') return false;
    p += 6;
  }
  if (p != v.size()) return false;
  if (month < 1 || month > 12) return false;
  if (hour >= 24 || mi >= 60 || sec >= 60) return false;
  if (day < 1 || day > go_days_in(month, year)) return false;
  out = go_make_time(year, month, day, hour, mi, sec, nsec, zone);
  return true;
}

inline bool go_parse_rfc3339nano(const std::string& s, GoTime& out) {
  if (go_parse_rfc3339_fast(s, out)) return true;
  return go_parse_rfc3339_generic(s, out);
}

// time.Time.Sub with Go's saturation to [minDuration, maxDuration]
inline int64_t go_time_sub(const GoTime& t, int64_t now_ns) {
  __int128 tn = (__int128)t.sec * 1000000000 + t.nsec;
  __int128 d = tn - (__int128)now_ns;
  if (d > (__int128)INT64_MAX) return INT64_MAX;
  if (d < (__int128)INT64_MIN) return INT64_MIN;
  return (int64_t)d;
}

// Go float64 -> int64 conversion as compiled for amd64 (CVTTSD2SQ): out-of-range and NaN
// give 0x8000000000000000 (value_int_from.go:73 `int64(t)`).
inline int64_t go_f64_to_i64(double x) {
  if (!(x >= -9223372036854775808.0 && x < 9223372036854775808.0)) return INT64_MIN;
  return (int64_t)x;
}

}  // namespace refcpu
