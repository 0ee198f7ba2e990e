// JSON DOM and parser shared by the host libraries (encoder.cpp, patch.cpp).
#pragma once
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

namespace kwkjson {

struct JV {
  enum T : uint8_t { NUL, BOOL, NUM, STR, ARR, OBJ } t = NUL;
  bool b = false;
  bool is_int = false;     // a JSON number literal without fraction / exponent
  bool gint = false;       // a gojq int computed by a jq query (jqc.hpp); JSON input numbers are float64
  std::string s;           // STR: the string; NUM: the literal text
  std::vector<JV> a;       // ARR items / OBJ values
  std::vector<std::string> k;  // OBJ keys (input order; duplicate keys: the last wins on lookup)
  const JV* get(const std::string& key) const {
    for (size_t i = k.size(); i-- > 0;)
      if (k[i] == key) return &a[i];
    return nullptr;
  }
};

struct Parser {
  const char* p;
  const char* e;
  bool ok = true;
  void ws() { while (p < e && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) ++p; }
  bool lit(const char* w) {
    size_t n = strlen(w);
    if ((size_t)(e - p) < n || memcmp(p, w, n) != 0) return false;
    p += n;
    return true;
  }
  static void utf8(std::string& o, uint32_t c) {
    if (c < 0x80) o += (char)c;
    else if (c < 0x800) { o += (char)(0xC0 | (c >> 6)); o += (char)(0x80 | (c & 0x3F)); }
    else if (c < 0x10000) { o += (char)(0xE0 | (c >> 12)); o += (char)(0x80 | ((c >> 6) & 0x3F)); o += (char)(0x80 | (c & 0x3F)); }
    else { o += (char)(0xF0 | (c >> 18)); o += (char)(0x80 | ((c >> 12) & 0x3F)); o += (char)(0x80 | ((c >> 6) & 0x3F)); o += (char)(0x80 | (c & 0x3F)); }
  }
  int hex4(uint32_t& v) {
    if (e - p < 4) return 0;
    v = 0;
    for (int i = 0; i < 4; ++i) {
      char c = *p++;
      v <<= 4;
      if (c >= '0' && c <= '9') v |= c - '0';
      else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
      else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
      else return 0;
    }
    return 1;
  }
  bool str(std::string& o) {
    if (p >= e || *p != '"') return false;
    ++p;
    while (p < e && *p != '"') {
      char c = *p++;
      if (c != '\\') { o += c; continue; }
      if (p >= e) return false;
      char x = *p++;
      switch (x) {
        case '"': o += '"'; break;
        case '\\': o += '\\'; break;
        case '/': o += '/'; break;
        case 'b': o += '\b'; break;
        case 'f': o += '\f'; break;
        case 'n': o += '\n'; break;
        case 'r': o += '\r'; break;
        case 't': o += '\t'; break;
        case 'u': {
          uint32_t v;
          if (!hex4(v)) return false;
          if (v >= 0xD800 && v < 0xDC00 && e - p >= 6 && p[0] == '\\' && p[1] == 'u') {
            const char* save = p;
            p += 2;
            uint32_t lo;
            if (hex4(lo) && lo >= 0xDC00 && lo < 0xE000) v = 0x10000 + ((v - 0xD800) << 10) + (lo - 0xDC00);
            else p = save;
          }
          utf8(o, v);
          break;
        }
        default: return false;
      }
    }
    if (p >= e) return false;
    ++p;
    return true;
  }
  bool value(JV& v, int depth = 0) {
    if (depth > 256) return false;
    ws();
    if (p >= e) return false;
    char c = *p;
    if (c == '{') {
      ++p;
      v.t = JV::OBJ;
      ws();
      if (p < e && *p == '}') { ++p; return true; }
      for (;;) {
        ws();
        std::string key;
        if (!str(key)) return false;
        ws();
        if (p >= e || *p != ':') return false;
        ++p;
        v.k.push_back(std::move(key));
        v.a.emplace_back();
        if (!value(v.a.back(), depth + 1)) return false;
        ws();
        if (p < e && *p == ',') { ++p; continue; }
        if (p < e && *p == '}') { ++p; return true; }
        return false;
      }
    }
    if (c == '[') {
      ++p;
      v.t = JV::ARR;
      ws();
      if (p < e && *p == ']') { ++p; return true; }
      for (;;) {
        v.a.emplace_back();
        if (!value(v.a.back(), depth + 1)) return false;
        ws();
        if (p < e && *p == ',') { ++p; continue; }
        if (p < e && *p == ']') { ++p; return true; }
        return false;
      }
    }
    if (c == '"') { v.t = JV::STR; return str(v.s); }
    if (lit("true")) { v.t = JV::BOOL; v.b = true; return true; }
    if (lit("false")) { v.t = JV::BOOL; v.b = false; return true; }
    if (lit("null")) { v.t = JV::NUL; return true; }
    const char* b = p;
    bool frac = false;
    if (p < e && *p == '-') ++p;
    while (p < e && ((*p >= '0' && *p <= '9') || *p == '.' || *p == 'e' || *p == 'E' || *p == '+' || *p == '-')) {
      if (*p == '.' || *p == 'e' || *p == 'E') frac = true;
      ++p;
    }
    if (p == b) return false;
    v.t = JV::NUM;
    v.s.assign(b, p);
    v.is_int = !frac;
    return true;
  }
};

}  // namespace kwkjson
