// Label selectors for need()'s disregard filters, native form of kwok_amd/host/labelsel.py.
//
// Reference: pkg/kwok/controllers/pod_controller.go:392-409, node_controller.go:153-166 (a selector
// applies to a non-empty annotation / label map), controllers/utils.go:116-121 (labelsParse: "" ->
// no selector, else k8s.io/apimachinery v0.30.2 labels.Parse, restated from its published
// selector.go: requirements joined by ',', key / !key / = == != / in notin (...) / > <; NotIn and
// != match a missing key; "()" means {""}; keys qualified names, values label values).
#pragma once
#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

#include "json_dom.hpp"

namespace kwklabels {

struct SelectorError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

enum Tok : uint8_t { ID, IN, NOTIN, NOT, NEQ, EQ, DEQ, GT, LT, OPEN, CLOSE, COMMA, END };

inline bool ws(char c) { return c == ' ' || c == '\t' || c == '\r' || c == '\n'; }
inline bool special(char c) { return c == '=' || c == '!' || c == '(' || c == ')' || c == ',' || c == '>' || c == '<'; }

inline bool parse_int10(const std::string& s, long long& v) {  // strconv.ParseInt(s, 10, 64)
  size_t i = 0;
  if (s.empty()) return false;
  bool neg = false;
  if (s[0] == '+' || s[0] == '-') { neg = s[0] == '-'; i = 1; }
  if (i >= s.size()) return false;
  unsigned __int128 x = 0;
  for (; i < s.size(); ++i) {
    if (s[i] < '0' || s[i] > '9') return false;
    x = x * 10 + (unsigned)(s[i] - '0');
    if (x > ((unsigned __int128)1 << 64)) return false;
  }
  if (!neg && x >= ((unsigned __int128)1 << 63)) return false;
  if (neg && x > ((unsigned __int128)1 << 63)) return false;
  v = neg ? (long long)(-(__int128)x) : (long long)x;
  return true;
}

inline bool alnum(char c) { return (c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z') || (c >= '0' && c <= '9'); }

// ([A-Za-z0-9][-A-Za-z0-9_.]*)?[A-Za-z0-9] (and empty when allow_empty)
inline bool qname(const std::string& s, bool allow_empty) {
  if (s.empty()) return allow_empty;
  if (!alnum(s.front()) || !alnum(s.back())) return false;
  for (char c : s)
    if (!(alnum(c) || c == '-' || c == '_' || c == '.')) return false;
  return true;
}

inline bool dns1123_subdomain(const std::string& s) {
  if (s.empty() || s.size() > 253) return false;
  size_t p = 0;
  for (;;) {
    const size_t q = s.find('.', p);
    const std::string part = s.substr(p, q == std::string::npos ? std::string::npos : q - p);
    if (part.empty()) return false;
    auto lo = [](char c) { return (c >= 'a' && c <= 'z') || (c >= '0' && c <= '9'); };
    if (!lo(part.front()) || !lo(part.back())) return false;
    for (char c : part)
      if (!(lo(c) || c == '-')) return false;
    if (q == std::string::npos) return true;
    p = q + 1;
  }
}

inline void check_key(const std::string& k) {
  const size_t sl = k.find('/');
  std::string name = k;
  if (sl != std::string::npos) {
    if (k.find('/', sl + 1) != std::string::npos) throw SelectorError("invalid label key '" + k + "'");
    const std::string prefix = k.substr(0, sl);
    name = k.substr(sl + 1);
    if (!dns1123_subdomain(prefix)) throw SelectorError("invalid label key '" + k + "': bad prefix");
  }
  if (name.empty() || name.size() > 63 || !qname(name, false)) throw SelectorError("invalid label key '" + k + "'");
}

inline void check_value(const std::string& v) {
  if (v.size() > 63 || !qname(v, true)) throw SelectorError("invalid label value '" + v + "'");
}

struct Requirement {
  std::string key;
  std::string op;  // in notin = == != exists ! gt lt
  std::vector<std::string> values;  // sorted, unique

  bool has_value(const std::string& v) const { return std::binary_search(values.begin(), values.end(), v); }

  bool matches(const std::map<std::string, std::string>& ls) const {
    const auto it = ls.find(key);
    const bool has = it != ls.end();
    if (op == "in" || op == "=" || op == "==") return has && has_value(it->second);
    if (op == "notin" || op == "!=") return !has || !has_value(it->second);
    if (op == "exists") return has;
    if (op == "!") return !has;
    if (!has) return false;
    long long v, r;
    if (!parse_int10(it->second, v) || values.size() != 1 || !parse_int10(values[0], r)) return false;
    return op == "gt" ? v > r : v < r;
  }
};

struct Selector {
  std::vector<Requirement> reqs;
  std::vector<std::pair<Tok, std::string>> t;
  size_t p = 0;

  explicit Selector(const std::string& text) {
    lex(text);
    for (;;) {
      const auto lk = look(true);
      if (lk.first == ID || lk.first == NOT) {
        reqs.push_back(requirement());
        const auto k2 = take(true);
        if (k2.first == END) break;
        if (k2.first == COMMA) {
          const auto k3 = look(true);
          if (k3.first != ID && k3.first != NOT) throw SelectorError("found '" + k3.second + "', expected: identifier after ','");
          continue;
        }
        throw SelectorError("found '" + k2.second + "', expected: ',' or 'end of string'");
      }
      if (lk.first == END) break;
      throw SelectorError("found '" + lk.second + "', expected: !, identifier, or 'end of string'");
    }
  }

  void lex(const std::string& s) {
    size_t i = 0;
    while (i < s.size()) {
      const char c = s[i];
      if (ws(c)) { ++i; continue; }
      if (special(c)) {
        const std::string two = s.substr(i, 2);
        if (two == "!=") { t.emplace_back(NEQ, two); i += 2; continue; }
        if (two == "==") { t.emplace_back(DEQ, two); i += 2; continue; }
        static const std::pair<char, Tok> one[] = {{'!', NOT}, {'(', OPEN}, {')', CLOSE}, {',', COMMA}, {'=', EQ}, {'>', GT}, {'<', LT}};
        for (const auto& o : one)
          if (o.first == c) t.emplace_back(o.second, std::string(1, c));
        ++i;
        continue;
      }
      size_t j = i;
      while (j < s.size() && !ws(s[j]) && !special(s[j])) ++j;
      const std::string lit = s.substr(i, j - i);
      t.emplace_back(lit == "in" ? IN : lit == "notin" ? NOTIN : ID, lit);
      i = j;
    }
    t.emplace_back(END, "");
  }
  std::pair<Tok, std::string> look(bool values) const {
    auto r = t[p];
    if (values && (r.first == IN || r.first == NOTIN)) r.first = ID;
    return r;
  }
  std::pair<Tok, std::string> take(bool values) {
    auto r = look(values);
    ++p;
    return r;
  }

  Requirement requirement() {
    Requirement R;
    bool neg = false;
    auto k = take(true);
    if (k.first == NOT) {
      neg = true;
      k = take(true);
    }
    if (k.first != ID) throw SelectorError("found '" + k.second + "', expected: identifier");
    R.key = k.second;
    check_key(R.key);
    const Tok nx = look(true).first;
    if (nx == END || nx == COMMA) {
      R.op = neg ? "!" : "exists";
      return R;
    }
    if (neg) {
      R.op = "!";
      return R;
    }
    const auto o = take(false);
    switch (o.first) {
      case IN: R.op = "in"; break;
      case NOTIN: R.op = "notin"; break;
      case EQ: R.op = "="; break;
      case DEQ: R.op = "=="; break;
      case NEQ: R.op = "!="; break;
      case GT: R.op = "gt"; break;
      case LT: R.op = "lt"; break;
      default: throw SelectorError("found '" + o.second + "', expected: one of in, notin, =, ==, !=, gt, lt");
    }
    std::vector<std::string> vals;
    if (R.op == "in" || R.op == "notin") {
      if (take(true).first != OPEN) throw SelectorError("expected: '('");
      const auto lk = look(true);
      if (lk.first == CLOSE) {
        take(true);
        vals.push_back("");
      } else if (lk.first == ID || lk.first == COMMA) {
        for (;;) {
          const auto x = take(true);
          if (x.first == ID) {
            vals.push_back(x.second);
            const auto y = look(true);
            if (y.first == COMMA) continue;
            if (y.first == CLOSE) break;
            throw SelectorError("found '" + y.second + "', expected: ',' or ')'");
          } else if (x.first == COMMA) {
            if (vals.empty()) vals.push_back("");
            const Tok y = look(true).first;
            if (y == CLOSE) { vals.push_back(""); break; }
            if (y == COMMA) { take(true); vals.push_back(""); }
          } else {
            throw SelectorError("found '" + x.second + "', expected: ',', or identifier");
          }
        }
        if (take(true).first != CLOSE) throw SelectorError("expected: ')'");
      } else {
        throw SelectorError("found '" + lk.second + "', expected: ',', ')' or identifier");
      }
    } else {
      const auto lk = look(true);
      if (lk.first == END || lk.first == COMMA) {
        vals.push_back("");
      } else {
        const auto x = take(true);
        if (x.first != ID) throw SelectorError("found '" + x.second + "', expected: identifier");
        vals.push_back(x.second);
      }
    }
    std::sort(vals.begin(), vals.end());
    vals.erase(std::unique(vals.begin(), vals.end()), vals.end());
    if ((R.op == "in" || R.op == "notin") && vals.empty()) throw SelectorError("for 'in', 'notin' operators, values set can't be empty");
    if ((R.op == "=" || R.op == "==" || R.op == "!=") && vals.size() != 1)
      throw SelectorError("exact-match compatibility requires one single value");
    long long dummy;
    if ((R.op == "gt" || R.op == "lt") && (vals.size() != 1 || !parse_int10(vals[0], dummy)))
      throw SelectorError("for 'Gt', 'Lt' operators, the value must be an integer");
    for (const std::string& v : vals) check_value(v);
    R.values = vals;
    return R;
  }

  bool matches(const std::map<std::string, std::string>& ls) const {
    for (const Requirement& r : reqs)
      if (!r.matches(ls)) return false;
    return true;
  }
};

// need()'s selector part (pod_controller.go:397-407): the object is disregarded when a configured
// selector matches its non-empty annotation / label map
struct Disregard {
  bool has_ann = false, has_lab = false;
  std::string ann_text, lab_text;
  std::vector<Selector> sel;  // [ann][lab] as configured

  Disregard() = default;
  Disregard(const std::string& ann, const std::string& lab) : ann_text(ann), lab_text(lab) {
    if (!ann.empty()) { has_ann = true; sel.emplace_back(ann); }
    if (!lab.empty()) { has_lab = true; sel.emplace_back(lab); }
  }
  bool active() const { return has_ann || has_lab; }

  static std::map<std::string, std::string> str_map(const kwkjson::JV* m) {
    std::map<std::string, std::string> out;
    if (!m || m->t != kwkjson::JV::OBJ) return out;
    for (size_t i = 0; i < m->k.size(); ++i) {
      const kwkjson::JV& v = m->a[i];
      out[m->k[i]] = v.t == kwkjson::JV::STR ? v.s : v.t == kwkjson::JV::BOOL ? (v.b ? "True" : "False") : v.s;
    }
    return out;
  }

  bool disregarded(const kwkjson::JV& obj) const {
    const kwkjson::JV* md = obj.t == kwkjson::JV::OBJ ? obj.get("metadata") : nullptr;
    if (!md || md->t != kwkjson::JV::OBJ) return false;
    size_t k = 0;
    if (has_ann) {
      const auto m = str_map(md->get("annotations"));
      if (!m.empty() && sel[k].matches(m)) return true;
      ++k;
    }
    if (has_lab) {
      const auto m = str_map(md->get("labels"));
      if (!m.empty() && sel[k].matches(m)) return true;
    }
    return false;
  }
};

}  // namespace kwklabels
