// ORACLE / TEST INFRASTRUCTURE — not product code.
// A jq-subset interpreter restating the behaviour KWOK gets from
// github.com/itchyny/gojq v0.12.16 (go.mod:17; not vendored in /root/reference) for the
// query forms KWOK's Stage CRs and tests use:
//   paths `.a.b`, `.a["k"]`, `."k"`, `.a.[]`, `.a[]`, `.[n]`, pipes `|`, `,`,
//   `select(f)`, comparisons, `and`/`or`/`not`, `//`, literals, `[...]`, `{...}`,
//   `length`, `empty`, `has(k)`, `keys`, `type`, `if-then-elif-else-end`, unary `-`, and the
//   update forms `p = v`, `p += v` exercised by pkg/utils/expression/query_test.go:127-166.
// gojq's value model: JSON input numbers are float64, number literals / `length` / int
// arithmetic give ints (JV::integer) — selector.go hasValue matches ints (FormatInt), never
// float64s; objects iterate and list their keys sorted (gojq holds them in Go maps).
// Call sites restated: Query.Execute (pkg/utils/expression/query.go:48-69): a runtime error
// makes the whole result nil; null outputs are dropped.
#pragma once
#include <algorithm>
#include <climits>
#include <functional>
#include <map>

#include "json.hpp"

namespace refcpu {

struct JqError : std::runtime_error { using std::runtime_error::runtime_error; };

struct JqNode {
  enum K {
    IDENT,     // .
    FIELD,     // <sub>.name   (sub may be null => input)
    INDEX,     // <sub>[expr]
    ITER,      // <sub>[]
    PIPE, COMMA, ALT, OR, AND, NOT_FN, CMP, ADD, SUB,
    LIT, ARRAY, OBJECT, SELECT, LENGTH, EMPTY, ASSIGN, UPDATE_ADD, TRY,
    HAS, KEYS, TYPE, IF, NEG
  } k;
  std::string name;  // FIELD name / CMP op
  JVP lit;
  std::shared_ptr<JqNode> a, b;  // operands (a = sub-expression / lhs)
  std::vector<std::pair<std::shared_ptr<JqNode>, std::shared_ptr<JqNode>>> obj;  // OBJECT entries
  std::vector<std::shared_ptr<JqNode>> branches;  // IF: cond, then, cond, then, ..., [else]
};
using JqNodeP = std::shared_ptr<JqNode>;

class JqParser {
 public:
  explicit JqParser(const std::string& s) : s_(s) {}
  JqNodeP parse() {
    JqNodeP n = pipe();
    ws();
    if (i_ != s_.size()) throw JqError("unexpected token at " + std::to_string(i_) + " in " + s_);
    return n;
  }

 private:
  const std::string& s_;
  size_t i_ = 0;
  static JqNodeP mk(JqNode::K k) { auto n = std::make_shared<JqNode>(); n->k = k; return n; }
  void ws() { while (i_ < s_.size() && isspace((unsigned char)s_[i_])) ++i_; }
  bool peek(const char* t) { ws(); size_t n = strlen(t); return s_.compare(i_, n, t) == 0; }
  bool eat(const char* t) { if (peek(t)) { i_ += strlen(t); return true; } return false; }
  bool eat_kw(const char* t) {
    ws();
    size_t n = strlen(t);
    if (s_.compare(i_, n, t) != 0) return false;
    if (i_ + n < s_.size() && (isalnum((unsigned char)s_[i_ + n]) || s_[i_ + n] == '_')) return false;
    i_ += n;
    return true;
  }
  std::string ident() {
    size_t st = i_;
    while (i_ < s_.size() && (isalnum((unsigned char)s_[i_]) || s_[i_] == '_')) ++i_;
    if (st == i_) throw JqError("expected identifier in " + s_);
    return s_.substr(st, i_ - st);
  }
  std::string strlit() {
    // jq string literal with JSON escapes (no interpolation support)
    size_t st = i_;
    if (s_[i_] != '"') throw JqError("expected string");
    ++i_;
    while (i_ < s_.size() && s_[i_] != '"') { if (s_[i_] == '\\') ++i_; ++i_; }
    if (i_ >= s_.size()) throw JqError("unterminated string");
    ++i_;
    return parse_json(s_.substr(st, i_ - st))->s;
  }
  JqNodeP pipe() {
    JqNodeP l = comma();
    if (eat("|") ) {
      if (i_ < s_.size() && s_[i_] == '=') throw JqError("|= unsupported");
      auto n = mk(JqNode::PIPE); n->a = l; n->b = pipe(); return n;
    }
    return l;
  }
  // jq precedence, loosest first: '|', ',', '//' (right), '=' / '+=' (non-assoc), or, and, comparisons
  JqNodeP comma() {
    JqNodeP l = alt();
    while (true) {
      ws();
      if (i_ < s_.size() && s_[i_] == ',') { ++i_; auto n = mk(JqNode::COMMA); n->a = l; n->b = alt(); l = n; }
      else return l;
    }
  }
  JqNodeP alt() {
    JqNodeP l = assign();
    if (eat("//")) { auto n = mk(JqNode::ALT); n->a = l; n->b = alt(); return n; }
    return l;
  }
  JqNodeP assign() {
    JqNodeP l = orx();
    ws();
    if (s_.compare(i_, 2, "+=") == 0) { i_ += 2; auto n = mk(JqNode::UPDATE_ADD); n->a = l; n->b = orx(); return n; }
    if (i_ < s_.size() && s_[i_] == '=' && s_.compare(i_, 2, "==") != 0) { ++i_; auto n = mk(JqNode::ASSIGN); n->a = l; n->b = orx(); return n; }
    return l;
  }
  JqNodeP orx() {
    JqNodeP l = andx();
    while (eat_kw("or")) { auto n = mk(JqNode::OR); n->a = l; n->b = andx(); l = n; }
    return l;
  }
  JqNodeP andx() {
    JqNodeP l = cmp();
    while (eat_kw("and")) { auto n = mk(JqNode::AND); n->a = l; n->b = cmp(); l = n; }
    return l;
  }
  JqNodeP cmp() {
    JqNodeP l = additive();
    static const char* ops[] = {"==", "!=", "<=", ">=", "<", ">"};
    for (const char* op : ops) {
      if (peek(op)) {
        i_ += strlen(op);
        auto n = mk(JqNode::CMP); n->name = op; n->a = l; n->b = additive(); return n;
      }
    }
    return l;
  }
  JqNodeP additive() {
    JqNodeP l = postfix();
    while (true) {
      ws();
      if (i_ < s_.size() && s_[i_] == '+' && s_.compare(i_, 2, "+=") != 0) { ++i_; auto n = mk(JqNode::ADD); n->a = l; n->b = postfix(); l = n; }
      else if (i_ < s_.size() && s_[i_] == '-' && s_.compare(i_, 2, "-=") != 0) { ++i_; auto n = mk(JqNode::SUB); n->a = l; n->b = postfix(); l = n; }
      else return l;
    }
  }
  // suffix chain after a term: .name  ."str"  [expr]  []  .[expr]  .[]  ?
  JqNodeP suffixes(JqNodeP base) {
    while (true) {
      ws();
      if (i_ >= s_.size()) return base;
      char c = s_[i_];
      if (c == '.' && i_ + 1 < s_.size() && (isalpha((unsigned char)s_[i_ + 1]) || s_[i_ + 1] == '_')) {
        ++i_;
        auto n = mk(JqNode::FIELD); n->a = base; n->name = ident(); base = n; continue;
      }
      if (c == '.' && i_ + 1 < s_.size() && s_[i_ + 1] == '"') {
        ++i_;
        auto n = mk(JqNode::FIELD); n->a = base; n->name = strlit(); base = n; continue;
      }
      if (c == '.' && i_ + 1 < s_.size() && s_[i_ + 1] == '[') { ++i_; c = '['; }
      if (c == '[') {
        ++i_;
        ws();
        if (i_ < s_.size() && s_[i_] == ']') { ++i_; auto n = mk(JqNode::ITER); n->a = base; base = n; continue; }
        auto n = mk(JqNode::INDEX); n->a = base; n->b = pipe();
        if (!eat("]")) throw JqError("expected ]");
        base = n; continue;
      }
      if (c == '?') { ++i_; auto n = mk(JqNode::TRY); n->a = base; base = n; continue; }
      return base;
    }
  }
  JqNodeP postfix() {
    ws();
    if (i_ < s_.size() && s_[i_] == '-' && !(i_ + 1 < s_.size() && isdigit((unsigned char)s_[i_ + 1]))) {
      ++i_;
      auto n = mk(JqNode::NEG); n->a = postfix(); return n;
    }
    return suffixes(term());
  }
  JqNodeP term() {
    ws();
    if (i_ >= s_.size()) throw JqError("unexpected end in " + s_);
    char c = s_[i_];
    if (c == '.') {
      if (i_ + 1 < s_.size() && (isalpha((unsigned char)s_[i_ + 1]) || s_[i_ + 1] == '_' || s_[i_ + 1] == '"' || s_[i_ + 1] == '[')) {
        return mk(JqNode::IDENT);  // suffixes() consumes the .name/.["x"]/.[...]
      }
      ++i_;
      return mk(JqNode::IDENT);
    }
    if (c == '"') { auto n = mk(JqNode::LIT); n->lit = JV::str(strlit()); return n; }
    if (isdigit((unsigned char)c) || (c == '-' && i_ + 1 < s_.size() && isdigit((unsigned char)s_[i_ + 1]))) {
      size_t st = i_;
      ++i_;
      bool frac = false;
      while (i_ < s_.size() && (isdigit((unsigned char)s_[i_]) || s_[i_] == '.' || s_[i_] == 'e' || s_[i_] == 'E')) {
        frac |= !isdigit((unsigned char)s_[i_]);
        ++i_;
      }
      const std::string t = s_.substr(st, i_ - st);
      auto n = mk(JqNode::LIT);
      // gojq: a literal that fits an int is an int
      n->lit = !frac && t.size() < 19 ? JV::integer(strtoll(t.c_str(), nullptr, 10)) : JV::number(strtod(t.c_str(), nullptr));
      return n;
    }
    if (c == '(') { ++i_; JqNodeP n = pipe(); if (!eat(")")) throw JqError("expected )"); return n; }
    if (c == '[') {
      ++i_;
      auto n = mk(JqNode::ARRAY);
      if (!eat("]")) { n->a = pipe(); if (!eat("]")) throw JqError("expected ]"); }
      return n;
    }
    if (c == '{') {
      ++i_;
      auto n = mk(JqNode::OBJECT);
      if (eat("}")) return n;
      while (true) {
        ws();
        JqNodeP key;
        if (s_[i_] == '"') { key = mk(JqNode::LIT); key->lit = JV::str(strlit()); }
        else { key = mk(JqNode::LIT); key->lit = JV::str(ident()); }
        JqNodeP val;
        if (eat(":")) val = alt();
        else { val = mk(JqNode::FIELD); val->a = nullptr; val->name = key->lit->s; }
        n->obj.emplace_back(key, val);
        if (eat(",")) continue;
        if (eat("}")) return n;
        throw JqError("expected , or }");
      }
    }
    if (eat_kw("true")) { auto n = mk(JqNode::LIT); n->lit = JV::boolean(true); return n; }
    if (eat_kw("false")) { auto n = mk(JqNode::LIT); n->lit = JV::boolean(false); return n; }
    if (eat_kw("null")) { auto n = mk(JqNode::LIT); n->lit = JV::null(); return n; }
    if (eat_kw("select")) {
      if (!eat("(")) throw JqError("expected ( after select");
      auto n = mk(JqNode::SELECT); n->a = pipe();
      if (!eat(")")) throw JqError("expected )");
      return n;
    }
    if (eat_kw("not")) return mk(JqNode::NOT_FN);
    if (eat_kw("length")) return mk(JqNode::LENGTH);
    if (eat_kw("empty")) return mk(JqNode::EMPTY);
    if (eat_kw("keys")) return mk(JqNode::KEYS);
    if (eat_kw("type")) return mk(JqNode::TYPE);
    if (eat_kw("has")) {
      if (!eat("(")) throw JqError("expected ( after has");
      auto n = mk(JqNode::HAS); n->a = pipe();
      if (!eat(")")) throw JqError("expected )");
      return n;
    }
    if (eat_kw("if")) {
      auto n = mk(JqNode::IF);
      while (true) {
        n->branches.push_back(pipe());
        if (!eat_kw("then")) throw JqError("expected then");
        n->branches.push_back(pipe());
        if (eat_kw("elif")) continue;
        if (eat_kw("else")) n->branches.push_back(pipe());
        if (!eat_kw("end")) throw JqError("expected end");
        return n;
      }
    }
    throw JqError("unsupported jq syntax at " + std::to_string(i_) + " in " + s_);
  }
};

using Emit = std::function<void(const JVP&)>;
using Path = std::vector<JVP>;  // each element: string key or number index
using EmitPath = std::function<void(const Path&, const JVP&)>;

inline const char* jq_type(const JVP& v) {
  switch (v->t) {
    case JV::NUL: return "null";
    case JV::BOOL: return "boolean";
    case JV::NUM: return "number";
    case JV::STR: return "string";
    case JV::ARR: return "array";
    case JV::OBJ: return "object";
  }
  return "?";
}

// an object's entries as a Go map holds them: the last duplicate key wins, keys sorted
inline std::vector<std::pair<std::string, JVP>> jq_entries(const JVP& v) {
  std::vector<std::pair<std::string, JVP>> e;
  for (size_t i = 0; i < v->o.size(); ++i) {
    bool later = false;
    for (size_t j = i + 1; j < v->o.size(); ++j) later |= v->o[j].first == v->o[i].first;
    if (!later) e.push_back(v->o[i]);
  }
  std::sort(e.begin(), e.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
  return e;
}

inline JVP jq_index(const JVP& v, const JVP& key) {
  if (v->t == JV::NUL) return JV::null();
  if (key->t == JV::STR) {
    if (v->t != JV::OBJ) throw JqError(std::string("expected an object but got: ") + jq_type(v));
    auto* x = v->get(key->s);
    return x ? *x : JV::null();
  }
  if (key->t == JV::NUM) {
    if (v->t != JV::ARR) throw JqError(std::string("expected an array but got: ") + jq_type(v));
    long long i = (long long)std::floor(key->n);
    if (i < 0) i += (long long)v->a.size();
    if (i < 0 || i >= (long long)v->a.size()) return JV::null();
    return v->a[(size_t)i];
  }
  throw JqError("cannot index with " + std::string(jq_type(key)));
}

inline int jq_order(const JVP& v) {
  switch (v->t) {
    case JV::NUL: return 0;
    case JV::BOOL: return v->b ? 2 : 1;
    case JV::NUM: return 3;
    case JV::STR: return 4;
    case JV::ARR: return 5;
    case JV::OBJ: return 6;
  }
  return 7;
}

inline int jq_compare(const JVP& x, const JVP& y) {
  int ox = jq_order(x), oy = jq_order(y);
  if (ox != oy) return ox < oy ? -1 : 1;
  if (x->t == JV::NUM) {
    if (x->gint && y->gint) return x->i < y->i ? -1 : (x->i > y->i ? 1 : 0);
    return x->n < y->n ? -1 : (x->n > y->n ? 1 : 0);
  }
  if (x->t == JV::STR) return x->s < y->s ? -1 : (x->s > y->s ? 1 : 0);
  if (x->t == JV::ARR) {
    for (size_t i = 0; i < x->a.size() && i < y->a.size(); ++i) {
      int c = jq_compare(x->a[i], y->a[i]);
      if (c) return c;
    }
    return x->a.size() < y->a.size() ? -1 : (x->a.size() > y->a.size() ? 1 : 0);
  }
  if (x->t == JV::OBJ) {  // sorted key lists first, then the values key by key
    const auto ex = jq_entries(x), ey = jq_entries(y);
    for (size_t i = 0; i < ex.size() && i < ey.size(); ++i)
      if (ex[i].first != ey[i].first) return ex[i].first < ey[i].first ? -1 : 1;
    if (ex.size() != ey.size()) return ex.size() < ey.size() ? -1 : 1;
    for (size_t i = 0; i < ex.size(); ++i) {
      int c = jq_compare(ex[i].second, ey[i].second);
      if (c) return c;
    }
    return 0;
  }
  return 0;
}

inline JVP jq_add(const JVP& x, const JVP& y) {
  if (x->t == JV::NUL) return y;
  if (y->t == JV::NUL) return x;
  if (x->t == JV::NUM && y->t == JV::NUM) {
    long long z;
    if (x->gint && y->gint && !__builtin_add_overflow(x->i, y->i, &z)) return JV::integer(z);
    return JV::number(x->n + y->n);
  }
  if (x->t == JV::STR && y->t == JV::STR) return JV::str(x->s + y->s);
  if (x->t == JV::ARR && y->t == JV::ARR) {
    auto v = std::make_shared<JV>(*x);
    for (auto& e : y->a) v->a.push_back(e);
    return v;
  }
  if (x->t == JV::OBJ && y->t == JV::OBJ) {
    auto v = std::make_shared<JV>(*x);
    for (auto& kv : y->o) {
      bool done = false;
      for (auto& e : v->o) if (e.first == kv.first) { e.second = kv.second; done = true; }
      if (!done) v->o.push_back(kv);
    }
    return v;
  }
  throw JqError(std::string("cannot add: ") + jq_type(x) + " and " + jq_type(y));
}

inline JVP jq_setpath(const JVP& root, const Path& p, size_t i, const JVP& val) {
  if (i == p.size()) return val;
  const JVP& k = p[i];
  if (k->t == JV::STR) {
    if (root->t != JV::NUL && root->t != JV::OBJ) throw JqError("cannot set field on non-object");
    auto v = root->t == JV::OBJ ? std::make_shared<JV>(*root) : std::make_shared<JV>();
    v->t = JV::OBJ;
    for (auto& e : v->o) if (e.first == k->s) { e.second = jq_setpath(e.second, p, i + 1, val); return v; }
    v->o.emplace_back(k->s, jq_setpath(JV::null(), p, i + 1, val));
    return v;
  }
  if (root->t != JV::NUL && root->t != JV::ARR) throw JqError("cannot set index on non-array");
  auto v = root->t == JV::ARR ? std::make_shared<JV>(*root) : std::make_shared<JV>();
  v->t = JV::ARR;
  long long idx = (long long)k->n;
  if (idx < 0) idx += (long long)v->a.size();
  if (idx < 0) throw JqError("out of bounds negative array index");
  while ((long long)v->a.size() <= idx) v->a.push_back(JV::null());
  v->a[(size_t)idx] = jq_setpath(v->a[(size_t)idx], p, i + 1, val);
  return v;
}

inline JVP jq_getpath(const JVP& root, const Path& p) {
  JVP cur = root;
  for (auto& k : p) cur = jq_index(cur, k);
  return cur;
}

inline void jq_eval(const JqNode* n, const JVP& in, const Emit& emit);

// path-expression evaluation (for `=`/`+=` and nothing else)
inline void jq_paths(const JqNode* n, const JVP& in, const Path& base, const EmitPath& emit) {
  switch (n->k) {
    case JqNode::IDENT: emit(base, in); return;
    case JqNode::FIELD: {
      auto f = [&](const Path& p, const JVP& v) {
        Path q = p; q.push_back(JV::str(n->name));
        emit(q, jq_index(v, JV::str(n->name)));
      };
      if (n->a) jq_paths(n->a.get(), in, base, f); else f(base, in);
      return;
    }
    case JqNode::INDEX:
      jq_paths(n->a.get(), in, base, [&](const Path& p, const JVP& v) {
        jq_eval(n->b.get(), in, [&](const JVP& key) {
          Path q = p; q.push_back(key);
          emit(q, jq_index(v, key));
        });
      });
      return;
    case JqNode::ITER:
      jq_paths(n->a.get(), in, base, [&](const Path& p, const JVP& v) {
        if (v->t == JV::ARR) {
          for (size_t i = 0; i < v->a.size(); ++i) { Path q = p; q.push_back(JV::number((double)i)); emit(q, v->a[i]); }
        } else if (v->t == JV::OBJ) {
          for (auto& kv : jq_entries(v)) { Path q = p; q.push_back(JV::str(kv.first)); emit(q, kv.second); }
        } else if (v->t != JV::NUL) {
          throw JqError(std::string("cannot iterate over: ") + jq_type(v));
        }
      });
      return;
    case JqNode::PIPE:
      jq_paths(n->a.get(), in, base, [&](const Path& p, const JVP& v) { jq_paths(n->b.get(), v, p, emit); });
      return;
    case JqNode::SELECT: {
      bool keep = false;
      jq_eval(n->a.get(), in, [&](const JVP& c) { if (jv_truthy(c)) emit(base, in); (void)keep; });
      return;
    }
    default: throw JqError("invalid path expression");
  }
}

inline void jq_eval(const JqNode* n, const JVP& in, const Emit& emit) {
  switch (n->k) {
    case JqNode::IDENT: emit(in); return;
    case JqNode::FIELD:
      if (!n->a) { emit(jq_index(in, JV::str(n->name))); return; }
      jq_eval(n->a.get(), in, [&](const JVP& v) { emit(jq_index(v, JV::str(n->name))); });
      return;
    case JqNode::INDEX:
      jq_eval(n->a.get(), in, [&](const JVP& v) {
        jq_eval(n->b.get(), in, [&](const JVP& key) { emit(jq_index(v, key)); });
      });
      return;
    case JqNode::ITER:
      jq_eval(n->a.get(), in, [&](const JVP& v) {
        // gojq: `.[]` over null is an error ("cannot iterate over: null")
        if (v->t == JV::ARR) { for (auto& e : v->a) emit(e); }
        else if (v->t == JV::OBJ) { for (auto& kv : jq_entries(v)) emit(kv.second); }
        else throw JqError(std::string("cannot iterate over: ") + jq_type(v));
      });
      return;
    case JqNode::TRY: {  // the outputs before an error; errors of the consumer are not caught here
      std::vector<JVP> got;
      try { jq_eval(n->a.get(), in, [&](const JVP& v) { got.push_back(v); }); } catch (const JqError&) {}
      for (auto& v : got) emit(v);
      return;
    }
    case JqNode::PIPE:
      jq_eval(n->a.get(), in, [&](const JVP& v) { jq_eval(n->b.get(), v, emit); });
      return;
    case JqNode::COMMA:
      jq_eval(n->a.get(), in, emit);
      jq_eval(n->b.get(), in, emit);
      return;
    case JqNode::ALT: {
      std::vector<JVP> got;
      try {
        jq_eval(n->a.get(), in, [&](const JVP& v) { if (jv_truthy(v)) got.push_back(v); });
      } catch (const JqError&) {}
      if (got.empty()) jq_eval(n->b.get(), in, emit);
      for (auto& v : got) emit(v);
      return;
    }
    case JqNode::OR:
      jq_eval(n->a.get(), in, [&](const JVP& l) {
        if (jv_truthy(l)) { emit(JV::boolean(true)); return; }
        jq_eval(n->b.get(), in, [&](const JVP& r) { emit(JV::boolean(jv_truthy(r))); });
      });
      return;
    case JqNode::AND:
      jq_eval(n->a.get(), in, [&](const JVP& l) {
        if (!jv_truthy(l)) { emit(JV::boolean(false)); return; }
        jq_eval(n->b.get(), in, [&](const JVP& r) { emit(JV::boolean(jv_truthy(r))); });
      });
      return;
    case JqNode::NOT_FN: emit(JV::boolean(!jv_truthy(in))); return;
    case JqNode::CMP:
      // jq evaluates the right operand first in binary operators; outputs are a cartesian product
      jq_eval(n->b.get(), in, [&](const JVP& r) {
        jq_eval(n->a.get(), in, [&](const JVP& l) {
          int c = jq_compare(l, r);
          const std::string& op = n->name;
          bool res = op == "==" ? c == 0 : op == "!=" ? c != 0 : op == "<" ? c < 0 : op == "<=" ? c <= 0 : op == ">" ? c > 0 : c >= 0;
          emit(JV::boolean(res));
        });
      });
      return;
    case JqNode::ADD:
      jq_eval(n->b.get(), in, [&](const JVP& r) {
        jq_eval(n->a.get(), in, [&](const JVP& l) { emit(jq_add(l, r)); });
      });
      return;
    case JqNode::SUB:
      jq_eval(n->b.get(), in, [&](const JVP& r) {
        jq_eval(n->a.get(), in, [&](const JVP& l) {
          long long z;
          if (l->t == JV::NUM && r->t == JV::NUM && l->gint && r->gint && !__builtin_sub_overflow(l->i, r->i, &z))
            emit(JV::integer(z));
          else if (l->t == JV::NUM && r->t == JV::NUM) emit(JV::number(l->n - r->n));
          else throw JqError("cannot subtract");
        });
      });
      return;
    case JqNode::LIT: emit(n->lit); return;
    case JqNode::ARRAY: {
      auto v = std::make_shared<JV>();
      v->t = JV::ARR;
      if (n->a) jq_eval(n->a.get(), in, [&](const JVP& x) { v->a.push_back(x); });
      emit(v);
      return;
    }
    case JqNode::OBJECT: {
      // cartesian product over entry outputs (single-output entries in practice)
      std::vector<std::pair<std::string, JVP>> cur;
      std::function<void(size_t)> rec = [&](size_t i) {
        if (i == n->obj.size()) {
          auto v = std::make_shared<JV>();
          v->t = JV::OBJ;
          for (auto& kv : cur) {
            bool done = false;
            for (auto& e : v->o) if (e.first == kv.first) { e.second = kv.second; done = true; }
            if (!done) v->o.push_back(kv);
          }
          emit(v);
          return;
        }
        jq_eval(n->obj[i].first.get(), in, [&](const JVP& k) {
          if (k->t != JV::STR) throw JqError("object key must be a string");
          jq_eval(n->obj[i].second.get(), in, [&](const JVP& val) {
            cur.emplace_back(k->s, val);
            rec(i + 1);
            cur.pop_back();
          });
        });
      };
      rec(0);
      return;
    }
    case JqNode::SELECT:
      jq_eval(n->a.get(), in, [&](const JVP& c) { if (jv_truthy(c)) emit(in); });
      return;
    case JqNode::LENGTH:
      switch (in->t) {
        case JV::NUL: emit(JV::integer(0)); return;
        case JV::BOOL: throw JqError("boolean has no length");
        case JV::NUM:
          if (in->gint && in->i != LLONG_MIN) emit(JV::integer(in->i < 0 ? -in->i : in->i));
          else emit(JV::number(std::fabs(in->n)));
          return;
        case JV::STR: {
          long long cps = 0;
          for (unsigned char c : in->s) if ((c & 0xC0) != 0x80) ++cps;
          emit(JV::integer(cps));
          return;
        }
        case JV::ARR: emit(JV::integer((long long)in->a.size())); return;
        case JV::OBJ: emit(JV::integer((long long)jq_entries(in).size())); return;
      }
      return;
    case JqNode::EMPTY: return;
    case JqNode::KEYS: {
      auto v = std::make_shared<JV>();
      v->t = JV::ARR;
      if (in->t == JV::OBJ) for (auto& kv : jq_entries(in)) v->a.push_back(JV::str(kv.first));
      else if (in->t == JV::ARR) for (size_t i = 0; i < in->a.size(); ++i) v->a.push_back(JV::integer((long long)i));
      else throw JqError("keys cannot be applied to: " + std::string(jq_type(in)));
      emit(v);
      return;
    }
    case JqNode::TYPE: emit(JV::str(jq_type(in))); return;
    case JqNode::HAS:
      jq_eval(n->a.get(), in, [&](const JVP& k) {
        if (in->t == JV::OBJ && k->t == JV::STR) { emit(JV::boolean(in->get(k->s) != nullptr)); return; }
        if (in->t == JV::ARR && k->t == JV::NUM) {
          const long long i = k->gint ? k->i : (long long)k->n;
          emit(JV::boolean(i >= 0 && i < (long long)in->a.size()));
          return;
        }
        throw JqError("has cannot be applied");
      });
      return;
    case JqNode::NEG:
      jq_eval(n->a.get(), in, [&](const JVP& v) {
        if (v->t != JV::NUM) throw JqError("cannot negate");
        if (v->gint && v->i != LLONG_MIN) emit(JV::integer(-v->i));
        else emit(JV::number(-v->n));
      });
      return;
    case JqNode::IF: {
      const size_t nc = n->branches.size() / 2;
      std::function<void(size_t)> branch = [&](size_t i) {
        if (i == nc) {
          if (n->branches.size() % 2) jq_eval(n->branches.back().get(), in, emit);
          else emit(in);
          return;
        }
        jq_eval(n->branches[2 * i].get(), in, [&](const JVP& c) {
          if (jv_truthy(c)) jq_eval(n->branches[2 * i + 1].get(), in, emit);
          else branch(i + 1);
        });
      };
      branch(0);
      return;
    }
    case JqNode::ASSIGN:
      jq_eval(n->b.get(), in, [&](const JVP& val) {
        JVP out = in;
        jq_paths(n->a.get(), in, Path{}, [&](const Path& p, const JVP&) { out = jq_setpath(out, p, 0, val); });
        emit(out);
      });
      return;
    case JqNode::UPDATE_ADD:
      jq_eval(n->b.get(), in, [&](const JVP& val) {
        JVP out = in;
        jq_paths(n->a.get(), in, Path{}, [&](const Path& p, const JVP&) {
          out = jq_setpath(out, p, 0, jq_add(jq_getpath(out, p), val));
        });
        emit(out);
      });
      return;
  }
}

// Compiled query (gojq.Parse + gojq.Compile, query.go:33-45)
struct Query {
  JqNodeP root;
  std::string src;
  explicit Query(const std::string& s) : src(s) { root = JqParser(src).parse(); }
  // Query.Execute (query.go:48-69). Returns false for the `nil` result (runtime error);
  // otherwise fills `out` with the non-null outputs.
  bool execute(const JVP& v, std::vector<JVP>& out) const {
    out.clear();
    try {
      jq_eval(root.get(), v, [&](const JVP& x) { if (x->t != JV::NUL) out.push_back(x); });
    } catch (const JqError&) {
      out.clear();
      return false;
    }
    return true;
  }
};

}  // namespace refcpu
