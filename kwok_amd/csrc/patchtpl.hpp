// Merge-patch byte-template compiler: the native form of kwok_amd/host/patchtpl.py
// (TemplateCompiler / PatchProgram), producing the spec libkwok_patch (patch.cpp) interprets.
//
// Reference: the per-fired-object patch of playStage — Next.Patches (next.go:73-160) renders each
// Stage patch template with text/template + sprig (gotpl/renderer.go:59-124) and wraps it under
// the patch's root key.  A template is compiled once: its YAML block structure resolved at compile
// time (mapping keys in encoding/json's sorted order, literal scalars as their final JSON bytes,
// `key:` followed by items from ranges a lazily opened array); only the slots stay dynamic.
// Program nodes and expressions are the Python compiler's, byte for byte in the spec JSON.
#pragma once
#include <algorithm>
#include <map>
#include <set>
#include <string>
#include <vector>

#include "gotpl.hpp"

namespace kwkpatch {

using kwkjson::JV;
using kwktpl::Node;
using kwktpl::Operand;
using kwktpl::Pipe;
using kwktpl::TplError;

// ------------------------------------------------------------------ Python json.dumps values
struct PJ {
  enum K : uint8_t { NUL, BOOL, INT, STR, LIST, DICT, RAW } k = NUL;
  bool b = false;
  long long i = 0;
  std::string s;  // STR / RAW (pre-rendered JSON text)
  std::vector<PJ> l;
  std::vector<std::pair<std::string, PJ>> d;

  static PJ null() { return PJ(); }
  static PJ boolean(bool x) { PJ p; p.k = BOOL; p.b = x; return p; }
  static PJ integer(long long x) { PJ p; p.k = INT; p.i = x; return p; }
  static PJ str(std::string x) { PJ p; p.k = STR; p.s = std::move(x); return p; }
  static PJ raw(std::string x) { PJ p; p.k = RAW; p.s = std::move(x); return p; }
  static PJ list(std::vector<PJ> x = {}) { PJ p; p.k = LIST; p.l = std::move(x); return p; }
  static PJ dict() { PJ p; p.k = DICT; return p; }
  PJ& set(const std::string& key, PJ v) {
    for (auto& kv : d)
      if (kv.first == key) { kv.second = std::move(v); return *this; }
    d.emplace_back(key, std::move(v));
    return *this;
  }
  PJ& push(PJ v) { l.push_back(std::move(v)); return *this; }
};

// json.dumps(v) with the default separators (", ", ": ") and ensure_ascii
inline void pj_dump(std::string& o, const PJ& v) {
  switch (v.k) {
    case PJ::NUL: o += "null"; return;
    case PJ::BOOL: o += v.b ? "true" : "false"; return;
    case PJ::INT: o += std::to_string(v.i); return;
    case PJ::STR: kwkhost::esc(o, v.s); return;
    case PJ::RAW: o += v.s; return;
    case PJ::LIST:
      o += '[';
      for (size_t i = 0; i < v.l.size(); ++i) {
        if (i) o += ", ";
        pj_dump(o, v.l[i]);
      }
      o += ']';
      return;
    case PJ::DICT:
      o += '{';
      for (size_t i = 0; i < v.d.size(); ++i) {
        if (i) o += ", ";
        kwkhost::esc(o, v.d[i].first);
        o += ": ";
        pj_dump(o, v.d[i].second);
      }
      o += '}';
      return;
  }
}

// a JV as Python holds it after json.loads, for json.dumps (numbers in Python's text)
inline PJ pj_of(const JV& v) {
  switch (v.t) {
    case JV::NUL: return PJ::null();
    case JV::BOOL: return PJ::boolean(v.b);
    case JV::NUM: return PJ::raw(kwktpl::py_num_text(v));
    case JV::STR: return PJ::str(v.s);
    case JV::ARR: {
      PJ l = PJ::list();
      for (const JV& x : v.a) l.push(pj_of(x));
      return l;
    }
    case JV::OBJ: {
      PJ d = PJ::dict();
      for (size_t i = 0; i < v.k.size(); ++i) d.set(v.k[i], pj_of(v.a[i]));
      return d;
    }
  }
  return PJ();
}

struct Unsupported : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// ------------------------------------------------------------------ template -> line entries
// pieces: ("t", text) | ("v", pipe) | ("a", pipe) | ("r", pipe, pieces)
struct Piece {
  char k;  // 't' 'v' 'a' 'r'
  std::string text;
  const Pipe* pipe = nullptr;
  std::vector<Piece> sub;
};
// entries: line (indent, pieces) | block (kind, pipe, body, else) | assign (pipe)
struct Entry {
  enum K : uint8_t { LINE, BLOCK, ASSIGN } k = LINE;
  int indent = 0;
  std::vector<Piece> pieces;
  Node::K kind = Node::IF;
  const Pipe* pipe = nullptr;
  std::vector<Entry> body, els;
};

inline bool blank(const std::string& s) { return kwktpl::py_strip(s).empty(); }

inline bool is_ws(const std::vector<Piece>& ps) {
  for (const Piece& p : ps)
    if (p.k != 't' || !blank(p.text)) return false;
  return true;
}

inline bool body_starts_line(const std::vector<Node>& nodes) {
  for (const Node& n : nodes) {
    if (n.k == Node::TEXT) {
      const size_t nl = n.text.find('\n');
      const std::string head = n.text.substr(0, nl);
      return blank(head) && nl != std::string::npos;
    }
    return false;
  }
  return true;
}

inline std::vector<Piece> inline_pieces(const std::vector<Node>& nodes) {
  std::vector<Piece> out;
  for (const Node& n : nodes) {
    if (n.k == Node::TEXT) {
      if (n.text.find('\n') != std::string::npos) throw Unsupported("inline range spanning lines");
      out.push_back({'t', n.text});
    } else if (n.k == Node::ACTION && !n.pipe.has_decl) {
      out.push_back({'v', "", &n.pipe});
    } else if (n.k == Node::RANGE && !n.has_else) {
      Piece p{'r', "", &n.pipe};
      p.sub = inline_pieces(n.body);
      out.push_back(std::move(p));
    } else {
      throw Unsupported("inline construct");
    }
  }
  return out;
}

inline std::vector<Entry> entries_of(const std::vector<Node>& nodes) {
  std::vector<Entry> out;
  std::vector<Piece> cur;
  auto flush = [&]() {
    std::vector<Piece> content;
    for (const Piece& p : cur)
      if (p.k != 't' || !blank(p.text)) content.push_back(p);
    if (content.empty()) {
    } else {
      bool any_a = false;
      for (const Piece& p : content) any_a |= p.k == 'a';
      if (any_a) {
        if (content.size() != 1) throw Unsupported("an assignment shares its line with content");
        Entry e;
        e.k = Entry::ASSIGN;
        e.pipe = content[0].pipe;
        out.push_back(std::move(e));
      } else {
        const std::string text = cur[0].k == 't' ? cur[0].text : "";
        size_t sp = 0;
        while (sp < text.size() && text[sp] == ' ') ++sp;
        Entry e;
        e.k = Entry::LINE;
        e.indent = (int)sp;
        e.pieces = cur;
        out.push_back(std::move(e));
      }
    }
    cur.clear();
  };
  for (const Node& n : nodes) {
    if (n.k == Node::TEXT) {
      size_t p = 0;
      for (;;) {
        const size_t nl = n.text.find('\n', p);
        const std::string part = n.text.substr(p, nl == std::string::npos ? std::string::npos : nl - p);
        if (!part.empty()) {
          if (!cur.empty() && cur.back().k == 't') cur.back().text += part;
          else cur.push_back({'t', part});
        }
        if (nl == std::string::npos) break;
        flush();
        p = nl + 1;
      }
    } else if (n.k == Node::ACTION) {
      cur.push_back({n.pipe.has_decl ? 'a' : 'v', "", &n.pipe});
    } else {
      if (is_ws(cur) && body_starts_line(n.body)) {
        cur.clear();
        if (n.k == Node::WITH) throw Unsupported("{{ with }}");
        if (n.k == Node::RANGE && n.has_else) throw Unsupported("{{ range }} ... {{ else }}");
        Entry e;
        e.k = Entry::BLOCK;
        e.kind = n.k;
        e.pipe = &n.pipe;
        e.body = entries_of(n.body);
        if (n.has_else) e.els = entries_of(n.els);
        out.push_back(std::move(e));
      } else {
        if (n.k != Node::RANGE || n.has_else)
          throw Unsupported(std::string("inline {{ ") + (n.k == Node::IF ? "if" : n.k == Node::WITH ? "with" : "range") + " }}");
        Piece p{'r', "", &n.pipe};
        p.sub = inline_pieces(n.body);
        cur.push_back(std::move(p));
      }
    }
  }
  flush();
  return out;
}

inline const Entry* first_line(const std::vector<Entry>& es, size_t from = 0) {
  for (size_t i = from; i < es.size(); ++i) {
    const Entry& e = es[i];
    if (e.k == Entry::LINE) return &e;
    if (e.k == Entry::BLOCK) {
      const Entry* f = first_line(e.body);
      if (!f) f = first_line(e.els);
      if (f) return f;
    }
  }
  return nullptr;
}

inline std::string lead(const Entry& line) {
  if (!line.pieces.empty() && line.pieces[0].k == 't') {
    const std::string& t = line.pieces[0].text;
    return (size_t)line.indent <= t.size() ? t.substr((size_t)line.indent) : "";
  }
  return "";
}

inline bool is_item(const Entry& line) {
  const std::string s = lead(line);
  return s.rfind("- ", 0) == 0 || s == "-";
}

// patchtpl._KEY: ^(key)[ \t]*:(?=[ \t]|$), key = [A-Za-z0-9_][A-Za-z0-9_./-]* | "..." | '...'
inline bool match_key(const std::string& s, std::string& key_src, size_t& end) {
  size_t i = 0;
  if (s.empty()) return false;
  if (s[0] == '"') {
    i = 1;
    while (i < s.size() && s[i] != '"') i += s[i] == '\\' ? 2 : 1;
    if (i >= s.size()) return false;
    ++i;
  } else if (s[0] == '\'') {
    i = 1;
    for (;;) {
      while (i < s.size() && s[i] != '\'') ++i;
      if (i >= s.size()) return false;
      if (i + 1 < s.size() && s[i + 1] == '\'') { i += 2; continue; }
      ++i;
      break;
    }
  } else {
    auto head = [](char c) { return kwktpl::is_alnum_(c); };
    auto tail = [](char c) { return kwktpl::is_alnum_(c) || c == '.' || c == '/' || c == '-'; };
    if (!head(s[0])) return false;
    i = 1;
    while (i < s.size() && tail(s[i])) ++i;
  }
  key_src = s.substr(0, i);
  size_t j = i;
  while (j < s.size() && (s[j] == ' ' || s[j] == '\t')) ++j;
  if (j >= s.size() || s[j] != ':') return false;
  if (j + 1 < s.size() && !(s[j + 1] == ' ' || s[j + 1] == '\t')) return false;
  end = j + 1;
  return true;
}

// ------------------------------------------------------------------ compiler
struct Scope {
  const Scope* parent = nullptr;
  std::map<std::string, int> vars;
  int find(const std::string& name) const {
    for (const Scope* s = this; s; s = s->parent) {
      auto it = s->vars.find(name);
      if (it != s->vars.end()) return it->second;
    }
    throw Unsupported("undefined variable " + name);
  }
};

inline bool is_builtin(const std::string& n) {
  static const char* b[] = {"or", "and", "not", "eq", "ne", "index", "dict", "len", "Quote", "Now"};
  for (const char* x : b)
    if (n == x) return true;
  return false;
}

struct TemplateCompiler {
  const std::map<std::string, int>& funcs;
  const std::map<std::string, int>& const_ids;
  std::vector<PJ> exprs;
  int n_vars = 0, n_regs = 0;
  std::map<int, int> reg_parent, reg_sibling;

  TemplateCompiler(const std::map<std::string, int>& f, const std::map<std::string, int>& c) : funcs(f), const_ids(c) {}

  int expr(PJ e) {
    exprs.push_back(std::move(e));
    return (int)exprs.size() - 1;
  }
  int var() { return n_vars++; }

  static bool is_int_literal(const std::string& s) {  // -?(0|[1-9][0-9]*)
    size_t i = s.size() && s[0] == '-' ? 1 : 0;
    if (i >= s.size()) return false;
    if (s[i] == '0') return i + 1 == s.size();
    for (; i < s.size(); ++i)
      if (!kwktpl::is_digit(s[i])) return false;
    return true;
  }

  PJ operand(const Operand& node, const Scope& scope) {
    switch (node.k) {
      case Operand::LIT: {
        const kwktpl::TV& v = node.lit;
        if (v.k == kwktpl::TV::NUM) {
          if (!is_int_literal(v.s)) throw Unsupported("number literal " + v.s);
          return PJ::dict().set("k", PJ::str("num")).set("v", PJ::str(v.s));
        }
        if (v.k == kwktpl::TV::NIL) return PJ::dict().set("k", PJ::str("nil"));
        if (v.k == kwktpl::TV::BOOL) return PJ::dict().set("k", PJ::str("bool")).set("v", PJ::boolean(v.b));
        return PJ::dict().set("k", PJ::str("str")).set("v", PJ::str(v.s));
      }
      case Operand::DOT: return PJ::dict().set("k", PJ::str("dot"));
      case Operand::VAR:
        if (node.name == "$") return PJ::dict().set("k", PJ::str("root"));
        return PJ::dict().set("k", PJ::str("var")).set("i", PJ::integer(scope.find(node.name)));
      case Operand::FIELD: {
        PJ p = PJ::list();
        for (const std::string& f : node.path) p.push(PJ::str(f));
        return PJ::dict().set("k", PJ::str("field")).set("a", PJ::list({operand(*node.base, scope)})).set("p", p);
      }
      case Operand::PAREN: return pipeline(*node.pipe, scope);
      case Operand::IDENT: return call(node.name, nullptr, 0, scope, nullptr);
    }
    throw Unsupported("operand");
  }

  PJ call(const std::string& name, const kwktpl::Cmd* cmd, size_t from, const Scope& scope, const PJ* piped) {
    PJ a = PJ::list();
    if (cmd)
      for (size_t i = from; i < cmd->size(); ++i) a.push(operand((*cmd)[i], scope));
    if (piped) a.push(*piped);
    const size_t na = a.l.size();
    auto f = funcs.find(name);
    if (f != funcs.end()) return PJ::dict().set("k", PJ::str("ext")).set("f", PJ::integer(f->second)).set("a", a);
    auto c = const_ids.find(name);
    if (c != const_ids.end()) {
      if (na) throw Unsupported(name + " with arguments");
      return PJ::dict().set("k", PJ::str("const")).set("i", PJ::integer(c->second));
    }
    if (is_builtin(name)) {
      if (((name == "dict" || name == "Now") && na) || ((name == "not" || name == "len" || name == "Quote") && na != 1) ||
          ((name == "eq" || name == "ne" || name == "index") && na < 2) || ((name == "or" || name == "and") && !na))
        throw Unsupported(name + " with " + std::to_string(na) + " arguments");
      return PJ::dict().set("k", PJ::str(name)).set("a", a);
    }
    throw Unsupported("function '" + name + "'");
  }

  PJ pipeline(const Pipe& pipe, const Scope& scope) {
    PJ val;
    bool have = false;
    for (const kwktpl::Cmd& cmd : pipe.cmds) {
      const Operand& head = cmd[0];
      if (head.k == Operand::IDENT) {
        val = call(head.name, &cmd, 1, scope, have ? &val : nullptr);
      } else {
        if (cmd.size() > 1 || have) throw Unsupported("argument to a non-function");
        val = operand(head, scope);
      }
      have = true;
    }
    return val;
  }

  static bool is_quote_ident(const Operand& o) { return o.k == Operand::IDENT && o.name == "Quote"; }

  PJ slot(const Pipe& pipe, const Scope& scope) {
    if (pipe.has_decl) throw Unsupported("assignment as a value");
    const auto& cmds = pipe.cmds;
    const kwktpl::Cmd& last = cmds.back();
    if (is_quote_ident(last[0]) && last.size() == 1 && cmds.size() > 1) {
      Pipe p2;
      p2.cmds.assign(cmds.begin(), cmds.end() - 1);
      return PJ::list({PJ::str("q"), PJ::integer(expr(pipeline(p2, scope)))});
    }
    if (is_quote_ident(last[0]) && last.size() == 2 && cmds.size() == 1)
      return PJ::list({PJ::str("q"), PJ::integer(expr(operand(last[1], scope)))});
    return PJ::list({PJ::str("raw"), PJ::integer(expr(pipeline(pipe, scope)))});
  }

  void assign(const Pipe& pipe, Scope& scope, PJ& sets) {
    if (!pipe.decl || pipe.names.size() != 1) throw Unsupported("variable re-assignment");
    Pipe p2;
    p2.cmds = pipe.cmds;
    PJ e = pipeline(p2, scope);
    const int v = var();
    scope.vars[pipe.names[0]] = v;
    sets.push(PJ::list({PJ::integer(v), PJ::integer(expr(std::move(e)))}));
  }

  std::pair<int, int> range_vars(const Pipe& pipe, Scope& scope) {
    if (!pipe.has_decl) return {-1, -1};
    if (!pipe.decl) throw Unsupported("range with '='");
    if (pipe.names.size() == 1) {
      const int ve = var();
      scope.vars[pipe.names[0]] = ve;
      return {-1, ve};
    }
    const int vi = var(), ve = var();
    scope.vars[pipe.names[0]] = vi;
    scope.vars[pipe.names[1]] = ve;
    return {vi, ve};
  }

  // -- scalars
  bool scalar(std::vector<Piece> pieces, const Scope& scope, PJ& out) {
    if (!pieces.empty() && pieces[0].k == 't') pieces[0].text = kwktpl::py_lstrip(pieces[0].text);
    if (!pieces.empty() && pieces.back().k == 't') pieces.back().text = kwktpl::py_rstrip(pieces.back().text);
    std::vector<Piece> ps;
    for (Piece& p : pieces)
      if (p.k != 't' || !p.text.empty()) ps.push_back(p);
    if (ps.empty()) return false;
    bool all_t = true;
    for (const Piece& p : ps) all_t &= p.k == 't';
    if (all_t) {
      std::string text;
      for (const Piece& p : ps) text += p.text;
      if (text.rfind("#", 0) == 0 || text.find(" #") != std::string::npos || text.find("\t#") != std::string::npos)
        throw Unsupported("YAML comment");
      JV v;
      try {
        JV doc = kwktpl::yaml_to_json("k: " + text);
        const JV* x = doc.t == JV::OBJ ? doc.get("k") : nullptr;
        if (!x) throw TplError("no value");
        v = *x;
      } catch (const TplError& e) {
        throw Unsupported(std::string("YAML literal ") + text + ": " + e.what());
      }
      std::string b;
      kwktpl::go_json_bytes(b, v);
      out = PJ::list({PJ::str("lit"), PJ::str(b)});
      return true;
    }
    if (ps.size() == 1 && ps[0].k == 'v') {
      out = slot(*ps[0].pipe, scope);
      return true;
    }
    const Piece& first = ps.front();
    const Piece& last = ps.back();
    if (ps.size() > 1 && first.k == 't' && last.k == 't' && first.text.rfind("'", 0) == 0 && !last.text.empty() &&
        last.text.back() == '\'') {
      std::vector<Piece> inner;
      inner.push_back({'t', first.text.substr(1)});
      for (size_t i = 1; i + 1 < ps.size(); ++i) inner.push_back(ps[i]);
      inner.push_back({'t', last.text.substr(0, last.text.size() - 1)});
      out = PJ::list({PJ::str("sq"), sq_pieces(inner, scope)});
      return true;
    }
    throw Unsupported("scalar mixing text and actions outside single quotes");
  }

  PJ sq_pieces(const std::vector<Piece>& pieces, const Scope& scope) {
    PJ out = PJ::list();
    for (const Piece& p : pieces) {
      if (p.k == 't') {
        std::string t = p.text, u;
        // a lone quote (not part of '') inside the scalar
        std::string stripped;
        for (size_t i = 0; i < t.size(); ++i) {
          if (t[i] == '\'' && i + 1 < t.size() && t[i + 1] == '\'') { ++i; continue; }
          stripped += t[i];
        }
        if (stripped.find('\'') != std::string::npos) throw Unsupported("quote inside a single-quoted scalar");
        for (size_t i = 0; i < t.size(); ++i) {
          u += t[i];
          if (t[i] == '\'' && i + 1 < t.size() && t[i + 1] == '\'') ++i;
        }
        if (!t.empty()) out.push(PJ::list({PJ::str("t"), PJ::str(u)}));
      } else if (p.k == 'v') {
        if (p.pipe->has_decl) throw Unsupported("assignment inside a scalar");
        out.push(PJ::list({PJ::str("v"), PJ::integer(expr(pipeline(*p.pipe, scope)))}));
      } else {
        Scope sub;
        sub.parent = &scope;
        Pipe p2;
        p2.cmds = p.pipe->cmds;
        const int it = expr(pipeline(p2, scope));
        const auto vv = range_vars(*p.pipe, sub);
        out.push(PJ::list({PJ::str("r"), PJ::integer(it), PJ::integer(vv.first), PJ::integer(vv.second),
                           sq_pieces(p.sub, sub)}));
      }
    }
    return out;
  }

  // -- block structure
  struct Item {
    std::string key;
    int reg;
    PJ node;
  };

  PJ value_after(const std::vector<Entry>& es, size_t& pos, int indent, Scope& scope, PJ& sets) {
    const Entry* nxt = first_line(es, pos);
    if (nxt && nxt->indent >= indent && is_item(*nxt)) return seq(es, pos, nxt->indent, scope, sets);
    if (nxt && nxt->indent > indent) return mapping(es, pos, nxt->indent, scope, sets, nullptr);
    return PJ::list({PJ::str("lit"), PJ::str("null")});
  }

  std::vector<int> ancestors(int r) const {
    std::vector<int> out;
    while (r != -1) {
      out.push_back(r);
      auto it = reg_parent.find(r);
      r = it == reg_parent.end() ? -1 : it->second;
    }
    return out;
  }
  bool exclusive(int a, int b) const {
    if (a == -1 || b == -1) return false;
    const std::vector<int> anc_b = ancestors(b);
    for (int x : ancestors(a)) {
      auto it = reg_sibling.find(x);
      if (it != reg_sibling.end() && std::find(anc_b.begin(), anc_b.end(), it->second) != anc_b.end()) return true;
    }
    return false;
  }

  PJ mapping(const std::vector<Entry>& es, size_t& pos, int indent, Scope& scope, PJ& sets, const Entry* first) {
    PJ guards = PJ::list();
    std::vector<Item> items;
    entries_into(es, pos, indent, scope, sets, guards, items, -1, first);
    std::map<std::string, std::vector<int>> by_key;
    for (const Item& it : items) by_key[it.key].push_back(it.reg);
    for (const auto& kv : by_key)
      for (size_t i = 0; i < kv.second.size(); ++i)
        for (size_t j = i + 1; j < kv.second.size(); ++j)
          if (!exclusive(kv.second[i], kv.second[j])) throw Unsupported("mapping key '" + kv.first + "' defined twice");
    std::stable_sort(items.begin(), items.end(), [](const Item& a, const Item& b) { return a.key < b.key; });
    PJ ents = PJ::list();
    for (Item& it : items) ents.push(PJ::list({PJ::str(kwktpl::go_json_string(it.key) + ":"), PJ::integer(it.reg), it.node}));
    return PJ::list({PJ::str("map"), guards, ents});
  }

  void entries_into(const std::vector<Entry>& es, size_t& pos, int indent, Scope& scope, PJ& sets, PJ& guards,
                    std::vector<Item>& items, int reg, const Entry* first) {
    if (first) entry(*first, es, pos, indent, scope, sets, items, reg);
    while (pos < es.size()) {
      const Entry& e = es[pos];
      if (e.k == Entry::ASSIGN) {
        if (reg != -1) throw Unsupported("assignment inside a conditional block");
        assign(*e.pipe, scope, sets);
        ++pos;
        continue;
      }
      if (e.k == Entry::BLOCK) {
        std::vector<Entry> one{e};
        const Entry* fl = first_line(one);
        if (!fl) throw Unsupported("control block without content");
        if (fl->indent < indent || is_item(*fl)) return;
        if (fl->indent > indent || e.kind != Node::IF)
          throw Unsupported(std::string("{{ ") + (e.kind == Node::IF ? "if" : e.kind == Node::RANGE ? "range" : "with") +
                            " }} around mapping entries");
        map_if(e, indent, scope, sets, guards, items, reg);
        ++pos;
        continue;
      }
      if (e.indent < indent || is_item(e)) return;
      if (e.indent > indent) throw Unsupported("unexpected indentation");
      ++pos;
      entry(e, es, pos, indent, scope, sets, items, reg);
    }
  }

  void entry(const Entry& line, const std::vector<Entry>& es, size_t& pos, int indent, Scope& scope, PJ& sets,
             std::vector<Item>& items, int reg) {
    const std::string s = lead(line);
    std::string key_src;
    size_t end;
    if (!match_key(s, key_src, end)) throw Unsupported("not a mapping entry: " + s);
    std::string key = key_src;
    if (key[0] == '"' || key[0] == '\'') {
      try {
        JV k = kwktpl::yaml_to_json(key);
        if (k.t != JV::STR) throw TplError("key");
        key = k.s;
      } catch (const TplError&) {
        throw Unsupported("mapping key " + key_src);
      }
    }
    std::vector<Piece> ps;
    ps.push_back({'t', s.substr(end)});
    for (size_t i = 1; i < line.pieces.size(); ++i) ps.push_back(line.pieces[i]);
    PJ node;
    if (!scalar(ps, scope, node)) node = value_after(es, pos, indent, scope, sets);
    items.push_back({key, reg, node});
  }

  void map_if(const Entry& block, int indent, Scope& scope, PJ& sets, PJ& guards, std::vector<Item>& items, int parent) {
    const int cond = expr(pipeline(*block.pipe, scope));
    const int rt = n_regs, re = n_regs + 1;
    n_regs += 2;
    reg_parent[rt] = reg_parent[re] = parent;
    reg_sibling[rt] = re;
    reg_sibling[re] = rt;
    guards.push(PJ::list({PJ::integer(cond), PJ::integer(rt), PJ::integer(re), PJ::integer(parent)}));
    const std::vector<Entry>* bodies[2] = {&block.body, &block.els};
    const int regs[2] = {rt, re};
    for (int b = 0; b < 2; ++b) {
      Scope sub;
      sub.parent = &scope;
      size_t p = 0;
      entries_into(*bodies[b], p, indent, sub, sets, guards, items, regs[b], nullptr);
      if (p != bodies[b]->size()) throw Unsupported("conditional block does not hold whole mapping entries");
    }
  }

  PJ seq(const std::vector<Entry>& es, size_t& pos, int indent, Scope& scope, PJ& sets) {
    PJ items = PJ::list();
    items_into(es, pos, indent, scope, sets, items);
    return PJ::list({PJ::str("seq"), items});
  }

  void items_into(const std::vector<Entry>& es, size_t& pos, int indent, Scope& scope, PJ& sets, PJ& items) {
    while (pos < es.size()) {
      const Entry& e = es[pos];
      if (e.k == Entry::ASSIGN) {
        assign(*e.pipe, scope, sets);
        ++pos;
        continue;
      }
      if (e.k == Entry::BLOCK) {
        std::vector<Entry> one{e};
        const Entry* fl = first_line(one);
        if (!fl) throw Unsupported("control block without content");
        if (fl->indent != indent || !is_item(*fl)) {
          if (fl->indent > indent) throw Unsupported("unexpected indentation");
          return;
        }
        ++pos;
        if (e.kind == Node::RANGE) {
          Scope sub;
          sub.parent = &scope;
          Pipe p2;
          p2.cmds = e.pipe->cmds;
          const int it = expr(pipeline(p2, scope));
          const auto vv = range_vars(*e.pipe, sub);
          PJ body_sets = PJ::list(), body = PJ::list();
          size_t p = 0;
          items_into(e.body, p, indent, sub, body_sets, body);
          if (p != e.body.size()) throw Unsupported("range body does not hold whole sequence items");
          items.push(PJ::list({PJ::str("range"), PJ::integer(it), PJ::integer(vv.first), PJ::integer(vv.second), body_sets, body}));
        } else {
          const int cond = expr(pipeline(*e.pipe, scope));
          PJ branches[2];
          const std::vector<Entry>* bodies[2] = {&e.body, &e.els};
          for (int b = 0; b < 2; ++b) {
            Scope sub;
            sub.parent = &scope;
            PJ bsets = PJ::list(), bitems = PJ::list();
            size_t p = 0;
            items_into(*bodies[b], p, indent, sub, bsets, bitems);
            if (p != bodies[b]->size()) throw Unsupported("if body does not hold whole sequence items");
            if (!bsets.l.empty()) throw Unsupported("assignment inside a conditional block");
            branches[b] = bitems;
          }
          items.push(PJ::list({PJ::str("if"), PJ::integer(cond), branches[0], branches[1]}));
        }
        continue;
      }
      if (e.indent != indent || !is_item(e)) {
        if (e.indent > indent) throw Unsupported("unexpected indentation");
        return;
      }
      const std::string rest0 = lead(e).substr(1);
      size_t sp = 0;
      while (sp < rest0.size() && rest0[sp] == ' ') ++sp;
      const int inner = e.indent + 1 + (int)sp;
      const std::string rest = rest0.substr(sp);
      std::string ks;
      size_t kend;
      PJ node;
      if (match_key(rest, ks, kend)) {
        Entry first;
        first.k = Entry::LINE;
        first.indent = inner;
        first.pieces.push_back({'t', std::string((size_t)inner, ' ') + rest});
        for (size_t i = 1; i < e.pieces.size(); ++i) first.pieces.push_back(e.pieces[i]);
        ++pos;
        node = mapping(es, pos, inner, scope, sets, &first);
      } else {
        std::vector<Piece> ps;
        ps.push_back({'t', rest});
        for (size_t i = 1; i < e.pieces.size(); ++i) ps.push_back(e.pieces[i]);
        if (!scalar(ps, scope, node)) throw Unsupported("nested block sequence item");
        ++pos;
      }
      items.push(PJ::list({PJ::str("item"), node}));
    }
  }

  PJ compile(const std::string& text, const std::string& root) {
    const std::vector<Node> tree = kwktpl::parse_template(kwktpl::py_strip(text));
    const std::vector<Entry> es = entries_of(tree);
    const Entry* fl = first_line(es);
    if (!fl || is_item(*fl)) throw Unsupported("template is not a mapping");
    PJ sets = PJ::list();
    Scope top;
    size_t pos = 0;
    PJ node = mapping(es, pos, fl->indent, top, sets, nullptr);
    if (pos != es.size()) throw Unsupported("content after the top-level mapping");
    PJ ex = PJ::list(exprs);
    return PJ::dict()
        .set("n_vars", PJ::integer(n_vars))
        .set("n_regs", PJ::integer(n_regs))
        .set("exprs", ex)
        .set("prologue", sets)
        .set("head", PJ::str(root.empty() ? "" : "{" + kwktpl::go_json_string(root) + ":"))
        .set("body", node)
        .set("tail", PJ::str(root.empty() ? "" : "}"));
  }
};

}  // namespace kwkpatch
