// Native patch renderer: precompiled merge-patch byte templates.
//
// Reference: per fired object, playStage renders every Stage patch — Next.Patches →
// computeMergePatch → gotpl.Renderer.ToJSON → wrapMergePatchData (pkg/utils/lifecycle/
// next.go:73-160; pkg/utils/gotpl/renderer.go:59-124: the object's JSON round trip,
// text/template Execute with sprig + kwok's funcs (funcs.go:42-82), sigs.k8s.io/yaml
// YAMLToJSON = YAML decode + encoding/json Marshal: sorted keys, HTML escaping).
//
// The host compiles each template once (kwok_amd/host/patchtpl.py: TemplateCompiler) into a
// tree program whose YAML structure is already resolved: literal runs are final JSON bytes,
// mapping entries are in Go's sorted key order, and only the slots — quoted values, printed
// plain scalars, single-quoted scalars with inline ranges, range / if structure, variables and
// template functions — are evaluated here, over the object's JSON parsed once.  A value the
// program cannot place exactly (YAML would re-type a printed value, a character YAML treats
// specially) or a template execution error marks the object KWK_PATCH_NEEDS_RENDER; the host
// renders that one object with the full renderer.  Evaluation follows the product's template
// mirror (kwok_amd/host/gotpl.py), which tests/test_patch.py checks byte for byte.
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "../../include/kwok_engine.h"
#include "../../include/kwok_patch.h"
#include "json_dom.hpp"
#include "timefmt.hpp"

namespace {

using kwkjson::JV;
using kwkjson::Parser;

// the failing call's message: per handle (the call's own object, see ErrScope) and per thread
// (calls without a handle: create)
thread_local std::string g_err;
thread_local std::string* tl_err = nullptr;
struct ErrScope {
  std::string* prev;
  explicit ErrScope(std::string* target) : prev(tl_err) { tl_err = target; }
  ~ErrScope() { tl_err = prev; }
};
kwk_status fail(kwk_status code, const std::string& msg) {
  g_err = msg;
  if (tl_err) *tl_err = msg;
  return code;
}

struct NeedsRender {};  // thrown while rendering one object: fall back to the host renderer
// skeleton mode: the template's bytes depend on more than the object's class, Now and the values
// of its call sites (see kwk_patch_skeleton)
struct Ineligible {
  const char* why;
};
struct BadSpec {
  std::string what;
};

// ------------------------------------------------------------------ program
enum EK : uint8_t { E_ROOT, E_DOT, E_VAR, E_FIELD, E_NUM, E_STR, E_BOOL, E_NIL, E_CONST, E_OR, E_AND, E_NOT,
                    E_EQ, E_NE, E_INDEX, E_DICT, E_LEN, E_QUOTE, E_NOW, E_EXT };

struct Expr {
  EK k = E_NIL;
  bool b = false;
  int i = -1;
  std::string s;
  std::vector<std::string> path;
  std::vector<Expr> a;
};

enum NK : uint8_t { N_LIT, N_Q, N_RAW, N_SQ, N_MAP, N_SEQ };
enum IK : uint8_t { I_ITEM, I_RANGE, I_IF };
enum PK : uint8_t { P_TEXT, P_VAL, P_RANGE };

struct Node;
struct Set { int var, expr; };
struct Guard { int expr, then_reg, else_reg, parent; };
struct Piece {
  PK k;
  std::string text;
  int expr = -1, vi = -1, ve = -1;
  std::vector<Piece> sub;
};
struct Item;
struct Entry;
struct Node {
  NK k = N_LIT;
  std::string lit;
  int expr = -1;
  std::vector<Piece> pieces;
  std::vector<Guard> guards;
  std::vector<Entry> entries;
  std::vector<Item> items;
};
struct Entry {
  std::string key;  // "\"key\":"
  int reg = -1;
  Node node;
};
struct Item {
  IK k = I_ITEM;
  Node node;
  int expr = -1, vi = -1, ve = -1;
  std::vector<Set> sets;
  std::vector<Item> items, else_items;
};

struct Template {
  int n_vars = 0, n_regs = 0;
  std::vector<Expr> exprs;
  std::vector<Set> prologue;
  std::string head, tail;
  Node body;
};

struct Func {
  bool callback = false;
  std::string value;
};

// ------------------------------------------------------------------ spec loading
const JV& at(const JV& v, size_t i) {
  if (v.t != JV::ARR || i >= v.a.size()) throw BadSpec{"array index"};
  return v.a[i];
}
const JV& member(const JV& v, const char* k) {
  const JV* x = v.t == JV::OBJ ? v.get(k) : nullptr;
  if (!x) throw BadSpec{std::string("missing ") + k};
  return *x;
}
int num(const JV& v) {
  if (v.t != JV::NUM) throw BadSpec{"number"};
  return atoi(v.s.c_str());
}
const std::string& str(const JV& v) {
  if (v.t != JV::STR) throw BadSpec{"string"};
  return v.s;
}

Expr load_expr(const JV& j) {
  static const struct { const char* n; EK k; } kinds[] = {
      {"root", E_ROOT}, {"dot", E_DOT}, {"var", E_VAR}, {"field", E_FIELD}, {"num", E_NUM}, {"str", E_STR},
      {"bool", E_BOOL}, {"nil", E_NIL}, {"const", E_CONST}, {"or", E_OR}, {"and", E_AND}, {"not", E_NOT},
      {"eq", E_EQ}, {"ne", E_NE}, {"index", E_INDEX}, {"dict", E_DICT}, {"len", E_LEN}, {"Quote", E_QUOTE},
      {"Now", E_NOW}, {"ext", E_EXT}};
  Expr e;
  const std::string& k = str(member(j, "k"));
  bool found = false;
  for (const auto& kk : kinds)
    if (k == kk.n) { e.k = kk.k; found = true; break; }
  if (!found) throw BadSpec{"expression kind " + k};
  if (const JV* v = j.get("v")) {
    if (v->t == JV::BOOL) e.b = v->b;
    else e.s = v->s;
  }
  if (const JV* i = j.get("i")) e.i = num(*i);
  if (const JV* f = j.get("f")) e.i = num(*f);
  if (const JV* p = j.get("p"))
    for (const JV& x : p->a) e.path.push_back(str(x));
  if (const JV* a = j.get("a"))
    for (const JV& x : a->a) e.a.push_back(load_expr(x));
  return e;
}

std::vector<Set> load_sets(const JV& j) {
  std::vector<Set> out;
  for (const JV& s : j.a) out.push_back(Set{num(at(s, 0)), num(at(s, 1))});
  return out;
}

std::vector<Piece> load_pieces(const JV& j) {
  std::vector<Piece> out;
  for (const JV& p : j.a) {
    Piece x;
    const std::string& t = str(at(p, 0));
    if (t == "t") { x.k = P_TEXT; x.text = str(at(p, 1)); }
    else if (t == "v") { x.k = P_VAL; x.expr = num(at(p, 1)); }
    else if (t == "r") {
      x.k = P_RANGE;
      x.expr = num(at(p, 1));
      x.vi = num(at(p, 2));
      x.ve = num(at(p, 3));
      x.sub = load_pieces(at(p, 4));
    } else throw BadSpec{"piece " + t};
    out.push_back(std::move(x));
  }
  return out;
}

Node load_node(const JV& j);

std::vector<Item> load_items(const JV& j) {
  std::vector<Item> out;
  for (const JV& it : j.a) {
    Item x;
    const std::string& t = str(at(it, 0));
    if (t == "item") { x.k = I_ITEM; x.node = load_node(at(it, 1)); }
    else if (t == "range") {
      x.k = I_RANGE;
      x.expr = num(at(it, 1));
      x.vi = num(at(it, 2));
      x.ve = num(at(it, 3));
      x.sets = load_sets(at(it, 4));
      x.items = load_items(at(it, 5));
    } else if (t == "if") {
      x.k = I_IF;
      x.expr = num(at(it, 1));
      x.items = load_items(at(it, 2));
      x.else_items = load_items(at(it, 3));
    } else throw BadSpec{"item " + t};
    out.push_back(std::move(x));
  }
  return out;
}

Node load_node(const JV& j) {
  Node n;
  const std::string& t = str(at(j, 0));
  if (t == "lit") { n.k = N_LIT; n.lit = str(at(j, 1)); }
  else if (t == "q") { n.k = N_Q; n.expr = num(at(j, 1)); }
  else if (t == "raw") { n.k = N_RAW; n.expr = num(at(j, 1)); }
  else if (t == "sq") { n.k = N_SQ; n.pieces = load_pieces(at(j, 1)); }
  else if (t == "map") {
    n.k = N_MAP;
    for (const JV& g : at(j, 1).a) n.guards.push_back(Guard{num(at(g, 0)), num(at(g, 1)), num(at(g, 2)), num(at(g, 3))});
    for (const JV& e : at(j, 2).a) n.entries.push_back(Entry{str(at(e, 0)), num(at(e, 1)), load_node(at(e, 2))});
  } else if (t == "seq") {
    n.k = N_SEQ;
    n.items = load_items(at(j, 1));
  } else throw BadSpec{"node " + t};
  return n;
}

}  // namespace

struct kwk_patcher {
  std::string err;  // message of the last failing call on this handle
  std::vector<Template> templates;
  std::vector<Func> funcs;
  std::vector<JV> consts;
  std::string out;  // the last render's patches
  std::string skel;  // the last kwk_patch_skeleton result
};

namespace {

// ------------------------------------------------------------------ values
enum VK : uint8_t { V_MISSING, V_NIL, V_BOOL, V_NUM, V_STR, V_ARR, V_OBJ };

struct Val {
  VK k = V_MISSING;
  bool b = false;
  // skeleton mode only (see Skel): 1 = per-object data, not read (status, identity); 2 = holds
  // such data below it (the object, its metadata / spec)
  uint8_t taint = 0;
  int8_t sent = -1;     // skeleton mode: a slot's value (0 = Now, 1 + c = call site c)
  int32_t path = -1;    // skeleton mode: interned root-relative path of a value read from the object
  int32_t idx_of = -1;  // skeleton mode: a range index over the array at this path
  const std::string* sp = nullptr;  // V_NUM / V_STR text held by the DOM or the program
  std::string own;                  // computed V_NUM / V_STR text
  const JV* j = nullptr;            // V_ARR / V_OBJ
  const std::string& text() const { return sp ? *sp : own; }
};

Val from_jv(const JV* v) {
  Val r;
  if (!v) return r;
  switch (v->t) {
    case JV::NUL: r.k = V_NIL; break;
    case JV::BOOL: r.k = V_BOOL; r.b = v->b; break;
    case JV::NUM: r.k = V_NUM; r.sp = &v->s; break;
    case JV::STR: r.k = V_STR; r.sp = &v->s; break;
    case JV::ARR: r.k = V_ARR; r.j = v; break;
    case JV::OBJ: r.k = V_OBJ; r.j = v; break;
  }
  return r;
}

Val str_val(std::string s) {
  Val r;
  r.k = V_STR;
  r.own = std::move(s);
  return r;
}

// numbers reach the template as json.Number text: only canonical integers are placed here
// (other forms print differently after the host's JSON round trip)
const std::string& num_text(const Val& v) {
  const std::string& s = v.text();
  size_t i = (s.size() > 1 && s[0] == '-') ? 1 : 0;
  if (i == s.size() || s == "-0" || (s[i] == '0' && s.size() > i + 1)) throw NeedsRender{};
  for (; i < s.size(); ++i)
    if (s[i] < '0' || s[i] > '9') throw NeedsRender{};
  return s;
}

bool truth(const Val& v) {
  switch (v.k) {
    case V_MISSING:
    case V_NIL: return false;
    case V_BOOL: return v.b;
    case V_NUM:
    case V_STR: return !v.text().empty();
    case V_ARR:
    case V_OBJ: return !v.j->a.empty();
  }
  return false;
}

// encoding/json string with escapeHTML (Go 1.22); invalid UTF-8 -> the host renderer
void go_string(std::string& o, const std::string& s) {
  static const char* hex = "0123456789abcdef";
  o += '"';
  const size_t n = s.size();
  for (size_t i = 0; i < n;) {
    const unsigned char c = (unsigned char)s[i];
    if (c < 0x80) {
      switch (c) {
        case '"': o += "\\\""; break;
        case '\\': o += "\\\\"; break;
        case '\n': o += "\\n"; break;
        case '\r': o += "\\r"; break;
        case '\t': o += "\\t"; break;
        case '\b': o += "\\b"; break;
        case '\f': o += "\\f"; break;
        case '<': case '>': case '&':
          o += "\\u00";
          o += hex[c >> 4];
          o += hex[c & 15];
          break;
        default:
          if (c < 0x20) {
            o += "\\u00";
            o += hex[c >> 4];
            o += hex[c & 15];
          } else {
            o += (char)c;
          }
      }
      ++i;
      continue;
    }
    int len = (c >> 5) == 6 ? 2 : (c >> 4) == 14 ? 3 : (c >> 3) == 30 ? 4 : 0;
    if (!len || i + len > n) throw NeedsRender{};
    uint32_t cp = c & (0x7F >> len);
    for (int k = 1; k < len; ++k) {
      const unsigned char d = (unsigned char)s[i + k];
      if ((d & 0xC0) != 0x80) throw NeedsRender{};
      cp = (cp << 6) | (d & 0x3F);
    }
    if ((len == 2 && cp < 0x80) || (len == 3 && cp < 0x800) || (len == 4 && (cp < 0x10000 || cp > 0x10FFFF)) ||
        (cp >= 0xD800 && cp < 0xE000))
      throw NeedsRender{};
    if (cp == 0x2028 || cp == 0x2029) {
      o += cp == 0x2028 ? "\\u2028" : "\\u2029";
    } else {
      o.append(s, i, len);
    }
    i += len;
  }
  o += '"';
}

// characters a YAML double-quoted scalar does not carry through unchanged (PyYAML's
// printable set; NEL is a line break): such values are rendered by the host
void check_yaml_dq(const std::string& s) {
  for (size_t i = 0; i < s.size(); ++i) {
    const unsigned char c = (unsigned char)s[i];
    if (c == 0x7F) throw NeedsRender{};
    if (c == 0xC2 && i + 1 < s.size() && (unsigned char)s[i + 1] >= 0x80 && (unsigned char)s[i + 1] < 0xA0)
      throw NeedsRender{};  // U+0080..U+009F
    if (c == 0xEF && i + 2 < s.size() && (unsigned char)s[i + 1] == 0xBB && (unsigned char)s[i + 2] == 0xBF)
      throw NeedsRender{};  // U+FEFF
    if (c == 0xEF && i + 2 < s.size() && (unsigned char)s[i + 1] == 0xBF && (unsigned char)s[i + 2] >= 0xBE)
      throw NeedsRender{};  // U+FFFE, U+FFFF
  }
}

// json.Marshal of a decoded JSON value (maps: sorted keys)
void go_marshal(std::string& o, const JV& v) {
  switch (v.t) {
    case JV::NUL: o += "null"; return;
    case JV::BOOL: o += v.b ? "true" : "false"; return;
    case JV::NUM: {
      Val t;
      t.k = V_NUM;
      t.sp = &v.s;
      o += num_text(t);
      return;
    }
    case JV::STR: go_string(o, v.s); return;
    case JV::ARR:
      o += '[';
      for (size_t i = 0; i < v.a.size(); ++i) {
        if (i) o += ',';
        go_marshal(o, v.a[i]);
      }
      o += ']';
      return;
    case JV::OBJ: {
      std::vector<size_t> idx;
      for (size_t i = 0; i < v.k.size(); ++i) {
        bool last = true;  // duplicate keys: the last occurrence
        for (size_t k = i + 1; k < v.k.size(); ++k)
          if (v.k[k] == v.k[i]) { last = false; break; }
        if (last) idx.push_back(i);
      }
      std::sort(idx.begin(), idx.end(), [&](size_t a, size_t b) { return v.k[a] < v.k[b]; });
      o += '{';
      for (size_t n = 0; n < idx.size(); ++n) {
        if (n) o += ',';
        go_string(o, v.k[idx[n]]);
        o += ':';
        go_marshal(o, v.a[idx[n]]);
      }
      o += '}';
      return;
    }
  }
}

// fmt.Sprint of a template value (gotpl.go_sprint); arrays / maps print Go syntax -> host
std::string sprint(const Val& v) {
  switch (v.k) {
    case V_MISSING: return "<no value>";
    case V_NIL: return "<nil>";
    case V_BOOL: return v.b ? "true" : "false";
    case V_NUM: return num_text(v);
    case V_STR: return v.text();
    default: throw NeedsRender{};
  }
}

// funcs.go:43-55 Quote, read back by YAML: the resulting string
std::string quote_text(const Val& v) {
  switch (v.k) {
    case V_STR: return v.text();
    case V_NUM: return num_text(v);
    case V_BOOL: return v.b ? "true" : "false";
    case V_MISSING:
    case V_NIL: return "null";
    default: {
      std::string o;
      go_marshal(o, *v.j);
      return o;
    }
  }
}

// a printed value in a plain-scalar position, as YAML resolves it: canonical ints, the
// true/false spellings and plain words are placed here; everything else goes to the host
void emit_plain(std::string& o, const std::string& t) {
  const size_t n = t.size();
  if (n == 0) throw NeedsRender{};
  {
    size_t i = t[0] == '-' ? 1 : 0;
    bool digits = i < n && n - i <= 18 && !(t[i] == '0' && n > i + 1) && t != "-0";
    for (size_t k = i; digits && k < n; ++k) digits = t[k] >= '0' && t[k] <= '9';
    if (digits) { o += t; return; }
  }
  if (t == "true" || t == "True" || t == "TRUE") { o += "true"; return; }
  if (t == "false" || t == "False" || t == "FALSE") { o += "false"; return; }
  static const char* kw[] = {"yes", "Yes", "YES", "no", "No", "NO", "on", "On", "ON", "off", "Off", "OFF",
                             "y", "Y", "n", "N", "null", "Null", "NULL"};
  for (const char* k : kw)
    if (t == k) throw NeedsRender{};
  const char c0 = t[0];
  if (!((c0 >= 'A' && c0 <= 'Z') || (c0 >= 'a' && c0 <= 'z') || c0 == '_')) throw NeedsRender{};
  if (t[n - 1] == ' ') throw NeedsRender{};
  for (char c : t)
    if (!((c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z') || (c >= '0' && c <= '9') || c == '_' || c == '.' ||
          c == '/' || c == '-' || c == ' '))
      throw NeedsRender{};
  go_string(o, t);
}

// Go's text/template eq on basic kinds (gotpl._eq): json.Number compares as a string
int basic(const Val& v) {
  switch (v.k) {
    case V_MISSING:
    case V_NIL: return 0;
    case V_BOOL: return 1;
    case V_NUM:
    case V_STR: return 2;
    default: return 3;
  }
}

using kwkfmt::rfc3339nano;

// ------------------------------------------------------------------ skeleton mode
// A template rendered over a class representative with every per-object input replaced: the
// object's status and identity (the parts kwok_amd/host/compiler.py:class_key drops — status,
// metadata identity keys and ownerReferences, spec.nodeName / hostname) are never read, Now and
// every call of a controller function become slots.  The render succeeds only if those inputs
// reach the output solely as slot text (Quote'd / single-quoted scalars), call arguments
// (identity only: a call's value is fixed per object) or the one status read the pod Stages make,
// `index $root.status.<list> $i` inside `range $i, ... := <class-level list>` whose only effect is
// its error when the status list is shorter (a guard: the device checks a per-object bit instead).
// Every object of the class then renders to the skeleton's bytes with the slots filled in.
constexpr const char* kMarker = "\xF4\x8F\xBF\xBD";  // U+10FFFD: JSON and YAML carry it unchanged
constexpr size_t kMarkerLen = 4;
constexpr int kMaxSites = 24;

struct Skel {
  bool calls = false;  // per-object mode: call sites evaluated for real, their values recorded
  int in_ext = 0;      // > 0 while a call's arguments are evaluated
  std::vector<std::vector<std::string>> paths{{}};  // [0] = the object itself
  std::vector<std::pair<int, int>> guards;          // (status list path, range collection path)
  std::vector<const Expr*> sites;
  std::vector<std::string> values;
  uint32_t markers = 0;

  int extend(int base, const std::string& name) {
    std::vector<std::string> p = paths[(size_t)base];
    p.push_back(name);
    for (size_t i = 0; i < paths.size(); ++i)
      if (paths[i] == p) return (int)i;
    paths.push_back(std::move(p));
    return (int)paths.size() - 1;
  }
  // 0 class-level, 1 per-object, 2 an ancestor of per-object fields (compiler.py class_key)
  int taint_of(int id) const {
    static const char* identity[] = {"name", "generateName", "namespace", "uid", "resourceVersion", "creationTimestamp",
                                     "generation", "managedFields", "deletionTimestamp", "deletionGracePeriodSeconds",
                                     "finalizers", "labels", "annotations", "selfLink", "ownerReferences"};
    const std::vector<std::string>& p = paths[(size_t)id];
    if (p.empty()) return 2;
    if (p[0] == "status") return 1;
    if (p[0] == "metadata") {
      if (p.size() == 1) return 2;
      for (const char* k : identity)
        if (p[1] == k) return 1;
      return 0;
    }
    if (p[0] == "spec") {
      if (p.size() == 1) return 2;
      return p[1] == "nodeName" || p[1] == "hostname" ? 1 : 0;
    }
    return 0;
  }
  void marker(std::string& o, int id) {
    o += kMarker;
    o += (char)('A' + id);
    o += kMarker;
    ++markers;
  }
};

// a value whose data is per-object (or a slot's) must not be tested, printed or transformed
inline bool safe_value_char(unsigned char c) {
  return c >= 0x20 && c <= 0x7E && c != '"' && c != '\\' && c != '<' && c != '>' && c != '&' && c != '\'';
}

// ------------------------------------------------------------------ rendering
struct Ctx {
  const kwk_patcher& P;
  const Template* T = nullptr;
  const JV* root = nullptr;
  std::vector<Val> vars;
  std::vector<uint8_t> regs;
  std::string now;
  kwk_patch_fn fn = nullptr;
  void* user = nullptr;
  std::string* out = nullptr;
  JV empty_obj;
  std::vector<char> fbuf;
  Skel* sk = nullptr;  // skeleton mode

  explicit Ctx(const kwk_patcher& p) : P(p) { empty_obj.t = JV::OBJ; fbuf.resize(256); }

  // skeleton mode: v is consumed (tested, printed, transformed, passed to a call)
  void use(const Val& v) const {
    if (!sk) return;
    if (v.sent >= 0) throw Ineligible{"a Now / call value is tested or transformed"};
    if (v.taint == 1) throw Ineligible{"per-object data reaches the output or a test"};
    if (v.taint == 2 && (sk->in_ext == 0 || v.path == 0)) throw Ineligible{"a value holding per-object data is consumed"};
  }

  Val field_sk(Val v, const std::vector<std::string>& names) {
    for (const std::string& name : names) {
      const int np = v.path >= 0 ? sk->extend(v.path, name) : -1;
      if (v.taint == 1) {
        v.path = np;
        continue;
      }
      if (v.k == V_MISSING) return Val{};  // absent for the whole class (the parent's presence is)
      if (v.k != V_OBJ) throw NeedsRender{};
      const int t = np >= 0 ? sk->taint_of(np) : 0;
      if (t == 1) {
        if (sk->in_ext == 0) {
          Val x;
          x.taint = 1;
          x.path = np;
          v = x;
          continue;
        }
        if (sk->paths[(size_t)np][0] == "status") throw Ineligible{"a call argument reads status"};
      }
      const JV* x = v.j->get(name);
      v = x ? from_jv(x) : Val{};
      v.path = np;
      v.taint = t == 2 ? 2 : 0;
    }
    return v;
  }

  Val eval(const Expr& e, const Val& dot) {
    switch (e.k) {
      case E_ROOT: {
        Val r = from_jv(root);
        if (sk) { r.path = 0; r.taint = 2; }
        return r;
      }
      case E_DOT: return dot;
      case E_VAR: return vars[(size_t)e.i];
      case E_FIELD: {
        Val v = eval(e.a[0], dot);
        if (sk) return field_sk(v, e.path);
        for (const std::string& name : e.path) {
          if (v.k == V_MISSING) return v;
          if (v.k != V_OBJ) throw NeedsRender{};  // nil pointer / field of a non-map
          const JV* x = v.j->get(name);
          v = x ? from_jv(x) : Val{};
        }
        return v;
      }
      case E_NUM: {
        Val r;
        r.k = V_NUM;
        r.sp = &e.s;
        return r;
      }
      case E_STR: {
        Val r;
        r.k = V_STR;
        r.sp = &e.s;
        return r;
      }
      case E_BOOL: {
        Val r;
        r.k = V_BOOL;
        r.b = e.b;
        return r;
      }
      case E_NIL: {
        Val r;
        r.k = V_NIL;
        return r;
      }
      case E_CONST: return from_jv(&P.consts[(size_t)e.i]);
      case E_OR:
      case E_AND: {
        Val v;
        for (const Expr& x : e.a) {
          v = eval(x, dot);
          use(v);
          if ((e.k == E_OR) == truth(v)) return v;
        }
        return v;
      }
      case E_NOT: {
        Val r;
        r.k = V_BOOL;
        const Val x = eval(e.a[0], dot);
        use(x);
        r.b = !truth(x);
        return r;
      }
      case E_EQ:
      case E_NE: {
        const Val a = eval(e.a[0], dot);
        use(a);
        const int ka = basic(a);
        bool eq = false;
        for (size_t i = 1; i < e.a.size() && !eq; ++i) {
          const Val b = eval(e.a[i], dot);
          use(b);
          const int kb = basic(b);
          if (ka != kb) {
            if (ka && kb) throw NeedsRender{};  // incompatible types for comparison
            continue;
          }
          if (ka == 3) throw NeedsRender{};
          if (ka == 0) eq = true;
          else if (ka == 1) eq = a.b == b.b;
          else eq = (a.k == V_NUM ? num_text(a) : a.text()) == (b.k == V_NUM ? num_text(b) : b.text());
        }
        Val r;
        r.k = V_BOOL;
        r.b = e.k == E_EQ ? eq : !eq;
        return r;
      }
      case E_INDEX: {
        Val x = eval(e.a[0], dot);
        if (sk && x.taint == 1 && sk->in_ext == 0) {  // the status guard, or ineligible
          const Val key = e.a.size() == 2 ? eval(e.a[1], dot) : Val{};
          if (e.a.size() != 2 || key.taint || key.sent >= 0 || key.idx_of < 0 || x.path < 0 ||
              sk->paths[(size_t)x.path].size() != 2 || sk->paths[(size_t)x.path][0] != "status")
            throw Ineligible{"per-object data indexed"};
          const std::pair<int, int> g{x.path, key.idx_of};
          if (std::find(sk->guards.begin(), sk->guards.end(), g) == sk->guards.end()) sk->guards.push_back(g);
          Val t;
          t.taint = 1;
          return t;
        }
        use(x);
        for (size_t i = 1; i < e.a.size(); ++i) {
          const Val key = eval(e.a[i], dot);
          use(key);
          if (x.k == V_OBJ) {
            const JV* y = x.j->get(sprint(key));
            if (y) x = from_jv(y);
            else { x = Val{}; x.k = V_NIL; }  // missing key: the zero value
          } else if (x.k == V_ARR) {
            if (key.k != V_NUM) throw NeedsRender{};
            const std::string& t = num_text(key);
            const long long k = atoll(t.c_str());
            if (k < 0 || (size_t)k >= x.j->a.size()) throw NeedsRender{};  // index out of range
            x = from_jv(&x.j->a[(size_t)k]);
          } else {
            throw NeedsRender{};  // index of untyped nil / of a scalar
          }
        }
        return x;
      }
      case E_DICT: {
        Val r;
        r.k = V_OBJ;
        r.j = &empty_obj;
        return r;
      }
      case E_LEN: {
        const Val v = eval(e.a[0], dot);
        use(v);
        size_t n;
        if (v.k == V_ARR || v.k == V_OBJ) n = v.j->a.size();
        else if (v.k == V_STR) {
          for (char c : v.text())
            if ((unsigned char)c >= 0x80) throw NeedsRender{};
          n = v.text().size();
        } else throw NeedsRender{};
        Val r;
        r.k = V_NUM;
        r.own = std::to_string(n);
        return r;
      }
      case E_QUOTE: {
        const Val v = eval(e.a[0], dot);
        if (sk && v.sent >= 0) return v;  // Quote of a slot value: its text (slot values need no quoting)
        use(v);
        return str_val(quote_text(v));
      }
      case E_NOW: {
        Val r;
        r.k = V_STR;
        r.sp = &now;
        if (sk) r.sent = 0;
        return r;
      }
      case E_EXT: {
        const Func& f = P.funcs[(size_t)e.i];
        if (!f.callback) {
          Val r;
          r.k = V_STR;
          r.sp = &f.value;
          return r;
        }
        int site = -1;
        if (sk && sk->in_ext == 0) {  // a call site: its value is a slot
          if (std::find(sk->sites.begin(), sk->sites.end(), &e) != sk->sites.end())
            throw Ineligible{"a call site evaluated twice"};
          if ((int)sk->sites.size() >= kMaxSites) throw Ineligible{"too many call sites"};
          site = (int)sk->sites.size();
          sk->sites.push_back(&e);
          if (!sk->calls) {  // the arguments are checked, the value is the slot
            ++sk->in_ext;
            for (const Expr& x : e.a) use(eval(x, dot));
            --sk->in_ext;
            Val r;
            r.k = V_STR;
            r.sent = (int8_t)(1 + site);
            return r;
          }
        }
        if (!fn) throw NeedsRender{};
        std::vector<std::string> texts;
        std::vector<uint8_t> kinds;
        if (site >= 0) ++sk->in_ext;
        for (const Expr& x : e.a) {
          const Val v = eval(x, dot);
          use(v);
          kinds.push_back((uint8_t)v.k);
          if (v.k == V_ARR || v.k == V_OBJ) {
            std::string o;
            go_marshal(o, *v.j);
            texts.push_back(o);
          } else {
            texts.push_back(sprint(v));
          }
        }
        std::vector<const char*> argv;
        std::vector<uint32_t> argl;
        for (const std::string& t : texts) {
          argv.push_back(t.data());
          argl.push_back((uint32_t)t.size());
        }
        uint32_t len = 0;
        int32_t st = fn(user, (uint32_t)e.i, (uint32_t)texts.size(), argv.data(), argl.data(), kinds.data(),
                        fbuf.data(), (uint32_t)fbuf.size(), &len);
        if (st == 2 && len > fbuf.size()) {
          fbuf.resize(len);
          st = fn(user, (uint32_t)e.i, (uint32_t)texts.size(), argv.data(), argl.data(), kinds.data(), fbuf.data(),
                  (uint32_t)fbuf.size(), &len);
        }
        if (st != 0 || len > fbuf.size()) throw NeedsRender{};
        if (site >= 0) {
          --sk->in_ext;
          sk->values.emplace_back(fbuf.data(), len);
          Val r;
          r.k = V_STR;
          r.sent = (int8_t)(1 + site);
          return r;
        }
        return str_val(std::string(fbuf.data(), len));
      }
    }
    throw NeedsRender{};
  }

  void run_sets(const std::vector<Set>& sets, const Val& dot) {
    for (const Set& s : sets) vars[(size_t)s.var] = eval(T->exprs[(size_t)s.expr], dot);
  }

  // range over a value (text/template walkRange): arrays by index, maps by sorted key
  template <class F>
  void range(const Val& it, int vi, int ve, F body) {
    use(it);
    if (it.k == V_MISSING) return;
    if (it.k == V_ARR) {
      for (size_t i = 0; i < it.j->a.size(); ++i) {
        Val elem = from_jv(&it.j->a[i]);
        if (vi >= 0) {
          Val idx;
          idx.k = V_NUM;
          idx.own = std::to_string(i);
          if (sk) idx.idx_of = it.path;
          vars[(size_t)vi] = idx;
        }
        if (ve >= 0) vars[(size_t)ve] = elem;
        body(elem);
      }
      return;
    }
    if (it.k == V_OBJ) {
      std::vector<size_t> idx;
      for (size_t i = 0; i < it.j->k.size(); ++i) {
        bool last = true;
        for (size_t k = i + 1; k < it.j->k.size(); ++k)
          if (it.j->k[k] == it.j->k[i]) { last = false; break; }
        if (last) idx.push_back(i);
      }
      std::sort(idx.begin(), idx.end(), [&](size_t a, size_t b) { return it.j->k[a] < it.j->k[b]; });
      for (size_t i : idx) {
        Val elem = from_jv(&it.j->a[i]);
        if (vi >= 0) {
          Val key;
          key.k = V_STR;
          key.sp = &it.j->k[i];
          vars[(size_t)vi] = key;
        }
        if (ve >= 0) vars[(size_t)ve] = elem;
        body(elem);
      }
      return;
    }
    throw NeedsRender{};  // range over nil / a scalar
  }

  void sq(std::string& acc, const std::vector<Piece>& pieces, const Val& dot) {
    for (const Piece& p : pieces) {
      if (p.k == P_TEXT) {
        acc += p.text;
      } else if (p.k == P_VAL) {
        const Val v = eval(T->exprs[(size_t)p.expr], dot);
        if (sk && v.sent >= 0) {
          sk->marker(acc, v.sent);
          continue;
        }
        use(v);
        const std::string t = sprint(v);
        for (char c : t)  // inside '...': printable ASCII without a quote stays as it is
          if (c < 0x20 || c > 0x7E || c == '\'') throw NeedsRender{};
        acc += t;
      } else {
        const Val it = eval(T->exprs[(size_t)p.expr], dot);
        range(it, p.vi, p.ve, [&](const Val& elem) { sq(acc, p.sub, elem); });
      }
    }
  }

  void items(const std::vector<Item>& its, const Val& dot, size_t& count) {
    std::string& o = *out;
    for (const Item& it : its) {
      if (it.k == I_ITEM) {
        o += count++ ? ',' : '[';
        node(it.node, dot);
      } else if (it.k == I_RANGE) {
        const Val v = eval(T->exprs[(size_t)it.expr], dot);
        range(v, it.vi, it.ve, [&](const Val& elem) {
          run_sets(it.sets, elem);
          items(it.items, elem, count);
        });
      } else {
        const Val c = eval(T->exprs[(size_t)it.expr], dot);
        use(c);
        if (truth(c)) items(it.items, dot, count);
        else items(it.else_items, dot, count);
      }
    }
  }

  void node(const Node& n, const Val& dot) {
    std::string& o = *out;
    switch (n.k) {
      case N_LIT: o += n.lit; return;
      case N_Q: {
        const Val v = eval(T->exprs[(size_t)n.expr], dot);
        if (sk && v.sent >= 0) {
          o += '"';
          sk->marker(o, v.sent);
          o += '"';
          return;
        }
        use(v);
        const std::string s = quote_text(v);
        check_yaml_dq(s);
        go_string(o, s);
        return;
      }
      case N_RAW: {
        const Val v = eval(T->exprs[(size_t)n.expr], dot);
        use(v);
        emit_plain(o, sprint(v));
        return;
      }
      case N_SQ: {
        std::string acc;
        sq(acc, n.pieces, dot);
        go_string(o, acc);
        return;
      }
      case N_MAP: {
        for (const Guard& g : n.guards) {
          if (g.parent < 0 || regs[(size_t)g.parent]) {
            const Val gv = eval(T->exprs[(size_t)g.expr], dot);
            use(gv);
            const bool t = truth(gv);
            regs[(size_t)g.then_reg] = t;
            regs[(size_t)g.else_reg] = !t;
          } else {
            regs[(size_t)g.then_reg] = regs[(size_t)g.else_reg] = 0;
          }
        }
        o += '{';
        bool first = true;
        for (const Entry& e : n.entries) {
          if (e.reg >= 0 && !regs[(size_t)e.reg]) continue;
          if (!first) o += ',';
          first = false;
          o += e.key;
          node(e.node, dot);
        }
        o += '}';
        return;
      }
      case N_SEQ: {
        size_t count = 0;
        items(n.items, dot, count);
        o += count ? "]" : "null";
        return;
      }
    }
  }

  // one object: true when rendered, false = KWK_PATCH_NEEDS_RENDER (out restored)
  bool render(const Template& t, const char* text, size_t len) {
    JV obj;
    Parser ps{text, text + len};
    if (!ps.value(obj)) return false;
    ps.ws();
    if (ps.p != ps.e) return false;
    const size_t mark = out->size();
    try {
      body(t, obj);
    } catch (const NeedsRender&) {
      out->resize(mark);
      return false;
    }
    return true;
  }

  void body(const Template& t, const JV& obj) {
    T = &t;
    root = &obj;
    vars.assign((size_t)t.n_vars, Val{});
    regs.assign((size_t)t.n_regs, 0);
    Val dot = from_jv(root);
    if (sk) {
      dot.path = 0;
      dot.taint = 2;
    }
    out->append(t.head);
    run_sets(t.prologue, dot);
    node(t.body, dot);
    out->append(t.tail);
  }
};

}  // namespace

extern "C" {

const char* kwk_patch_last_error(const kwk_patcher* h) { return h ? h->err.c_str() : g_err.c_str(); }

kwk_status kwk_patcher_create(const char* spec_json, kwk_patcher** out) {
  if (!spec_json || !out) return fail(KWK_EINVAL, "null argument");
  JV spec;
  Parser ps{spec_json, spec_json + strlen(spec_json)};
  if (!ps.value(spec)) return fail(KWK_EINVAL, "patch spec is not JSON");
  auto p = std::make_unique<kwk_patcher>();
  try {
    for (const JV& f : member(spec, "funcs").a) {
      Func fn;
      if (const JV* c = f.get("const")) fn.value = str(*c);
      else fn.callback = true;
      p->funcs.push_back(fn);
    }
    p->consts = member(spec, "consts").a;
    for (const JV& tj : member(spec, "templates").a) {
      Template t;
      t.n_vars = num(member(tj, "n_vars"));
      t.n_regs = num(member(tj, "n_regs"));
      for (const JV& e : member(tj, "exprs").a) t.exprs.push_back(load_expr(e));
      t.prologue = load_sets(member(tj, "prologue"));
      t.head = str(member(tj, "head"));
      t.tail = str(member(tj, "tail"));
      t.body = load_node(member(tj, "body"));
      p->templates.push_back(std::move(t));
    }
  } catch (const BadSpec& b) {
    return fail(KWK_EINVAL, "patch spec: " + b.what);
  }
  // every reference in the program is in range (checked once here, not per object)
  for (const Template& t : p->templates) {
    const size_t ne = t.exprs.size();
    std::vector<const Expr*> st;
    for (const Expr& e : t.exprs) st.push_back(&e);
    while (!st.empty()) {
      const Expr* e = st.back();
      st.pop_back();
      if ((e->k == E_VAR && (e->i < 0 || e->i >= t.n_vars)) || (e->k == E_CONST && (e->i < 0 || (size_t)e->i >= p->consts.size())) ||
          (e->k == E_EXT && (e->i < 0 || (size_t)e->i >= p->funcs.size())) ||
          ((e->k == E_FIELD || e->k == E_NOT || e->k == E_LEN || e->k == E_QUOTE) && e->a.empty()) ||
          ((e->k == E_EQ || e->k == E_NE || e->k == E_INDEX || e->k == E_OR || e->k == E_AND) && e->a.empty()))
        return fail(KWK_EINVAL, "patch spec: expression reference out of range");
      for (const Expr& x : e->a) st.push_back(&x);
    }
    std::vector<const Node*> nodes{&t.body};
    std::vector<const Item*> its;
    auto chk_set = [&](const std::vector<Set>& ss) {
      for (const Set& s : ss)
        if (s.var < 0 || s.var >= t.n_vars || s.expr < 0 || (size_t)s.expr >= ne) return false;
      return true;
    };
    if (!chk_set(t.prologue)) return fail(KWK_EINVAL, "patch spec: assignment out of range");
    std::vector<const std::vector<Piece>*> pcs;
    while (!nodes.empty() || !its.empty() || !pcs.empty()) {
      if (!pcs.empty()) {
        const std::vector<Piece>* ps2 = pcs.back();
        pcs.pop_back();
        for (const Piece& x : *ps2) {
          if (x.k != P_TEXT && (x.expr < 0 || (size_t)x.expr >= ne)) return fail(KWK_EINVAL, "patch spec: piece");
          if (x.k == P_RANGE) {
            if (x.vi >= t.n_vars || x.ve >= t.n_vars) return fail(KWK_EINVAL, "patch spec: range variable");
            pcs.push_back(&x.sub);
          }
        }
        continue;
      }
      if (!its.empty()) {
        const Item* it = its.back();
        its.pop_back();
        if (it->k == I_ITEM) nodes.push_back(&it->node);
        else {
          if (it->expr < 0 || (size_t)it->expr >= ne || it->vi >= t.n_vars || it->ve >= t.n_vars || !chk_set(it->sets))
            return fail(KWK_EINVAL, "patch spec: item");
          for (const Item& x : it->items) its.push_back(&x);
          for (const Item& x : it->else_items) its.push_back(&x);
        }
        continue;
      }
      const Node* n = nodes.back();
      nodes.pop_back();
      if ((n->k == N_Q || n->k == N_RAW) && (n->expr < 0 || (size_t)n->expr >= ne))
        return fail(KWK_EINVAL, "patch spec: slot");
      if (n->k == N_SQ) pcs.push_back(&n->pieces);
      for (const Guard& g : n->guards)
        if (g.expr < 0 || (size_t)g.expr >= ne || g.then_reg < 0 || g.then_reg >= t.n_regs || g.else_reg < 0 ||
            g.else_reg >= t.n_regs || g.parent >= t.n_regs)
          return fail(KWK_EINVAL, "patch spec: guard");
      for (const Entry& e : n->entries) {
        if (e.reg >= t.n_regs) return fail(KWK_EINVAL, "patch spec: entry register");
        nodes.push_back(&e.node);
      }
      for (const Item& x : n->items) its.push_back(&x);
    }
  }
  *out = p.release();
  return KWK_OK;
}

kwk_status kwk_patcher_destroy(kwk_patcher* p) {
  ErrScope es_(p ? &p->err : nullptr);
  delete p;
  return KWK_OK;
}

kwk_status kwk_patch_render(kwk_patcher* p, uint32_t n, const uint16_t* template_ids, const char* objs,
                            const uint64_t* obj_offsets, int64_t now_ns, kwk_patch_fn fn, void* user,
                            uint32_t n_threads, const char** out_data, uint64_t* out_offsets, uint8_t* status) {
  ErrScope es_(p ? &p->err : nullptr);
  if (!p || !out_data || !out_offsets || (n && (!template_ids || !objs || !obj_offsets || !status)))
    return fail(KWK_EINVAL, "null argument");
  for (uint32_t i = 0; i < n; ++i) {
    if (template_ids[i] >= p->templates.size()) return fail(KWK_EINVAL, "template id out of range");
    if (obj_offsets[i + 1] < obj_offsets[i]) return fail(KWK_EINVAL, "object offsets not ascending");
  }
  const std::string now = rfc3339nano(now_ns);
  const uint32_t nt = std::max(1u, std::min(n_threads, std::max(1u, n / 64)));
  std::vector<std::string> outs(nt);
  std::vector<std::vector<uint64_t>> lens(nt);
  auto work = [&](uint32_t t) {
    const uint32_t lo = (uint32_t)((uint64_t)n * t / nt), hi = (uint32_t)((uint64_t)n * (t + 1) / nt);
    Ctx c(*p);
    c.now = now;
    c.fn = fn;
    c.user = user;
    c.out = &outs[t];
    for (uint32_t i = lo; i < hi; ++i) {
      const size_t before = outs[t].size();
      const bool ok = c.render(p->templates[template_ids[i]], objs + obj_offsets[i], obj_offsets[i + 1] - obj_offsets[i]);
      status[i] = ok ? KWK_PATCH_OK : KWK_PATCH_NEEDS_RENDER;
      lens[t].push_back(outs[t].size() - before);
    }
  };
  if (nt == 1) {
    work(0);
  } else {
    std::vector<std::thread> th;
    for (uint32_t t = 0; t < nt; ++t) th.emplace_back(work, t);
    for (auto& x : th) x.join();
  }
  p->out.clear();
  size_t total = 0;
  for (const auto& o : outs) total += o.size();
  p->out.reserve(total);
  uint64_t off = 0;
  uint32_t i = 0;
  for (uint32_t t = 0; t < nt; ++t) {
    p->out += outs[t];
    for (uint64_t l : lens[t]) {
      out_offsets[i++] = off;
      off += l;
    }
  }
  out_offsets[n] = off;
  *out_data = p->out.data();
  return KWK_OK;
}

// ------------------------------------------------------------------ skeletons (device emission)
namespace {

// JSON string of arbitrary bytes the renderer produced (valid UTF-8)
void json_str(std::string& o, const std::string& s) {
  try {
    go_string(o, s);
  } catch (const NeedsRender&) {
    o += "\"\"";
  }
}

// split a skeleton text at its slot markers: literal runs and slot ids
bool split_skeleton(const std::string& t, uint32_t markers, std::vector<std::string>& lits, std::vector<int>& slots) {
  lits.assign(1, std::string());
  slots.clear();
  size_t i = 0;
  while (i < t.size()) {
    if (t.compare(i, kMarkerLen, kMarker) == 0) {
      if (i + 2 * kMarkerLen + 1 > t.size() || t.compare(i + kMarkerLen + 1, kMarkerLen, kMarker) != 0) return false;
      const int id = t[i + kMarkerLen] - 'A';
      if (id < 0 || id > kMaxSites) return false;
      slots.push_back(id);
      lits.emplace_back();
      i += 2 * kMarkerLen + 1;
      continue;
    }
    lits.back() += t[i++];
  }
  return slots.size() == markers;
}

}  // namespace

kwk_status kwk_patch_skeleton(kwk_patcher* p, uint32_t tid, const char* obj, uint64_t len, const char** out_json,
                              uint64_t* out_len) {
  ErrScope es_(p ? &p->err : nullptr);
  if (!p || !obj || !out_json || !out_len) return fail(KWK_EINVAL, "null argument");
  if (tid >= p->templates.size()) return fail(KWK_EINVAL, "template id out of range");
  JV o;
  Parser ps{obj, obj + len};
  if (!ps.value(o)) return fail(KWK_EINVAL, "object is not JSON");
  Skel sk;
  Ctx c(*p);
  c.sk = &sk;
  std::string text;
  c.out = &text;
  std::string& r = p->skel;
  r.clear();
  const char* why = nullptr;
  try {
    c.body(p->templates[tid], o);
  } catch (const Ineligible& x) {
    why = x.why;
  } catch (const NeedsRender&) {
    why = "the template does not render natively for this class";
  }
  std::vector<std::string> lits;
  std::vector<int> slots;
  if (!why && !split_skeleton(text, sk.markers, lits, slots)) why = "the object holds the slot marker";
  if (why) {
    r = "{\"eligible\":false,\"reason\":";
    json_str(r, why);
    r += "}";
  } else {
    r = "{\"eligible\":true,\"text\":";
    json_str(r, text);
    r += ",\"lits\":[";
    for (size_t i = 0; i < lits.size(); ++i) {
      if (i) r += ',';
      json_str(r, lits[i]);
    }
    r += "],\"slots\":[";
    for (size_t i = 0; i < slots.size(); ++i) r += (i ? "," : "") + std::to_string(slots[i]);
    r += "],\"calls\":" + std::to_string(sk.sites.size()) + ",\"guards\":[";
    for (size_t g = 0; g < sk.guards.size(); ++g) {
      r += g ? ",[" : "[";
      for (int side = 0; side < 2; ++side) {
        const std::vector<std::string>& path = sk.paths[(size_t)(side ? sk.guards[g].second : sk.guards[g].first)];
        r += side ? ",[" : "[";
        for (size_t k = 0; k < path.size(); ++k) {
          if (k) r += ',';
          json_str(r, path[k]);
        }
        r += ']';
      }
      r += ']';
    }
    r += "]}";
  }
  *out_json = r.data();
  *out_len = r.size();
  return KWK_OK;
}

kwk_status kwk_patch_object_values(kwk_patcher* p, uint32_t tid, uint32_t n, const char* objs, const uint64_t* obj_offsets,
                                   const char* skeleton, uint64_t skeleton_len, kwk_patch_fn fn, void* user,
                                   uint32_t n_threads, uint32_t n_calls, uint32_t stride, uint8_t* values, uint8_t* ok) {
  ErrScope es_(p ? &p->err : nullptr);
  if (!p || (n && (!objs || !obj_offsets || !ok || !skeleton || (n_calls && !values)))) return fail(KWK_EINVAL, "null argument");
  if (tid >= p->templates.size()) return fail(KWK_EINVAL, "template id out of range");
  if (n_calls && (stride < 2 || stride > 256)) return fail(KWK_EINVAL, "stride must be 2..256");
  for (uint32_t i = 0; i < n; ++i)
    if (obj_offsets[i + 1] < obj_offsets[i]) return fail(KWK_EINVAL, "object offsets not ascending");
  const std::string want(skeleton, skeleton_len);
  const uint32_t nt = std::max(1u, std::min(n_threads, std::max(1u, n / 64)));
  auto work = [&](uint32_t t) {
    const uint32_t lo = (uint32_t)((uint64_t)n * t / nt), hi = (uint32_t)((uint64_t)n * (t + 1) / nt);
    Ctx c(*p);
    c.fn = fn;
    c.user = user;
    std::string text;
    c.out = &text;
    for (uint32_t i = lo; i < hi; ++i) {
      uint8_t* v = values ? values + (uint64_t)i * n_calls * stride : nullptr;
      for (uint32_t k = 0; k < n_calls; ++k) v[(uint64_t)k * stride] = 0xFF;
      ok[i] = 0;
      JV o;
      Parser ps{objs + obj_offsets[i], objs + obj_offsets[i + 1]};
      if (!ps.value(o)) continue;
      Skel sk;
      sk.calls = true;
      c.sk = &sk;
      text.clear();
      try {
        c.body(p->templates[tid], o);
      } catch (const Ineligible&) {
        continue;
      } catch (const NeedsRender&) {
        continue;
      }
      if (text != want || sk.values.size() != n_calls) continue;
      bool good = true;
      for (uint32_t k = 0; k < n_calls; ++k) {
        const std::string& x = sk.values[k];
        bool safe = x.size() + 1 <= stride;
        for (char ch : x) safe = safe && safe_value_char((unsigned char)ch);
        if (!safe) { good = false; continue; }
        v[(uint64_t)k * stride] = (uint8_t)x.size();
        memcpy(v + (uint64_t)k * stride + 1, x.data(), x.size());
      }
      ok[i] = good ? 1 : 0;
    }
  };
  if (nt == 1) {
    work(0);
  } else {
    std::vector<std::thread> th;
    for (uint32_t t = 0; t < nt; ++t) th.emplace_back(work, t);
    for (auto& x : th) x.join();
  }
  return KWK_OK;
}

}  // extern "C"
