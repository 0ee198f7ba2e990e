// Native Stage compiler (include/kwok_compiler.h): lifecycle.NewLifecycle's compilation behind
// the C ABI, so that a Go host builds the device's stage table without the Python compiler.
//
// Reference: pkg/utils/lifecycle/lifecycle.go:33-46,194-267 (NewLifecycle / NewStage: selectors,
// gojq requirements, weight / delay / jitter getters, next), pkg/utils/expression/selector.go:
// 37-120 (Requirement), query.go:33-88 (Query, ToJSONStandard), value_int_from.go /
// value_duration_from.go (the *From getters), internalversion/conversion.go:395-425 (statusTemplate
// as one merge patch rooted at status), v1alpha1/zz_generated.defaults.go:55-63 (defaults),
// pkg/utils/lifecycle/next.go:43-173 + finalizers.go:32-111 (the next state the exploration
// applies), pkg/kwok/controllers/stages_manager.go:72-122 (rebuilt when Stage CRs change).
//
// This is the line-for-line native form of kwok_amd/host/compiler.py (KindProgram): feature bits
// per selector query (present / literal bits, the finalizer set), stage descriptors, value slots,
// the harness masks, the object classes and the (class, stage) deltas derived by exploring
// representative objects with the gotpl mirror (gotpl.hpp); the encoder and patch specs are
// written exactly as kwok_amd/host/encoder.py / patchtpl.py write them.  tests/
// test_native_compiler.py checks every output byte-equal against the Python compiler.
#include <cstdint>
#include <cstring>
#include <map>
#include <memory>
#include <set>
#include <string>
#include <utility>
#include <vector>

#include "../../include/kwok_compiler.h"
#include "../../include/kwok_engine.h"
#include "gotpl.hpp"
#include "host_common.hpp"
#include "labelsel.hpp"
#include "nextstate.hpp"
#include "patchtpl.hpp"

namespace {

using kwkjson::JV;
using kwkpatch::PJ;
using kwktpl::TplError;
using namespace kwknext;

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


// Python str(v) of a YAML / JSON scalar (stage_from_v1alpha1's str(...) of values and map entries)
std::string py_str(const JV& v) {
  switch (v.t) {
    case JV::STR: return v.s;
    case JV::BOOL: return v.b ? "True" : "False";
    case JV::NUL: return "None";
    case JV::NUM: return kwktpl::py_num_text(v);
    default: throw CompileError("a selector value must be a scalar");
  }
}
// Python truthiness / int() of the JSON values stage_from_v1alpha1 reads
bool py_truth(const JV* v) {
  if (!v) return false;
  switch (v->t) {
    case JV::NUL: return false;
    case JV::BOOL: return v->b;
    case JV::NUM: return strtod(v->s.c_str(), nullptr) != 0;
    case JV::STR: return !v->s.empty();
    default: return !v->a.empty();
  }
}
int64_t py_int(const JV* v, const char* what) {
  if (!v || v->t == JV::NUL) return 0;
  if (v->t == JV::NUM) return v->is_int ? strtoll(v->s.c_str(), nullptr, 10) : (int64_t)strtod(v->s.c_str(), nullptr);
  if (v->t == JV::BOOL) return v->b ? 1 : 0;
  if (v->t == JV::STR) {
    char* end = nullptr;
    const long long x = strtoll(v->s.c_str(), &end, 10);
    if (end && *end == 0 && !v->s.empty()) return x;
  }
  throw CompileError(std::string(what) + " must be an integer");
}

// ------------------------------------------------------------------ the Stage CRD surface
// kwok_amd/host/stages.py stage_from_v1alpha1 (v1alpha1 -> internal, conversion.go:395-425)
struct Requirement {
  std::string key, op;
  std::vector<std::string> values;
};
struct Stage {
  std::string name, api_group, kind;
  bool has_selector = false;
  bool has_ml = false, has_ma = false, has_exprs = false;
  std::vector<std::pair<std::string, std::string>> ml, ma;
  std::vector<Requirement> exprs;
  int64_t weight = 0;
  bool has_weight_from = false;
  std::string weight_from;
  bool has_delay = false;
  bool has_dur_ms = false, has_dur_from = false, has_jit_ms = false, has_jit_from = false;
  int64_t dur_ms = 0, jit_ms = 0;
  std::string dur_from, jit_from;
  bool has_fin = false, fin_empty = false;
  std::vector<std::string> fin_add, fin_remove;
  bool del = false, immediate = false;
  std::vector<Patch> patches;
};

bool expr_from(const JV* x, std::string& out) {
  if (!x || x->t == JV::NUL) return false;
  if (x->t != JV::OBJ) throw CompileError("expressionFrom source must be an object");
  const JV* e = x->get("expressionFrom");
  out = e && e->t == JV::STR ? e->s : (e && e->t != JV::NUL ? py_str(*e) : "");
  return true;
}

std::vector<std::pair<std::string, std::string>> str_map(const JV& m) {
  std::vector<std::pair<std::string, std::string>> out;
  if (m.t != JV::OBJ) throw CompileError("matchLabels / matchAnnotations must be a mapping");
  for (size_t i = 0; i < m.k.size(); ++i) {
    bool dup = false;
    for (auto& kv : out)
      if (kv.first == m.k[i]) { kv.second = py_str(m.a[i]); dup = true; }
    if (!dup) out.emplace_back(m.k[i], py_str(m.a[i]));
  }
  return out;
}

Stage stage_from_v1alpha1(const JV& obj) {
  if (obj.t != JV::OBJ) throw CompileError("a Stage must be an object");
  const JV* kind = obj.get("kind");
  if (kind && kind->t != JV::NUL && !(kind->t == JV::STR && kind->s == "Stage"))
    throw CompileError("not a Stage: " + (kind->t == JV::STR ? kind->s : std::string("?")));
  Stage st;
  const JV* spec = obj.get("spec");
  static const JV empty = jobj();
  if (!spec || spec->t != JV::OBJ) spec = &empty;
  const JV* ref = spec->get("resourceRef");
  if (!ref || ref->t != JV::OBJ || !ref->get("kind")) throw CompileError("spec.resourceRef.kind is required");
  st.kind = py_str(*ref->get("kind"));
  const JV* ag = ref->get("apiGroup");
  st.api_group = py_truth(ag) ? py_str(*ag) : "v1";
  const JV* sel = spec->get("selector");
  if (sel && sel->t != JV::NUL) {
    st.has_selector = true;
    if (const JV* me = sel->get("matchExpressions"); me && me->t != JV::NUL) {
      st.has_exprs = true;
      for (const JV& e : me->a) {
        Requirement r;
        const JV* op = e.get("operator");
        r.op = op && op->t == JV::STR ? op->s : "";
        if (const JV* vals = e.get("values"); vals && vals->t == JV::ARR)
          for (const JV& v : vals->a) r.values.push_back(py_str(v));
        if ((r.op == "In" || r.op == "NotIn") && r.values.empty())
          throw CompileError("for 'in', 'notin' operators, values set can't be empty");
        if ((r.op == "Exists" || r.op == "DoesNotExist") && !r.values.empty())
          throw CompileError("values set must be empty for exists and does not exist");
        if (r.op != "In" && r.op != "NotIn" && r.op != "Exists" && r.op != "DoesNotExist")
          throw CompileError("operator '" + r.op + "' is not supported");
        const JV* key = e.get("key");
        if (!key) throw CompileError("matchExpressions entry without key");
        r.key = py_str(*key);
        st.exprs.push_back(std::move(r));
      }
    }
    if (const JV* ml = sel->get("matchLabels"); ml && ml->t != JV::NUL) { st.has_ml = true; st.ml = str_map(*ml); }
    if (const JV* ma = sel->get("matchAnnotations"); ma && ma->t != JV::NUL) { st.has_ma = true; st.ma = str_map(*ma); }
  }
  if (const JV* d = spec->get("delay"); d && d->t != JV::NUL) {
    st.has_delay = true;
    if (const JV* x = d->get("durationMilliseconds"); x && x->t != JV::NUL) { st.has_dur_ms = true; st.dur_ms = py_int(x, "durationMilliseconds"); }
    st.has_dur_from = expr_from(d->get("durationFrom"), st.dur_from);
    if (const JV* x = d->get("jitterDurationMilliseconds"); x && x->t != JV::NUL) { st.has_jit_ms = true; st.jit_ms = py_int(x, "jitterDurationMilliseconds"); }
    st.has_jit_from = expr_from(d->get("jitterDurationFrom"), st.jit_from);
  }
  const JV* n = spec->get("next");
  if (!n || n->t != JV::OBJ) n = &empty;
  if (const JV* f = n->get("finalizers"); f && f->t != JV::NUL) {
    st.has_fin = true;
    auto vals = [&](const char* which, std::vector<std::string>& out) {
      if (const JV* l = f->get(which); l && l->t == JV::ARR)
        for (const JV& i : l->a) {
          const JV* v = i.get("value");
          out.push_back(v ? py_str(*v) : "");
        }
    };
    vals("add", st.fin_add);
    vals("remove", st.fin_remove);
    st.fin_empty = py_truth(f->get("empty"));
  }
  if (const JV* ps = n->get("patches"); ps && ps->t == JV::ARR) {
    for (const JV& p : ps->a) {
      Patch pt;
      if (const JV* x = p.get("root")) pt.root = py_str(*x);
      if (const JV* x = p.get("template")) pt.tmpl = py_str(*x);
      if (const JV* x = p.get("type"); py_truth(x)) pt.type = py_str(*x);
      if (const JV* x = p.get("subresource")) pt.subresource = py_str(*x);
      st.patches.push_back(std::move(pt));
    }
  }
  if (const JV* t = n->get("statusTemplate"); py_truth(t) && st.patches.empty()) {
    Patch pt;
    pt.root = "status";
    pt.tmpl = py_str(*t);
    const JV* sub = n->get("statusSubresource");
    pt.subresource = (!sub || sub->t == JV::NUL) ? "status" : py_str(*sub);
    st.patches.push_back(std::move(pt));
  }
  st.del = py_truth(n->get("delete"));
  const JV* md = obj.get("metadata");
  if (md && md->t == JV::OBJ)
    if (const JV* nm = md->get("name")) st.name = py_str(*nm);
  st.weight = py_int(spec->get("weight"), "weight");
  st.has_weight_from = expr_from(spec->get("weightFrom"), st.weight_from);
  st.immediate = py_truth(spec->get("immediateNextStage"));
  return st;
}

// ------------------------------------------------------------------ jq queries
// Selector keys and *From getters compile with the native jq subset (jqc.hpp, through
// kwkhost::compile_query); the encoder spec carries each query's source, which the encoder
// compiles the same way.
bool sp(char c) { return kwktpl::is_space(c); }

std::string strip(const std::string& s) { return kwktpl::py_strip(s); }

// a JSON string body as json.loads('"%s"' % body) reads it
std::string json_body(const std::string& body) {
  const std::string q = "\"" + body + "\"";
  JV v;
  kwkjson::Parser P{q.data(), q.data() + q.size()};
  if (!P.value(v) || v.t != JV::STR) throw CompileError("bad string in query: " + body);
  return v.s;
}

// compiler.path_prefix: the leading static path of a query
std::vector<std::string> path_prefix(const std::string& src) {
  std::vector<std::string> out;
  const std::string s = strip(src);
  size_t i = 0;
  while (i < s.size() && s[i] == '.') {
    const size_t j = i + 1;
    if (j < s.size() && kwktpl::is_alpha_(s[j])) {
      size_t k = j + 1;
      while (k < s.size() && kwktpl::is_alnum_(s[k])) ++k;
      out.push_back(s.substr(j, k - j));
      i = k;
      continue;
    }
    if (j < s.size() && s[j] == '[') {
      size_t q = j + 1;
      while (q < s.size() && sp(s[q])) ++q;
      if (q < s.size() && s[q] == '"') {
        size_t r = q + 1;
        while (r < s.size() && s[r] != '"') r += s[r] == '\\' ? 2 : 1;
        if (r < s.size()) {
          size_t t = r + 1;
          while (t < s.size() && sp(s[t])) ++t;
          if (t < s.size() && s[t] == ']') {
            out.push_back(json_body(s.substr(q + 1, r - q - 1)));
            i = t + 1;
            continue;
          }
        }
      }
      break;
    }
    if (j < s.size() && s[j] == '"') {
      size_t r = j + 1;
      while (r < s.size() && s[r] != '"') r += s[r] == '\\' ? 2 : 1;
      if (r < s.size()) {
        out.push_back(json_body(s.substr(j + 1, r - j - 1)));
        i = r + 1;
        continue;
      }
    }
    break;
  }
  return out;
}

// compiler._norm: the query without whitespace outside its string literals (the feature / slot key)
std::string norm(const std::string& s) {
  std::string o;
  bool in_str = false;
  for (size_t i = 0; i < s.size(); ++i) {
    const char c = s[i];
    if (in_str) {
      o += c;
      if (c == '\\' && i + 1 < s.size()) o += s[++i];
      else if (c == '"') in_str = false;
    } else if (c == '"') {
      in_str = true;
      o += c;
    } else if (!sp(c)) {
      o += c;
    }
  }
  return o;
}

bool is_fin_query(const std::string& n) {
  return n == ".metadata.finalizers" || n == ".metadata.finalizers.[]" || n == ".metadata.finalizers[]";
}

const char* const kIdentityMeta[] = {"name", "generateName", "namespace", "uid", "resourceVersion", "creationTimestamp",
                                     "generation", "managedFields", "deletionTimestamp", "deletionGracePeriodSeconds",
                                     "finalizers", "labels", "annotations", "selfLink"};

// ------------------------------------------------------------------ next state (nextstate.py)

// finalizers.go:83-111 (ops in order)
std::vector<JV> finalizers_modify(const JV* meta_fin, const Stage& st) {
  std::vector<JV> meta;
  if (meta_fin && meta_fin->t == JV::ARR) meta = meta_fin->a;
  std::vector<JV> ops;
  auto op = [](const char* o, const std::string& path) {
    JV x = jobj();
    obj_set(x, "op", jstr(o));
    obj_set(x, "path", jstr(path));
    return x;
  };
  auto in = [](const JV& v, const std::vector<std::string>& set) {
    if (v.t != JV::STR) return false;
    for (const std::string& s : set)
      if (s == v.s) return true;
    return false;
  };
  bool is_empty = false;
  if (st.fin_empty) {
    is_empty = true;
  } else if (!st.fin_remove.empty()) {
    std::vector<JV> removed;
    for (size_t i = meta.size(); i-- > 0;)
      if (in(meta[i], st.fin_remove)) removed.push_back(op("remove", "/metadata/finalizers/" + std::to_string(i)));
    if (removed.size() == meta.size()) is_empty = true;
    else ops.insert(ops.end(), removed.begin(), removed.end());
  }
  auto add = [&](const std::vector<JV>& m) {
    std::vector<JV> out;
    if (!m.empty()) {
      for (const std::string& f : st.fin_add) {
        bool present = false;
        for (const JV& x : m) present |= x.t == JV::STR && x.s == f;
        if (!present) {
          JV o = op("add", "/metadata/finalizers/-");
          obj_set(o, "value", jstr(f));
          out.push_back(o);
        }
      }
      return out;
    }
    JV o = op("add", "/metadata/finalizers");
    JV arr;
    arr.t = JV::ARR;
    for (const std::string& f : st.fin_add) arr.a.push_back(jstr(f));
    obj_set(o, "value", arr);
    out.push_back(o);
    return out;
  };
  if (!is_empty) {
    if (!st.fin_add.empty())
      for (JV& x : add(meta)) ops.push_back(std::move(x));
  } else {
    if (!meta.empty()) ops.push_back(op("remove", "/metadata/finalizers"));
    if (!st.fin_add.empty())
      for (JV& x : add({})) ops.push_back(std::move(x));
  }
  return ops;
}

// nextstate.apply_next: playStage's effect (pod_controller.go:290-360) -> (object | deleted, changed)
bool apply_next(const Stage& st, JV& obj, kwktpl::Renderer& r, bool& deleted) {
  bool changed = false;
  deleted = false;
  if (st.has_fin) {
    const JV* md = obj.t == JV::OBJ ? obj.get("metadata") : nullptr;
    const JV* fins = md && md->t == JV::OBJ ? md->get("finalizers") : nullptr;
    const std::vector<JV> ops = finalizers_modify(fins, st);
    if (!ops.empty()) {
      JV nw = json_patch(obj, ops);
      prune_empty(nw);
      changed = canon(nw) != canon(obj);
      obj = std::move(nw);
    }
  }
  if (st.del) {
    deleted = true;
    return true;
  }
  for (const Rendered& rp : render_patches(st.patches, obj, r)) {
    JV nw = apply_patch(obj, rp);
    prune_empty(nw);
    if (canon(nw) != canon(obj)) {
      changed = true;
      obj = std::move(nw);
    }
  }
  return changed;
}

JV strip_for_recreate(const JV& obj) {
  JV o = obj;
  obj_erase(o, "status");
  JV& md = obj_setdefault(o, "metadata");
  for (const char* k : {"deletionTimestamp", "deletionGracePeriodSeconds", "finalizers"}) obj_erase(md, k);
  return o;
}

}  // namespace

// ------------------------------------------------------------------ the program
struct kwk_program {
  std::string err;
  std::string out_json;  // the last JSON string handed out
  std::vector<Stage> stages;
  std::vector<std::string> names;

  struct Feature {
    std::string src;
    kwkhost::CQuery q;
    int present_bit = -1;
    std::vector<std::pair<std::string, int>> lit_bits;
    uint32_t mask() const {
      uint32_t m = present_bit < 0 ? 0u : 1u << present_bit;
      for (const auto& lb : lit_bits) m |= 1u << lb.second;
      return m;
    }
  };
  std::vector<std::string> feature_order;  // normalised sources in insertion order
  std::map<std::string, Feature> features;
  int nbits = 0;
  std::vector<std::pair<std::string, int>> fin_bits;
  int fin_other_bit = -1;
  std::vector<std::pair<std::string, std::string>> slots;  // (type, src)
  std::map<std::pair<std::string, std::string>, int> slot_index;
  std::vector<kwk_stage_desc> desc;

  bool harness = false;
  std::string terminal_query = ".status.phase", deletion_query = ".metadata.deletionTimestamp";
  std::vector<std::string> terminal_values{"Succeeded", "Failed"};
  uint32_t deletion_bit = 0, terminal_mask = 0, keep_mask = 0;
  kwklabels::Disregard disregard;  // need()'s selectors (options "disregard")
  int disregard_bit = -1;

  std::vector<std::string> class_keys;  // id -> key
  std::map<std::string, uint32_t> class_ids;
  std::map<std::pair<uint32_t, int>, std::pair<uint32_t, uint32_t>> deltas;
  std::vector<std::string> delta_conflicts;
  std::vector<std::pair<int, int>> applied_bits;  // (stage, bit) in assignment order

  std::vector<JV> roots;
  std::set<std::pair<std::string, uint32_t>> root_keys;
  bool explored = false;

  std::vector<std::string> identity_meta;

  // -- bits
  int bit() {
    if (nbits >= 32) throw CompileError("stage set needs more than 32 feature bits");
    return nbits++;
  }
  Feature& feature(const std::string& src) {
    const std::string key = norm(src);
    auto it = features.find(key);
    if (it != features.end()) return it->second;
    Feature f;
    f.src = src;
    try {
      f.q = kwkhost::compile_query(src);
    } catch (const kwkjq::Unsupported& e) {
      throw CompileError(e.what());
    }
    feature_order.push_back(key);
    return features.emplace(key, std::move(f)).first->second;
  }
  uint32_t present(const std::string& src) {
    Feature& f = feature(src);
    if (f.present_bit < 0) f.present_bit = bit();
    return 1u << f.present_bit;
  }
  uint32_t lits(const std::string& src, const std::vector<std::string>& values) {
    Feature* f = &feature(src);
    uint32_t m = 0;
    for (const std::string& v : values) {
      int b = -1;
      for (const auto& lb : f->lit_bits)
        if (lb.first == v) b = lb.second;
      if (b < 0) {
        b = bit();
        f->lit_bits.emplace_back(v, b);
      }
      m |= 1u << b;
    }
    return m;
  }
  int fin_bit_of(const std::string& v) const {
    for (const auto& fb : fin_bits)
      if (fb.first == v) return fb.second;
    return -1;
  }
  uint32_t fin_value(const std::string& v) {
    int b = fin_bit_of(v);
    if (b < 0) {
      b = bit();
      fin_bits.emplace_back(v, b);
    }
    return 1u << b;
  }
  uint32_t fin_group_mask() const {
    uint32_t m = 0;
    for (const auto& fb : fin_bits) m |= 1u << fb.second;
    if (fin_other_bit >= 0) m |= 1u << fin_other_bit;
    return m;
  }
  int32_t slot(const std::string& typ, bool has, const std::string& src) {
    if (!has) return KWK_SLOT_NONE;
    if (typ == "duration" && norm(src) == ".metadata.deletionTimestamp") return KWK_SLOT_DELETION;
    const auto key = std::make_pair(typ, norm(src));
    auto it = slot_index.find(key);
    if (it != slot_index.end()) return it->second;
    const int id = (int)slots.size();
    slot_index[key] = id;
    try {
      kwkhost::compile_query(src);
    } catch (const kwkjq::Unsupported& e) {
      throw CompileError(e.what());
    }
    slots.emplace_back(typ, src);
    return id;
  }

  // -- compile (KindProgram._compile)
  void compile() {
    bool uses_fin = false;
    for (const Stage& s : stages) {
      uses_fin |= s.has_fin;
      for (const Requirement& e : s.exprs) uses_fin |= is_fin_query(norm(e.key));
    }
    if (uses_fin) {
      for (const Stage& s : stages) {
        for (const Requirement& e : s.exprs) {
          const std::string nk = norm(e.key);
          if ((nk == ".metadata.finalizers.[]" || nk == ".metadata.finalizers[]") && (e.op == "In" || e.op == "NotIn"))
            for (const std::string& v : e.values) fin_value(v);
        }
        if (s.has_fin) {
          for (const std::string& v : s.fin_add) fin_value(v);
          for (const std::string& v : s.fin_remove) fin_value(v);
        }
      }
      fin_other_bit = bit();
    }
    for (const Stage& st : stages) {
      uint32_t eq_mask = 0, eq_val = 0;
      std::vector<std::pair<uint32_t, uint32_t>> anys;
      auto eq = [&](uint32_t mask, bool want) {
        eq_mask |= mask;
        if (want) eq_val |= mask;
      };
      auto popcount1 = [](uint32_t m) { return __builtin_popcount(m) == 1; };
      for (int which = 0; which < 2; ++which) {
        const bool has = which == 0 ? st.has_ml : st.has_ma;
        if (!has) continue;
        const auto& m = which == 0 ? st.ml : st.ma;
        const char* kind = which == 0 ? "labels" : "annotations";
        for (const auto& kv : m) {
          std::string q;
          kwkhost::esc(q, kv.first);  // json.dumps(k)
          eq(lits(std::string(".metadata.") + kind + "[" + q + "]", {kv.second}), true);
        }
      }
      for (const Requirement& e : st.exprs) {
        const std::string nk = norm(e.key);
        if (is_fin_query(nk)) {
          const uint32_t g = fin_group_mask();
          if (e.op == "Exists" || e.op == "DoesNotExist") {
            if (e.op == "Exists") anys.emplace_back(g, 1);
            else eq(g, false);
          } else if (nk == ".metadata.finalizers") {
            if (e.op == "In") anys.emplace_back(0, 1);
          } else {
            uint32_t m = 0;
            for (const std::string& v : e.values) m |= 1u << fin_bit_of(v);
            if (e.op == "In") {
              if (popcount1(m)) eq(m, true);
              else anys.emplace_back(m, 1);
            } else {
              eq(m, false);
            }
          }
          continue;
        }
        if (e.op == "Exists") eq(present(e.key), true);
        else if (e.op == "DoesNotExist") eq(present(e.key), false);
        else {
          const uint32_t m = lits(e.key, e.values);
          if (e.op == "In") {
            if (popcount1(m)) eq(m, true);
            else anys.emplace_back(m, 1);
          } else {
            eq(m, false);
          }
        }
      }
      if (anys.size() > KWK_MAX_ANY)
        throw CompileError("stage " + st.name + ": more than " + std::to_string(KWK_MAX_ANY) + " multi-value In requirements");
      kwk_stage_desc d;
      memset(&d, 0, sizeof d);
      d.eq_mask = eq_mask;
      d.eq_val = eq_val;
      d.n_any = (uint32_t)anys.size();
      for (size_t i = 0; i < anys.size(); ++i) {
        d.any_mask[i] = anys[i].first;
        d.any_want |= anys[i].second << i;
      }
      d.weight_default = st.weight;
      d.weight_slot = slot("int", st.has_weight_from, st.weight_from);
      if (st.has_delay) {
        d.has_delay = 1;
        d.delay_default = (st.has_dur_ms ? st.dur_ms : 0) * 1000000;
        d.delay_slot = slot("duration", st.has_dur_from, st.dur_from);
        if (st.has_jit_ms || st.has_jit_from) {
          d.has_jitter = 1;
          d.jitter_default = (st.has_jit_ms ? st.jit_ms : 0) * 1000000;
          d.jitter_default_ok = st.has_jit_ms ? 1 : 0;
          d.jitter_slot = slot("duration", st.has_jit_from, st.jit_from);
        } else {
          d.jitter_slot = KWK_SLOT_NONE;
        }
      } else {
        d.delay_slot = KWK_SLOT_NONE;
        d.jitter_slot = KWK_SLOT_NONE;
      }
      uint32_t fl = 0;
      if (st.del) fl |= KWK_NEXT_DELETE;
      if (st.immediate) fl |= KWK_NEXT_IMMEDIATE;
      if (!st.patches.empty()) fl |= KWK_NEXT_PATCHES;
      if (st.has_fin) {
        fl |= KWK_NEXT_FIN;
        if (st.fin_empty) fl |= KWK_NEXT_FIN_EMPTY;
        if (!st.fin_remove.empty()) fl |= KWK_NEXT_FIN_REMOVE;
        for (const std::string& v : st.fin_add) d.fin_add |= 1u << fin_bit_of(v);
        for (const std::string& v : st.fin_remove) d.fin_remove |= 1u << fin_bit_of(v);
      }
      d.flags = fl;
      desc.push_back(d);
    }
    if (harness) {
      deletion_bit = present(deletion_query);
      terminal_mask = lits(terminal_query, terminal_values);
    }
    if (disregard.active()) disregard_bit = bit();  // labels / annotations: kept on re-creation
    uint32_t keep = disregard_bit < 0 ? 0u : 1u << disregard_bit;
    for (const std::string& key : feature_order) {
      const Feature& f = features.at(key);
      const std::vector<std::string> p = path_prefix(f.src);
      const bool dyn = p.empty() || p[0] == "status" ||
                       (p.size() >= 2 && p[0] == "metadata" &&
                        (p[1] == "deletionTimestamp" || p[1] == "deletionGracePeriodSeconds" || p[1] == "finalizers"));
      if (!dyn) keep |= f.mask();
    }
    keep_mask = keep;
  }

  // -- per object
  uint32_t stage_matches(uint32_t pred) const {
    uint32_t m = 0;
    for (size_t i = 0; i < desc.size(); ++i) {
      const kwk_stage_desc& d = desc[i];
      bool ok = ((pred ^ d.eq_val) & d.eq_mask) == 0;
      for (uint32_t k = 0; k < d.n_any && ok; ++k) ok = ((pred & d.any_mask[k]) != 0) == (((d.any_want >> k) & 1u) != 0);
      if (ok) m |= 1u << i;
    }
    return m;
  }

  kwktpl::Renderer static_r = static_renderer();
  bool patch_applied(const Stage& st, const JV& obj) { return kwknext::patch_applied(st.patches, obj, static_r); }

  uint32_t pred_of(const JV& obj) {
    uint32_t pred = 0;
    std::vector<kwkjq::Val> out;
    for (const std::string& key : feature_order) {
      const Feature& f = features.at(key);
      if (!kwkhost::exec_query(f.q, obj, out) || out.empty()) continue;
      if (f.present_bit >= 0) pred |= 1u << f.present_bit;
      for (const auto& lb : f.lit_bits)
        for (const kwkjq::Val& d : out)
          if (kwkjq::has_value(*d.p, lb.first)) {
            pred |= 1u << lb.second;
            break;
          }
    }
    if (fin_other_bit >= 0) {
      const JV* md = obj.t == JV::OBJ ? obj.get("metadata") : nullptr;
      const JV* fins = md && md->t == JV::OBJ ? md->get("finalizers") : nullptr;
      if (fins && fins->t == JV::ARR)
        for (const JV& x : fins->a) {
          const int b = x.t == JV::STR ? fin_bit_of(x.s) : -1;
          pred |= 1u << (b < 0 ? fin_other_bit : b);
        }
    }
    for (const auto& sb : applied_bits)
      if (patch_applied(stages[(size_t)sb.first], obj)) pred |= 1u << sb.second;
    if (disregard_bit >= 0 && disregard.disregarded(obj)) pred |= 1u << disregard_bit;
    return pred;
  }

  uint32_t class_of(const JV& obj, bool reg) {
    JV o = obj;
    prune_empty(o);
    const std::string k = kwkhost::class_key(o, identity_meta);
    auto it = class_ids.find(k);
    if (it != class_ids.end()) return it->second;
    if (!reg) return 0xFFFFFFFFu;
    const uint32_t c = (uint32_t)class_keys.size();
    if (c >= (1u << 16)) throw CompileError("more than 65536 object classes");
    class_ids[k] = c;
    class_keys.push_back(k);
    return c;
  }

  // -- exploration (KindProgram.explore / _explore_pass)
  void explore(const std::vector<JV>& new_roots, size_t max_states = 256) {
    size_t added = 0;
    for (const JV& r0 : new_roots) {
      JV r = r0;
      prune_empty(r);
      const auto k = std::make_pair(kwkhost::class_key(r, identity_meta), pred_of(r));
      if (root_keys.count(k)) continue;
      root_keys.insert(k);
      roots.push_back(r);
      ++added;
    }
    if (explored && !added) return;
    explored = true;
    for (int pass = 0; pass < 2; ++pass) {
      const std::set<int> unchanged = explore_pass(max_states);
      std::vector<int> fresh;
      for (int s : unchanged) {
        bool known = false;
        for (const auto& sb : applied_bits) known |= sb.first == s;
        if (!known) fresh.push_back(s);
      }
      if (fresh.empty()) break;
      for (int s : fresh) {
        const int b = bit();
        applied_bits.emplace_back(s, b);
        desc[(size_t)s].flags |= KWK_NEXT_PATCH_STATIC;
        desc[(size_t)s].applied_mask = 1u << b;
      }
    }
  }

  std::set<int> explore_pass(size_t max_states) {
    deltas.clear();
    delta_conflicts.clear();
    std::set<int> unchanged;
    std::vector<std::pair<uint32_t, int>> trans_order;
    std::map<std::pair<uint32_t, int>, std::vector<std::pair<uint32_t, uint32_t>>> trans;
    kwktpl::Renderer renderer(0);
    renderer.exploration_funcs();
    const uint32_t fin = fin_group_mask();
    std::set<std::pair<uint32_t, uint32_t>> seen_roots;
    for (const JV& root0 : roots) {
      JV root = root0;
      prune_empty(root);
      const uint32_t c = class_of(root, true);
      std::vector<JV> start{root};
      if (harness) start.push_back(strip_for_recreate(root));
      for (const JV& r : start) {
        const auto rk = std::make_pair(c, pred_of(r));
        if (seen_roots.count(rk)) continue;
        seen_roots.insert(rk);
        std::vector<JV> frontier{r};
        std::set<uint32_t> seen{pred_of(r)};
        int64_t t_ns = 1700000000LL * 1000000000LL;
        while (!frontier.empty() && seen.size() <= max_states) {
          JV o = std::move(frontier.back());
          frontier.pop_back();
          const uint32_t p = pred_of(o);
          const uint32_t m = stage_matches(p);
          std::vector<JV> succ;
          for (size_t s = 0; s < stages.size(); ++s) {
            if (!((m >> s) & 1u)) continue;
            const Stage& st = stages[s];
            t_ns += 1000000000LL;
            renderer.set_now(t_ns);
            JV o2 = o;
            bool deleted;
            const bool changed = apply_next(st, o2, renderer, deleted);
            if (!st.patches.empty() && !changed && !st.del) unchanged.insert((int)s);
            if (deleted) continue;
            const uint32_t p2 = pred_of(o2);
            const auto key = std::make_pair(c, (int)s);
            if (!trans.count(key)) trans_order.push_back(key);
            trans[key].emplace_back(p, p2);
            bool known = false;
            for (const auto& sb : applied_bits) known |= sb.first == (int)s;
            if (!st.patches.empty() && !known && ((stage_matches(p2) >> s) & 1u)) {
              JV o3 = o2;
              bool d3;
              if (!apply_next(st, o3, renderer, d3)) unchanged.insert((int)s);
            }
            const kwk_stage_desc& d = desc[s];
            if (d.flags & KWK_NEXT_FIN) {
              const uint32_t F = p & fin;
              uint32_t F2;
              if ((d.flags & KWK_NEXT_FIN_EMPTY) || ((d.flags & KWK_NEXT_FIN_REMOVE) && (F & ~d.fin_remove) == 0)) F2 = d.fin_add;
              else F2 = (F & ~d.fin_remove) | (d.fin_add & ~F);
              if (F2 != (p2 & fin)) throw CompileError("stage " + st.name + ": finalizer algebra mismatch");
            }
            succ.push_back(std::move(o2));
          }
          if (harness && (p & terminal_mask) && !(p & deletion_bit)) {
            JV o2 = o;
            obj_set(obj_setdefault(o2, "metadata"), "deletionTimestamp", jstr("2023-11-14T22:13:20Z"));
            succ.push_back(std::move(o2));
          }
          for (JV& o2 : succ) {
            const uint32_t p2 = pred_of(o2);
            if (!seen.count(p2)) {
              seen.insert(p2);
              frontier.push_back(std::move(o2));
            }
          }
        }
      }
    }
    const uint32_t nonfin = ~fin;
    for (const auto& key : trans_order) {
      const auto& ts = trans[key];
      const int s = key.second;
      if (stages[(size_t)s].patches.empty()) {
        deltas[key] = {0xFFFFFFFFu, 0u};
        continue;
      }
      uint32_t and_m = 0xFFFFFFFFu, or_m = 0;
      bool ok = true;
      for (int b = 0; b < 32; ++b) {
        const uint32_t bitm = 1u << b;
        if (!(nonfin & bitm)) continue;
        bool keep = true, post0 = false, post1 = false;
        for (const auto& pp : ts) {
          keep &= ((pp.first & bitm) != 0) == ((pp.second & bitm) != 0);
          if (pp.second & bitm) post1 = true;
          else post0 = true;
        }
        if (keep) continue;
        if (post0 != post1) {
          and_m &= ~bitm;
          if (post1) or_m |= bitm;
        } else {
          ok = false;
          delta_conflicts.push_back("class " + std::to_string(key.first) + " stage " + stages[(size_t)s].name + ": bit " +
                                    std::to_string(b) + " depends on pre-state");
        }
      }
      deltas[key] = ok ? std::make_pair(and_m, or_m) : std::make_pair((uint32_t)KWK_DELTA_UNKNOWN_AND, (uint32_t)KWK_DELTA_UNKNOWN_OR);
    }
    return unchanged;
  }

  bool uses_deletion_column() const {
    for (const kwk_stage_desc& d : desc)
      if (d.delay_slot == KWK_SLOT_DELETION || d.jitter_slot == KWK_SLOT_DELETION) return true;
    return false;
  }

  // -- outputs
  std::string describe() const {
    PJ feats = PJ::list();
    for (const std::string& key : feature_order) {
      const Feature& f = features.at(key);
      PJ lit = PJ::dict();
      for (const auto& lb : f.lit_bits) lit.set(lb.first, PJ::integer(lb.second));
      feats.push(PJ::dict()
                     .set("query", PJ::str(f.src))
                     .set("present_bit", f.present_bit < 0 ? PJ::null() : PJ::integer(f.present_bit))
                     .set("literals", lit));
    }
    PJ names_pj = PJ::list();
    for (const std::string& n : names) names_pj.push(PJ::str(n));
    PJ applied = PJ::dict();
    for (const auto& sb : applied_bits) applied.set(names[(size_t)sb.first], PJ::integer(sb.second));
    PJ fins = PJ::dict();
    for (const auto& fb : fin_bits) fins.set(fb.first, PJ::integer(fb.second));
    PJ vs = PJ::list();
    for (const auto& s : slots) vs.push(PJ::list({PJ::str(s.first), PJ::str(s.second)}));
    PJ d = PJ::dict()
               .set("stages", names_pj)
               .set("bits", PJ::integer(nbits))
               .set("features", feats)
               .set("applied_bits", applied)
               .set("finalizers", fins)
               .set("finalizer_other_bit", fin_other_bit < 0 ? PJ::null() : PJ::integer(fin_other_bit))
               .set("value_slots", vs)
               .set("classes", PJ::integer((long long)class_keys.size()))
               .set("uses_deletion_column", PJ::boolean(uses_deletion_column()))
               .set("disregard", disregard_pj());
    std::string o;
    kwkpatch::pj_dump(o, d);
    return o;
  }

  PJ disregard_pj() const {
    if (disregard_bit < 0) return PJ::null();
    return PJ::dict()
        .set("bit", PJ::integer(disregard_bit))
        .set("annotation_selector", PJ::str(disregard.ann_text))
        .set("label_selector", PJ::str(disregard.lab_text));
  }

  std::string encoder_spec() const {
    PJ feats = PJ::list();
    for (const std::string& key : feature_order) {
      const Feature& f = features.at(key);
      PJ lit = PJ::dict();
      for (const auto& lb : f.lit_bits) lit.set(lb.first, PJ::integer(lb.second));
      feats.push(PJ::dict()
                     .set("query", PJ::str(f.src))
                     .set("present_bit", f.present_bit < 0 ? PJ::null() : PJ::integer(f.present_bit))
                     .set("literals", lit));
    }
    PJ fins = PJ::dict();
    for (const auto& fb : fin_bits) fins.set(fb.first, PJ::integer(fb.second));
    PJ sl = PJ::list();
    for (size_t i = 0; i < slots.size(); ++i)
      sl.push(PJ::dict().set("type", PJ::str(slots[i].first)).set("query", PJ::str(slots[i].second)));
    PJ cls = PJ::dict();
    for (size_t i = 0; i < class_keys.size(); ++i) cls.set(class_keys[i], PJ::integer((long long)i));
    PJ im = PJ::list();
    for (const std::string& k : identity_meta) im.push(PJ::str(k));
    PJ d = PJ::dict()
               .set("features", feats)
               .set("finalizers", fins)
               .set("finalizer_other_bit", fin_other_bit < 0 ? PJ::null() : PJ::integer(fin_other_bit))
               .set("slots", sl)
               .set("classes", cls)
               .set("identity_meta", im);
    if (disregard_bit >= 0) d.set("disregard", disregard_pj());
    if (!applied_bits.empty()) {
      // "patch already applied" bits (the host encoder_spec rejects them): the encoder renders the
      // stage's patches with the static renderer and compares, as KindProgram._patch_applied
      PJ ap = PJ::list();
      for (const auto& sb : applied_bits) {
        PJ ps = PJ::list();
        for (const Patch& pt : stages[(size_t)sb.first].patches)
          ps.push(PJ::dict().set("type", PJ::str(pt.type)).set("root", PJ::str(pt.root)).set("template", PJ::str(pt.tmpl)));
        ap.push(PJ::dict().set("bit", PJ::integer(sb.second)).set("patches", ps));
      }
      d.set("applied", ap);
    }
    std::string o;
    kwkpatch::pj_dump(o, d);
    return o;
  }

  // patchtpl.PatchProgram: the spec and (stage, patch) -> template id
  std::string patch_spec(const JV& funcs, const std::string& version, std::vector<std::vector<int>>& template_of) {
    std::map<std::string, std::pair<bool, std::string>> fmap;  // name -> (callback, const)
    if (funcs.t == JV::ARR)
      for (const JV& f : funcs.a) {
        const JV* n = f.get("name");
        if (!n || n->t != JV::STR) throw CompileError("patch funcs: an entry without a name");
        const JV* c = f.get("const");
        fmap[n->s] = c && c->t == JV::STR ? std::make_pair(false, c->s) : std::make_pair(true, std::string());
      }
    PJ fspec = PJ::list();
    std::map<std::string, int> fids;
    for (const auto& kv : fmap) {  // sorted by name
      fids[kv.first] = (int)fspec.l.size();
      if (kv.second.first) fspec.push(PJ::dict().set("name", PJ::str(kv.first)).set("callback", PJ::boolean(true)));
      else fspec.push(PJ::dict().set("name", PJ::str(kv.first)).set("const", PJ::str(kv.second.second)));
    }
    const std::map<std::string, int> const_ids{{"NodeConditions", 0}, {"Version", 1}};
    PJ consts = PJ::list({kwkpatch::pj_of(kwktpl::parse_json_text(kwktpl::node_conditions_json())), PJ::str(version)});
    PJ templates = PJ::list();
    template_of.assign(stages.size(), {});
    for (size_t si = 0; si < stages.size(); ++si) {
      for (size_t pi = 0; pi < stages[si].patches.size(); ++pi) {
        const Patch& p = stages[si].patches[pi];
        int id = -1;
        if (p.type == "merge" || p.type == "strategic") {
          try {
            kwkpatch::TemplateCompiler tc(fids, const_ids);
            PJ t = tc.compile(p.tmpl, p.root);
            id = (int)templates.l.size();
            templates.push(std::move(t));
          } catch (const kwkpatch::Unsupported&) {
          } catch (const TplError&) {
          }
        }
        template_of[si].push_back(id);
      }
    }
    PJ d = PJ::dict().set("templates", templates).set("funcs", fspec).set("consts", consts);
    std::string o;
    kwkpatch::pj_dump(o, d);
    return o;
  }
};

namespace {

std::vector<JV> split_objects(uint32_t n, const char* objs, const uint64_t* offsets) {
  std::vector<JV> out;
  for (uint32_t i = 0; i < n; ++i) {
    if (offsets[i + 1] < offsets[i]) throw CompileError("offsets must be non-decreasing");
    out.push_back(parse_json(objs + offsets[i], objs + offsets[i + 1], ("object " + std::to_string(i)).c_str()));
    if (out.back().t != JV::OBJ) throw CompileError("object " + std::to_string(i) + ": not a JSON object");
  }
  return out;
}

}  // namespace

extern "C" {

const char* kwk_program_last_error(const kwk_program* p) { return p ? p->err.c_str() : g_err.c_str(); }

kwk_status kwk_compile_stages(const char* stages_json, const char* options_json, kwk_program** out) {
  ErrScope es_(nullptr);
  if (!stages_json || !out) return fail(KWK_EINVAL, "null argument");
  try {
    const JV arr = parse_json(stages_json, stages_json + strlen(stages_json), "stages");
    if (arr.t != JV::ARR) return fail(KWK_EINVAL, "stages: a JSON array of Stage objects");
    std::unique_ptr<kwk_program> P(new kwk_program());
    for (const char* k : kIdentityMeta) P->identity_meta.push_back(k);
    std::string ref;
    for (const JV& d : arr.a) {
      Stage st = stage_from_v1alpha1(d);
      const std::string r = st.api_group + "/" + st.kind;
      if (ref.empty()) ref = r;
      else if (r != ref) return fail(KWK_EINVAL, "stages of more than one resourceRef (" + ref + ", " + r + "): one program per resourceRef");
      if (st.has_selector) P->stages.push_back(std::move(st));  // NewLifecycle drops nil selectors (lifecycle.go:199-201)
    }
    if (P->stages.size() > KWK_MAX_STAGES)
      return fail(KWK_EINVAL, std::to_string(P->stages.size()) + " stages > " + std::to_string(KWK_MAX_STAGES));
    for (const Stage& s : P->stages) P->names.push_back(s.name);
    if (options_json) {
      const JV opt = parse_json(options_json, options_json + strlen(options_json), "options");
      if (const JV* dg = opt.get("disregard"); dg && dg->t == JV::OBJ) {
        const JV* a = dg->get("annotation_selector");
        const JV* l = dg->get("label_selector");
        P->disregard = kwklabels::Disregard(a && a->t == JV::STR ? a->s : "", l && l->t == JV::STR ? l->s : "");
      }
      if (const JV* h = opt.get("harness"); h && h->t != JV::NUL && !(h->t == JV::BOOL && !h->b)) {
        P->harness = true;
        if (h->t == JV::OBJ) {
          if (const JV* x = h->get("terminal_query"); x && x->t == JV::STR) P->terminal_query = x->s;
          if (const JV* x = h->get("deletion_query"); x && x->t == JV::STR) P->deletion_query = x->s;
          if (const JV* x = h->get("terminal_values"); x && x->t == JV::ARR) {
            P->terminal_values.clear();
            for (const JV& v : x->a) P->terminal_values.push_back(py_str(v));
          }
        }
      }
    }
    P->compile();
    *out = P.release();
    return KWK_OK;
  } catch (const std::exception& e) {
    return fail(KWK_EINVAL, e.what());
  }
}

kwk_status kwk_program_destroy(kwk_program* p) {
  delete p;
  return KWK_OK;
}

kwk_status kwk_program_explore(kwk_program* p, uint32_t n, const char* objs, const uint64_t* offsets) {
  ErrScope es_(p ? &p->err : nullptr);
  if (!p || (n && (!objs || !offsets))) return fail(KWK_EINVAL, "null argument");
  try {
    p->explore(split_objects(n, objs, offsets));
    return KWK_OK;
  } catch (const std::exception& e) {
    return fail(KWK_EINVAL, e.what());
  }
}

kwk_status kwk_program_class(kwk_program* p, const char* obj, uint64_t len, int32_t reg, uint32_t* cls) {
  ErrScope es_(p ? &p->err : nullptr);
  if (!p || !obj || !cls) return fail(KWK_EINVAL, "null argument");
  try {
    const JV o = parse_json(obj, obj + len, "object");
    *cls = p->class_of(o, reg != 0);
    return KWK_OK;
  } catch (const std::exception& e) {
    return fail(KWK_EINVAL, e.what());
  }
}

kwk_status kwk_program_table(const kwk_program* p, uint32_t version, kwk_stage_table* out) {
  if (!p || !out) return fail(KWK_EINVAL, "null argument");
  memset(out, 0, sizeof *out);
  out->n_stages = (uint32_t)p->stages.size();
  out->fin_group_mask = p->fin_group_mask();
  out->n_classes = p->class_keys.empty() ? 1u : (uint32_t)p->class_keys.size();
  out->version = version;
  out->pred_bits = (uint32_t)p->nbits;
  out->disregard_mask = p->disregard_bit < 0 ? 0u : 1u << p->disregard_bit;
  for (size_t i = 0; i < p->desc.size(); ++i) out->stages[i] = p->desc[i];
  return KWK_OK;
}

kwk_status kwk_program_deltas(const kwk_program* p, kwk_delta* out, uint64_t cap, uint32_t* n_classes, uint32_t* n_stages) {
  if (!p || !n_classes || !n_stages) return fail(KWK_EINVAL, "null argument");
  const uint32_t nc = p->class_keys.empty() ? 1u : (uint32_t)p->class_keys.size();
  const uint32_t ns = p->stages.empty() ? 1u : (uint32_t)p->stages.size();
  *n_classes = nc;
  *n_stages = ns;
  if (!out) return KWK_OK;
  if (cap < (uint64_t)nc * ns) return fail(KWK_ECAP, "delta buffer too small");
  for (uint32_t c = 0; c < nc; ++c)
    for (uint32_t s = 0; s < ns; ++s) {
      kwk_delta d{KWK_DELTA_UNKNOWN_AND, KWK_DELTA_UNKNOWN_OR};
      auto it = p->deltas.find({c, (int)s});
      if (it != p->deltas.end()) d = kwk_delta{it->second.first, it->second.second};
      if (s < p->stages.size() && p->stages[s].patches.empty()) d = kwk_delta{0xFFFFFFFFu, 0u};
      out[(size_t)c * ns + s] = d;
    }
  return KWK_OK;
}

kwk_status kwk_program_harness(const kwk_program* p, kwk_harness* out) {
  if (!p || !out) return fail(KWK_EINVAL, "null argument");
  memset(out, 0, sizeof *out);
  if (p->harness) {
    out->enable = 1;
    out->keep_mask = p->keep_mask;
    out->terminal_mask = p->terminal_mask;
    out->deletion_bit = p->deletion_bit;
    out->track_deletion = p->uses_deletion_column() ? 1u : 0u;
  }
  return KWK_OK;
}

kwk_status kwk_program_value_slots(const kwk_program* p, uint32_t* n) {
  if (!p || !n) return fail(KWK_EINVAL, "null argument");
  *n = (uint32_t)p->slots.size();
  return KWK_OK;
}

kwk_status kwk_program_describe(kwk_program* p, const char** json) {
  ErrScope es_(p ? &p->err : nullptr);
  if (!p || !json) return fail(KWK_EINVAL, "null argument");
  p->out_json = p->describe();
  *json = p->out_json.c_str();
  return KWK_OK;
}

kwk_status kwk_program_class_keys(kwk_program* p, const char** json) {
  ErrScope es_(p ? &p->err : nullptr);
  if (!p || !json) return fail(KWK_EINVAL, "null argument");
  PJ d = PJ::dict();
  for (size_t i = 0; i < p->class_keys.size(); ++i) d.set(p->class_keys[i], PJ::integer((long long)i));
  p->out_json.clear();
  kwkpatch::pj_dump(p->out_json, d);
  *json = p->out_json.c_str();
  return KWK_OK;
}

kwk_status kwk_program_encoder_spec(kwk_program* p, const char** json) {
  ErrScope es_(p ? &p->err : nullptr);
  if (!p || !json) return fail(KWK_EINVAL, "null argument");
  try {
    p->out_json = p->encoder_spec();
  } catch (const std::exception& e) {
    return fail(KWK_EINVAL, e.what());
  }
  *json = p->out_json.c_str();
  return KWK_OK;
}

kwk_status kwk_program_patch_spec(kwk_program* p, const char* funcs_json, const char* version, const char** json,
                                  int32_t* template_of, uint32_t cap) {
  ErrScope es_(p ? &p->err : nullptr);
  if (!p || !json) return fail(KWK_EINVAL, "null argument");
  try {
    JV funcs;
    if (funcs_json) funcs = parse_json(funcs_json, funcs_json + strlen(funcs_json), "funcs");
    std::vector<std::vector<int>> tof;
    p->out_json = p->patch_spec(funcs, version ? version : "v0.6.0", tof);
    if (template_of) {
      if (cap < p->stages.size() * KWK_MAX_PATCHES) return fail(KWK_ECAP, "template_of buffer too small");
      for (size_t s = 0; s < p->stages.size(); ++s)
        for (size_t k = 0; k < KWK_MAX_PATCHES; ++k)
          template_of[s * KWK_MAX_PATCHES + k] = k < tof[s].size() ? tof[s][k] : -1;
    }
  } catch (const std::exception& e) {
    return fail(KWK_EINVAL, e.what());
  }
  *json = p->out_json.c_str();
  return KWK_OK;
}

}  // extern "C"
