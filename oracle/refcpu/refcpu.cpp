// ORACLE / TEST INFRASTRUCTURE — not product code.
// "refcpu": a CPU restatement of KWOK's Stage lifecycle hot path (reference
// liangyuanpeng/kwok @ 2024-08-07, Go).  Only tests/, __graft_entry__.smoke() and
// bench.py's cpu_baseline leg load this library, and only as the checker / CPU baseline.
//
// Restated reference functions (file:line under /root/reference):
//   NewLifecycle / Lifecycle.match / ListAllPossible / Match   pkg/utils/lifecycle/lifecycle.go:33-191
//   NewStage / Stage.match / Stage.Delay / Stage.Weight        pkg/utils/lifecycle/lifecycle.go:194-361
//   finalizersAdd / finalizersRemove / finalizersModify        pkg/utils/lifecycle/finalizers.go:32-111
//   NewRequirement / Requirement.Matches / hasValue(s)         pkg/utils/expression/selector.go:37-120
//   Query.Execute / ToJSONStandard                             pkg/utils/expression/query.go:48-88
//   NewIntFrom / int64From.Get                                 pkg/utils/expression/value_int_from.go:36-94
//   NewDurationFrom / durationFrom.Get                         pkg/utils/expression/value_duration_from.go:36-79
//   labels.SelectorFromSet(...).Matches (apimachinery v0.30.2) lifecycle.go:203-208,286-295
// Randomness: the reference draws from Go's global math/rand at lifecycle.go:157,163,175,180
// (pick) and :338 (jitter).  Those call sites take the injected Philox4x32-10 hook described
// in DESIGN.md §RNG (key = seed, counter = (global slot, step lo, step hi, site)), so this
// oracle and the HIP engine are bit-comparable.
#include <atomic>
#include <cmath>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "goparse.hpp"
#include "jq.hpp"
#include "json.hpp"

namespace refcpu {

// ---------------------------------------------------------------- Philox hook
static inline void philox_round(uint32_t c[4], const uint32_t k[2]) {
  const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
  const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
  const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
  const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
  uint32_t n0 = hi1 ^ c[1] ^ k[0];
  uint32_t n2 = hi0 ^ c[3] ^ k[1];
  c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
}
static inline void philox4x32_10(uint32_t c[4], uint64_t seed) {
  uint32_t k[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  for (int r = 0; r < 10; ++r) {
    philox_round(c, k);
    k[0] += 0x9E3779B9u;
    k[1] += 0xBB67AE85u;
  }
}

enum RngSite : uint32_t { SITE_PICK = 1, SITE_JITTER = 2 };

struct Rng {
  uint64_t seed = 0;
  uint64_t slot = 0;
  uint64_t step = 0;
  // sites 1 (pick) and 2 (jitter) share the block of counter site 1: words 0-1 / 2-3
  // (DESIGN.md §RNG); sites 3, 4 take words 0-1 of their own block
  uint64_t u64(uint32_t site) const {
    const bool jit = site == SITE_JITTER;
    uint32_t c[4] = {(uint32_t)slot, (uint32_t)step, (uint32_t)(step >> 32), jit ? (uint32_t)SITE_PICK : site};
    philox4x32_10(c, seed);
    return jit ? (uint64_t)c[2] | ((uint64_t)c[3] << 32) : (uint64_t)c[0] | ((uint64_t)c[1] << 32);
  }
  // rand.Intn / rand.Int63n replacement: floor(u64 * n / 2^64), n > 0
  int64_t below(uint32_t site, int64_t n) const {
    unsigned __int128 p = (unsigned __int128)u64(site) * (uint64_t)n;
    return (int64_t)(uint64_t)(p >> 64);
  }
};

// ---------------------------------------------------------------- expression
enum Op { OP_IN, OP_NOTIN, OP_EXISTS, OP_DNE };

struct Requirement {
  std::unique_ptr<Query> q;
  Op op;
  std::vector<std::string> vals;

  static bool has_value(const JVP& d, const std::vector<std::string>& vs) {
    std::string s;
    switch (d->t) {
      case JV::STR: s = d->s; break;
      case JV::BOOL: s = d->b ? "true" : "false"; break;
      case JV::NUM:  // a gojq int (length, literals) matches FormatInt; float64 JSON numbers never do
        if (!d->gint) return false;
        s = std::to_string(d->i);
        break;
      default: return false;  // selector.go:101-111
    }
    for (auto& v : vs) if (v == s) return true;
    return false;
  }
  bool matches(const JVP& data) const {
    std::vector<JVP> out;
    bool ok = q->execute(data, out);
    if (!ok) return op == OP_NOTIN || op == OP_DNE;  // data == nil
    switch (op) {
      case OP_IN: for (auto& d : out) if (has_value(d, vals)) return true; return false;
      case OP_NOTIN: for (auto& d : out) if (has_value(d, vals)) return false; return true;
      case OP_EXISTS: return !out.empty();
      case OP_DNE: return out.empty();
    }
    return false;
  }
};

struct IntGetter {
  enum Kind { NOOP, CONST, FROM } kind = NOOP;
  bool has_value = false;
  int64_t value = 0;
  std::unique_ptr<Query> q;
  bool get(const JVP& v, int64_t& out) const {
    out = 0;
    if (kind == NOOP) return false;
    if (kind == CONST) { out = value; return true; }
    std::vector<JVP> res;
    q->execute(v, res);
    if (res.empty()) { if (has_value) { out = value; return true; } return false; }
    const JVP& t = res[0];
    if (t->t == JV::STR) {
      if (t->s.empty()) return false;
      int64_t n;
      if (go_parse_int(t->s, n)) { out = n; return true; }
      return false;
    }
    if (t->t == JV::NUM && !t->gint) { out = go_f64_to_i64(t->n); return true; }  // float64 only: a gojq int
    if (has_value) { out = value; return true; }                                    // falls to the default
    return false;
  }
};

struct DurationGetter {
  enum Kind { NOOP, CONST, FROM } kind = NOOP;
  bool has_value = false;
  int64_t value = 0;
  std::unique_ptr<Query> q;
  bool get(const JVP& v, int64_t now, int64_t& out) const {
    out = 0;
    if (kind == NOOP) return false;
    if (kind == CONST) { out = value; return true; }
    std::vector<JVP> res;
    q->execute(v, res);
    if (res.empty()) { if (has_value) { out = value; return true; } return false; }
    if (res[0]->t == JV::STR) {
      const std::string& t = res[0]->s;
      if (t.empty()) return false;
      GoTime ti;
      if (go_parse_rfc3339nano(t, ti)) { out = go_time_sub(ti, now); return true; }
      int64_t du;
      if (go_parse_duration(t, du)) { out = du; return true; }
    }
    return false;
  }
};

static bool new_int_from(IntGetter& g, bool has_value, int64_t value, const std::string* src) {
  if (!has_value && !src) { g.kind = IntGetter::NOOP; return true; }
  if (!src) { g.kind = IntGetter::CONST; g.value = value; return true; }
  g.kind = IntGetter::FROM;
  g.has_value = has_value;
  g.value = value;
  g.q.reset(new Query(*src));
  return true;
}
static void new_duration_from(DurationGetter& g, bool has_value, int64_t value, const std::string* src) {
  if (!has_value && !src) { g.kind = DurationGetter::NOOP; return; }
  if (!src) { g.kind = DurationGetter::CONST; g.value = value; return; }
  g.kind = DurationGetter::FROM;
  g.has_value = has_value;
  g.value = value;
  g.q.reset(new Query(*src));
}

// ---------------------------------------------------------------- lifecycle
using StrMap = std::vector<std::pair<std::string, std::string>>;

struct Finalizers {
  std::vector<std::string> add, remove;
  bool empty = false;
};

struct Stage {
  std::string name;
  bool has_labels = false, has_annotations = false;
  StrMap labels, annotations;
  std::vector<Requirement> exprs;
  IntGetter weight;
  bool has_duration = false, has_jitter = false;
  DurationGetter duration, jitter;
  bool has_finalizers = false;
  Finalizers fin;
  bool del = false;
  bool immediate = false;
  bool has_patches = false;

  static bool set_matches(const StrMap& sel, const StrMap& have) {
    // labels.SelectorFromSet: every key present with equal value (empty set => Everything)
    for (auto& kv : sel) {
      bool found = false;
      for (auto& h : have) if (h.first == kv.first) { found = h.second == kv.second; break; }
      if (!found) return false;
    }
    return true;
  }
  bool match(const StrMap& lab, const StrMap& ann, const JVP& data) const {
    if (has_labels && !set_matches(labels, lab)) return false;
    if (has_annotations && !set_matches(annotations, ann)) return false;
    for (auto& r : exprs) if (!r.matches(data)) return false;
    return true;
  }
  // Stage.Delay (lifecycle.go:313-341)
  bool delay(const JVP& v, int64_t now, const Rng& rng, int64_t& out) const {
    out = 0;
    if (!has_duration) return false;
    int64_t d;
    if (!duration.get(v, now, d)) { out = 0; return false; }
    if (!has_jitter) { out = d; return true; }
    int64_t j;
    if (!jitter.get(v, now, j)) { out = d; return true; }
    if (j < d) { out = j; return true; }
    // jitter - duration may overflow int64 in Go (wraps); guard like Go's two's complement
    int64_t diff = (int64_t)((uint64_t)j - (uint64_t)d);
    if (diff > 0) d = (int64_t)((uint64_t)d + (uint64_t)rng.below(SITE_JITTER, diff));
    out = d;
    return true;
  }
};

static StrMap obj_map(const JVP& obj, const char* field) {
  StrMap out;
  if (obj->t != JV::OBJ) return out;
  auto* md = obj->get("metadata");
  if (!md || (*md)->t != JV::OBJ) return out;
  auto* m = (*md)->get(field);
  if (!m || (*m)->t != JV::OBJ) return out;
  for (auto& kv : (*m)->o) if (kv.second->t == JV::STR) out.emplace_back(kv.first, kv.second->s);
  return out;
}

static const JVP* jget(const JVP& o, const char* k) {
  if (!o || o->t != JV::OBJ) return nullptr;
  return o->get(k);
}
static std::string expr_from(const JVP* src) {
  if (!src || (*src)->t != JV::OBJ) return std::string();
  auto* e = (*src)->get("expressionFrom");
  return (e && (*e)->t == JV::STR) ? (*e)->s : std::string();
}

struct Lifecycle {
  std::vector<std::unique_ptr<Stage>> stages;

  // NewStage (lifecycle.go:194-267) from a v1alpha1 Stage object (JSON)
  static std::unique_ptr<Stage> new_stage(const JVP& s) {
    auto st = std::make_unique<Stage>();
    auto* md = jget(s, "metadata");
    if (md) { auto* n = jget(*md, "name"); if (n && (*n)->t == JV::STR) st->name = (*n)->s; }
    auto* spec = jget(s, "spec");
    if (!spec) throw std::runtime_error("stage without spec");
    auto* sel = jget(*spec, "selector");
    if (!sel || (*sel)->t == JV::NUL) return nullptr;  // selector == nil => dropped
    auto read_map = [](const JVP* m, StrMap& out) {
      for (auto& kv : (*m)->o) out.emplace_back(kv.first, kv.second->t == JV::STR ? kv.second->s : dumps(kv.second));
    };
    if (auto* ml = jget(*sel, "matchLabels"); ml && (*ml)->t == JV::OBJ) { st->has_labels = true; read_map(ml, st->labels); }
    if (auto* ma = jget(*sel, "matchAnnotations"); ma && (*ma)->t == JV::OBJ) { st->has_annotations = true; read_map(ma, st->annotations); }
    if (auto* me = jget(*sel, "matchExpressions"); me && (*me)->t == JV::ARR) {
      for (auto& e : (*me)->a) {
        Requirement r;
        auto* key = jget(e, "key");
        auto* op = jget(e, "operator");
        std::string ops = op ? (*op)->s : "";
        r.q.reset(new Query(key ? (*key)->s : ""));
        if (auto* vals = jget(e, "values"); vals && (*vals)->t == JV::ARR)
          for (auto& v : (*vals)->a) r.vals.push_back(v->s);
        if (ops == "In" || ops == "NotIn") {
          if (r.vals.empty()) throw std::runtime_error("for 'in', 'notin' operators, values set can't be empty");
          r.op = ops == "In" ? OP_IN : OP_NOTIN;
        } else if (ops == "Exists" || ops == "DoesNotExist") {
          if (!r.vals.empty()) throw std::runtime_error("values set must be empty for exists and does not exist");
          r.op = ops == "Exists" ? OP_EXISTS : OP_DNE;
        } else {
          throw std::runtime_error("operator \"" + ops + "\" is not supported");
        }
        st->exprs.push_back(std::move(r));
      }
    }
    if (auto* delay = jget(*spec, "delay"); delay && (*delay)->t == JV::OBJ) {
      st->has_duration = true;
      int64_t dms = 0;
      if (auto* x = jget(*delay, "durationMilliseconds"); x && (*x)->t == JV::NUM) dms = (int64_t)(*x)->n;
      auto* dfrom = jget(*delay, "durationFrom");
      std::string dsrc = expr_from(dfrom);
      new_duration_from(st->duration, true, dms * 1000000, dfrom ? &dsrc : nullptr);
      auto* jms = jget(*delay, "jitterDurationMilliseconds");
      auto* jfrom = jget(*delay, "jitterDurationFrom");
      bool has_jms = jms && (*jms)->t == JV::NUM;
      bool has_jfrom = jfrom && (*jfrom)->t != JV::NUL;
      if (has_jms || has_jfrom) {
        st->has_jitter = true;
        std::string jsrc = expr_from(jfrom);
        new_duration_from(st->jitter, has_jms, has_jms ? (int64_t)(*jms)->n * 1000000 : 0, has_jfrom ? &jsrc : nullptr);
      }
    }
    int64_t w = 0;
    if (auto* x = jget(*spec, "weight"); x && (*x)->t == JV::NUM) w = (int64_t)(*x)->n;
    auto* wf = jget(*spec, "weightFrom");
    std::string wsrc = expr_from(wf);
    new_int_from(st->weight, true, w, (wf && (*wf)->t != JV::NUL) ? &wsrc : nullptr);
    if (auto* im = jget(*spec, "immediateNextStage"); im && (*im)->t == JV::BOOL) st->immediate = (*im)->b;
    if (auto* next = jget(*spec, "next"); next && (*next)->t == JV::OBJ) {
      if (auto* f = jget(*next, "finalizers"); f && (*f)->t == JV::OBJ) {
        st->has_finalizers = true;
        if (auto* a = jget(*f, "add"); a && (*a)->t == JV::ARR)
          for (auto& it : (*a)->a) { auto* v = jget(it, "value"); st->fin.add.push_back(v ? (*v)->s : ""); }
        if (auto* r = jget(*f, "remove"); r && (*r)->t == JV::ARR)
          for (auto& it : (*r)->a) { auto* v = jget(it, "value"); st->fin.remove.push_back(v ? (*v)->s : ""); }
        if (auto* e = jget(*f, "empty"); e && (*e)->t == JV::BOOL) st->fin.empty = (*e)->b;
      }
      if (auto* d = jget(*next, "delete"); d && (*d)->t == JV::BOOL) st->del = (*d)->b;
      auto* tpl = jget(*next, "statusTemplate");
      auto* patches = jget(*next, "patches");
      st->has_patches = (tpl && (*tpl)->t == JV::STR && !(*tpl)->s.empty()) ||
                        (patches && (*patches)->t == JV::ARR && !(*patches)->a.empty());
    }
    return st;
  }

  explicit Lifecycle(const JVP& list) {
    if (list->t != JV::ARR) throw std::runtime_error("stages must be a JSON array");
    for (auto& s : list->a) {
      auto st = new_stage(s);
      if (st) stages.push_back(std::move(st));
    }
  }

  void match_all(const StrMap& lab, const StrMap& ann, const JVP& data, std::vector<int>& out) const {
    out.clear();
    for (size_t i = 0; i < stages.size(); ++i) if (stages[i]->match(lab, ann, data)) out.push_back((int)i);
  }

  // ListAllPossible (lifecycle.go:66-122)
  void list_all_possible(const StrMap& lab, const StrMap& ann, const JVP& data, std::vector<int>& res) const {
    std::vector<int> st;
    match_all(lab, ann, data, st);
    res.clear();
    if (st.size() <= 1) { res = st; return; }
    std::vector<int64_t> w;
    int64_t total = 0;
    size_t nerr = 0;
    for (int i : st) {
      int64_t x;
      if (stages[i]->weight.get(data, x)) { total += x; w.push_back(x); }
      else { w.push_back(-1); ++nerr; }
    }
    if (nerr == st.size()) { res = st; return; }
    if (total == 0) {
      if (nerr == 0) { res = st; return; }
      for (size_t k = 0; k < st.size(); ++k) if (w[k] >= 0) res.push_back(st[k]);
      return;
    }
    for (size_t k = 0; k < st.size(); ++k) if (w[k] > 0) res.push_back(st[k]);
  }

  // Match (lifecycle.go:125-191). Returns -1 for nil; -2 when Go would panic
  // (rand.Int63n with a negative total weight).
  int match(const StrMap& lab, const StrMap& ann, const JVP& data, const Rng& rng) const {
    std::vector<int> st;
    match_all(lab, ann, data, st);
    if (st.empty()) return -1;
    if (st.size() == 1) return st[0];
    std::vector<int64_t> w;
    int64_t total = 0;
    int64_t nerr = 0;
    for (int i : st) {
      int64_t x;
      if (stages[i]->weight.get(data, x)) { total = (int64_t)((uint64_t)total + (uint64_t)x); w.push_back(x); }
      else { w.push_back(-1); ++nerr; }
    }
    const int64_t n = (int64_t)st.size();
    if (nerr == n) return st[rng.below(SITE_PICK, n)];
    if (total == 0) {
      if (nerr == 0) return st[rng.below(SITE_PICK, n)];
      std::vector<int> ww;
      for (size_t k = 0; k < st.size(); ++k) if (w[k] >= 0) ww.push_back(st[k]);
      return ww[rng.below(SITE_PICK, (int64_t)ww.size())];
    }
    if (total < 0) return -2;
    int64_t off = rng.below(SITE_PICK, total);
    for (size_t k = 0; k < st.size(); ++k) {
      if (w[k] <= 0) continue;
      off -= w[k];
      if (off < 0) return st[k];
    }
    return st.back();
  }
};

// finalizers.go:32-111
struct JsonPatchOp { std::string op, path; JVP value; };

static std::vector<JsonPatchOp> finalizers_add(const std::vector<std::string>& meta, const std::vector<std::string>& add) {
  std::vector<JsonPatchOp> ops;
  if (!meta.empty()) {
    for (auto& f : add) {
      bool has = false;
      for (auto& m : meta) if (m == f) { has = true; break; }
      if (has) continue;
      ops.push_back({"add", "/metadata/finalizers/-", JV::str(f)});
    }
  } else {
    auto arr = std::make_shared<JV>();
    arr->t = JV::ARR;
    for (auto& f : add) arr->a.push_back(JV::str(f));
    ops.push_back({"add", "/metadata/finalizers", arr});
  }
  return ops;
}
static std::vector<JsonPatchOp> finalizers_remove(const std::vector<std::string>& meta, const std::vector<std::string>& rm) {
  std::vector<JsonPatchOp> ops;
  for (int i = (int)meta.size() - 1; i >= 0; --i) {
    bool has = false;
    for (auto& r : rm) if (r == meta[(size_t)i]) { has = true; break; }
    if (!has) continue;
    ops.push_back({"remove", "/metadata/finalizers/" + std::to_string(i), nullptr});
  }
  return ops;
}
static std::vector<JsonPatchOp> finalizers_modify(const std::vector<std::string>& meta, const Finalizers& f) {
  bool is_empty = false;
  std::vector<JsonPatchOp> ops;
  if (f.empty) {
    is_empty = true;
  } else if (!f.remove.empty()) {
    auto removed = finalizers_remove(meta, f.remove);
    if (removed.size() == meta.size()) is_empty = true;
    else ops.insert(ops.end(), removed.begin(), removed.end());
  }
  if (!is_empty) {
    if (!f.add.empty()) { auto a = finalizers_add(meta, f.add); ops.insert(ops.end(), a.begin(), a.end()); }
  } else {
    if (!meta.empty()) ops.push_back({"remove", "/metadata/finalizers", nullptr});
    if (!f.add.empty()) { auto a = finalizers_add({}, f.add); ops.insert(ops.end(), a.begin(), a.end()); }
  }
  return ops;
}
static std::string ops_json(const std::vector<JsonPatchOp>& ops) {
  std::string s = "[";
  for (size_t i = 0; i < ops.size(); ++i) {
    if (i) s += ",";
    s += "{\"op\":";
    dump_string(s, ops[i].op);
    s += ",\"path\":";
    dump_string(s, ops[i].path);
    if (ops[i].value) { s += ",\"value\":"; dump(s, ops[i].value); }
    s += "}";
  }
  return s + "]";
}

}  // namespace refcpu

using namespace refcpu;

// ---------------------------------------------------------------- C ABI (ctypes)
static thread_local std::string g_err;

static int put(const std::string& s, char* out, int cap) {
  if ((int)s.size() + 1 > cap) return -(int)s.size() - 1;
  memcpy(out, s.c_str(), s.size() + 1);
  return (int)s.size();
}

extern "C" {

const char* rc_last_error() { return g_err.c_str(); }

// One compiled feature of a selector key: bit 0 = the query has an output (Exists), bit 1 + i =
// hasValue(output, literal i) for some output (selector.go:65-120: strings, bools, gojq ints).
// -1 on a query the oracle cannot parse.
int64_t rc_feature(const char* src, const char* obj_json, const char* lits_json) {
  try {
    Query q(src);
    std::vector<JVP> res;
    q.execute(parse_json(obj_json), res);
    JVP lits = parse_json(lits_json);
    int64_t m = res.empty() ? 0 : 1;
    for (size_t i = 0; i < lits->a.size() && i < 62; ++i)
      for (auto& d : res)
        if (Requirement::has_value(d, {lits->a[i]->s})) { m |= (int64_t)1 << (i + 1); break; }
    return m;
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  }
}

// Query.Execute: writes JSON array of outputs, or "null" for the nil result.
int rc_query(const char* src, const char* obj_json, char* out, int cap) {
  try {
    Query q(src);
    std::vector<JVP> res;
    bool ok = q.execute(parse_json(obj_json), res);
    if (!ok) return put("null", out, cap);
    auto arr = std::make_shared<JV>();
    arr->t = JV::ARR;
    arr->a = res;
    return put(dumps(arr), out, cap);
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1000000;
  }
}

// NewRequirement + Matches. returns 0/1, -1 on construction error
int rc_requirement(const char* key, const char* op, const char* vals_json, const char* obj_json) {
  try {
    auto lst = std::make_shared<JV>();
    std::string stage = std::string("[{\"metadata\":{\"name\":\"t\"},\"spec\":{\"selector\":{\"matchExpressions\":[{\"key\":");
    dump_string(stage, key);
    stage += ",\"operator\":";
    dump_string(stage, op);
    stage += ",\"values\":";
    stage += vals_json;
    stage += "}]},\"next\":{}}}]";
    Lifecycle lc(parse_json(stage));
    JVP obj = parse_json(obj_json);
    return lc.stages[0]->exprs[0].matches(obj) ? 1 : 0;
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  }
}

int rc_int_from(int has_value, int64_t value, const char* src, const char* obj_json, int64_t* out) {
  try {
    IntGetter g;
    std::string s = src ? src : "";
    new_int_from(g, has_value != 0, value, src ? &s : nullptr);
    return g.get(parse_json(obj_json), *out) ? 1 : 0;
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  }
}

int rc_duration_from(int has_value, int64_t value, const char* src, const char* obj_json, int64_t now, int64_t* out) {
  try {
    DurationGetter g;
    std::string s = src ? src : "";
    new_duration_from(g, has_value != 0, value, src ? &s : nullptr);
    return g.get(parse_json(obj_json), now, *out) ? 1 : 0;
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  }
}

int rc_parse_int(const char* s, int64_t* out) { return go_parse_int(s, *out) ? 1 : 0; }
int rc_parse_duration(const char* s, int64_t* out) { return go_parse_duration(s, *out) ? 1 : 0; }
int rc_parse_rfc3339(const char* s, int64_t* sec, int32_t* nsec) {
  GoTime t;
  if (!go_parse_rfc3339nano(s, t)) return 0;
  *sec = t.sec;
  *nsec = t.nsec;
  return 1;
}
uint64_t rc_philox_u64(uint64_t seed, uint64_t slot, uint64_t step, uint32_t site) {
  Rng r;
  r.seed = seed; r.slot = slot; r.step = step;
  return r.u64(site);
}

// finalizersModify: meta = JSON array of strings; fin = StageFinalizers JSON
int rc_finalizers_modify(const char* meta_json, const char* fin_json, char* out, int cap) {
  try {
    std::vector<std::string> meta;
    JVP m = parse_json(meta_json);
    if (m->t == JV::ARR) for (auto& x : m->a) meta.push_back(x->s);
    Finalizers f;
    JVP fj = parse_json(fin_json);
    if (auto* a = jget(fj, "add"); a && (*a)->t == JV::ARR) for (auto& it : (*a)->a) f.add.push_back((*jget(it, "value"))->s);
    if (auto* r = jget(fj, "remove"); r && (*r)->t == JV::ARR) for (auto& it : (*r)->a) f.remove.push_back((*jget(it, "value"))->s);
    if (auto* e = jget(fj, "empty"); e && (*e)->t == JV::BOOL) f.empty = (*e)->b;
    return put(ops_json(finalizers_modify(meta, f)), out, cap);
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1000000;
  }
}

void* rc_lifecycle_new(const char* stages_json) {
  try {
    return new Lifecycle(parse_json(stages_json));
  } catch (const std::exception& e) {
    g_err = e.what();
    return nullptr;
  }
}
void rc_lifecycle_free(void* lc) { delete (Lifecycle*)lc; }
int rc_lifecycle_len(void* lc) { return (int)((Lifecycle*)lc)->stages.size(); }
int rc_lifecycle_name(void* lc, int i, char* out, int cap) { return put(((Lifecycle*)lc)->stages[(size_t)i]->name, out, cap); }
// flags: bit0 delete, bit1 immediate, bit2 has_finalizers, bit3 has_patches
int rc_stage_flags(void* lc, int i) {
  const Stage& s = *((Lifecycle*)lc)->stages[(size_t)i];
  return (s.del ? 1 : 0) | (s.immediate ? 2 : 0) | (s.has_finalizers ? 4 : 0) | (s.has_patches ? 8 : 0);
}

// Lifecycle.Match + Stage.Delay for one object. Returns stage index, -1 (nil), -2 (Go panic),
// -3 (object JSON error).
int rc_match(void* lcp, const char* obj_json, int64_t now, uint64_t seed, uint64_t step, uint64_t slot, int64_t* delay_out) {
  const Lifecycle& lc = *(Lifecycle*)lcp;
  JVP obj;
  try { obj = parse_json(obj_json); } catch (const std::exception& e) { g_err = e.what(); return -3; }
  Rng rng;
  rng.seed = seed; rng.slot = slot; rng.step = step;
  StrMap lab = obj_map(obj, "labels"), ann = obj_map(obj, "annotations");
  int s = lc.match(lab, ann, obj, rng);
  if (s >= 0) {
    int64_t d;
    lc.stages[(size_t)s]->delay(obj, now, rng, d);  // controllers ignore `ok` (pod_controller.go:234)
    *delay_out = d;
  }
  return s;
}

// ListAllPossible: returns count, indices into out
int rc_list_all_possible(void* lcp, const char* obj_json, int* out, int cap) {
  const Lifecycle& lc = *(Lifecycle*)lcp;
  try {
    JVP obj = parse_json(obj_json);
    std::vector<int> r;
    lc.list_all_possible(obj_map(obj, "labels"), obj_map(obj, "annotations"), obj, r);
    for (size_t i = 0; i < r.size() && (int)i < cap; ++i) out[i] = r[i];
    return (int)r.size();
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  }
}

// matched set as a bitmask (Lifecycle.match, lifecycle.go:51-63)
int64_t rc_match_mask(void* lcp, const char* obj_json) {
  const Lifecycle& lc = *(Lifecycle*)lcp;
  JVP obj = parse_json(obj_json);
  std::vector<int> r;
  lc.match_all(obj_map(obj, "labels"), obj_map(obj, "annotations"), obj, r);
  int64_t m = 0;
  for (int i : r) m |= (int64_t)1 << i;
  return m;
}

int rc_stage_weight(void* lcp, int i, const char* obj_json, int64_t* out) {
  const Lifecycle& lc = *(Lifecycle*)lcp;
  return lc.stages[(size_t)i]->weight.get(parse_json(obj_json), *out) ? 1 : 0;
}
int rc_stage_delay(void* lcp, int i, const char* obj_json, int64_t now, uint64_t seed, uint64_t step, uint64_t slot, int64_t* out) {
  const Lifecycle& lc = *(Lifecycle*)lcp;
  Rng rng;
  rng.seed = seed; rng.slot = slot; rng.step = step;
  return lc.stages[(size_t)i]->delay(parse_json(obj_json), now, rng, *out) ? 1 : 0;
}
int rc_stage_finalizers(void* lcp, int i, const char* meta_json, char* out, int cap) {
  const Lifecycle& lc = *(Lifecycle*)lcp;
  const Stage& s = *lc.stages[(size_t)i];
  if (!s.has_finalizers) return put("null", out, cap);
  std::vector<std::string> meta;
  JVP m = parse_json(meta_json);
  if (m->t == JV::ARR) for (auto& x : m->a) meta.push_back(x->s);
  return put(ops_json(finalizers_modify(meta, s.fin)), out, cap);
}

// Reference-faithful batch matcher for the CPU baseline: each object is re-parsed from its
// JSON text (the json.Marshal/Unmarshal round trip of ToJSONStandard, query.go:72-88), then
// Match + Delay run exactly as preprocess does (pod_controller.go:216-234).  `nthreads`
// workers split the objects statically (1 = the reference's single preprocess goroutine).
int64_t rc_match_batch(void* lcp, const char* blob, const int64_t* offsets, int64_t n, int64_t now, uint64_t seed,
                       uint64_t step, uint64_t slot_base, int32_t* stage_out, int64_t* delay_out, int nthreads) {
  const Lifecycle& lc = *(Lifecycle*)lcp;
  std::atomic<int64_t> matched{0};
  auto work = [&](int64_t lo, int64_t hi) {
    int64_t local = 0;
    for (int64_t i = lo; i < hi; ++i) {
      JVP obj = JsonParser(blob + offsets[i], (size_t)(offsets[i + 1] - offsets[i])).parse();
      Rng rng;
      rng.seed = seed; rng.slot = slot_base + (uint64_t)i; rng.step = step;
      int s = lc.match(obj_map(obj, "labels"), obj_map(obj, "annotations"), obj, rng);
      int64_t d = 0;
      if (s >= 0) { lc.stages[(size_t)s]->delay(obj, now, rng, d); ++local; }
      stage_out[i] = s;
      delay_out[i] = d;
    }
    matched += local;
  };
  if (nthreads <= 1) {
    work(0, n);
  } else {
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; ++t) th.emplace_back(work, n * t / nthreads, n * (t + 1) / nthreads);
    for (auto& x : th) x.join();
  }
  return matched.load();
}

}  // extern "C"

// ---------------------------------------------------------------- resource.Quantity
// k8s.io/apimachinery v0.30.2 api/resource/quantity.go ParseQuantity + AsApproximateFloat64
// (dependency not vendored in the reference; restated from its published source).  Exact
// arithmetic in __int128: inputs whose Dec-path magnitude exceeds ~1e29 are reported as
// out of the oracle's range (-1).
namespace refcpu {
static double go_pow10(int n) {
  static const double tab[32] = {1e0, 1e1, 1e2, 1e3, 1e4, 1e5, 1e6, 1e7, 1e8, 1e9, 1e10, 1e11, 1e12, 1e13, 1e14, 1e15,
                                 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22, 1e23, 1e24, 1e25, 1e26, 1e27, 1e28, 1e29,
                                 1e30, 1e31};
  static const double pos32[10] = {1e0, 1e32, 1e64, 1e96, 1e128, 1e160, 1e192, 1e224, 1e256, 1e288};
  static const double neg32[11] = {1e-0, 1e-32, 1e-64, 1e-96, 1e-128, 1e-160, 1e-192, 1e-224, 1e-256, 1e-288, 1e-320};
  if (n >= 0 && n <= 308) return pos32[n / 32] * tab[n % 32];
  if (n < 0 && n >= -323) return neg32[(-n) / 32] / tab[(-n) % 32];
  return n > 0 ? HUGE_VAL : 0.0;
}
// returns 1 ok, 0 parse error, -1 outside the oracle's exact range
static int quantity_f64(const std::string& s, double& out) {
  out = 0;
  if (s.empty()) return 0;
  if (s == "0") return 1;
  size_t pos = 0, end = s.size();
  bool positive = true;
  if (s[0] == '-') { positive = false; pos = 1; } else if (s[0] == '+') pos = 1;
  const size_t sign_end = pos;
  while (pos < end && s[pos] == '0') ++pos;
  if (pos >= end) return 1;  // all zeros
  size_t ns = pos;
  while (pos < end && isdigit((unsigned char)s[pos])) ++pos;
  std::string num = s.substr(ns, pos - ns), denom;
  if (num.empty()) num = "0";
  if (pos < end && s[pos] == '.') {
    ++pos;
    size_t ds = pos;
    while (pos < end && isdigit((unsigned char)s[pos])) ++pos;
    denom = s.substr(ds, pos - ds);
  }
  std::string suf = s.substr(pos);
  {  // suffix grammar: [eEinumkKMGTP]* [+-]? [0-9]*
    size_t k = 0;
    while (k < suf.size() && strchr("eEinumkKMGTP", suf[k])) ++k;
    if (k < suf.size() && (suf[k] == '+' || suf[k] == '-')) ++k;
    while (k < suf.size() && isdigit((unsigned char)suf[k])) ++k;
    if (k != suf.size()) return 0;
  }
  int base, exponent;
  bool binary = false;
  static const char* dn[] = {"n", "u", "m", "", "k", "M", "G", "T", "P", "E"};
  static const int de[] = {-9, -6, -3, 0, 3, 6, 9, 12, 15, 18};
  static const char* bn[] = {"Ki", "Mi", "Gi", "Ti", "Pi", "Ei"};
  bool found = false;
  for (int k = 0; k < 10 && !found; ++k) if (suf == dn[k]) { base = 10; exponent = de[k]; found = true; }
  for (int k = 0; k < 6 && !found; ++k) if (suf == bn[k]) { base = 2; exponent = 10 * (k + 1); binary = true; found = true; }
  if (!found) {
    if (suf.size() > 1 && (suf[0] == 'e' || suf[0] == 'E')) {
      int64_t e;
      std::string body = suf.substr(1);
      // strconv.ParseInt(body, 10, 64)
      bool neg = false;
      size_t k = 0;
      if (!body.empty() && (body[0] == '+' || body[0] == '-')) { neg = body[0] == '-'; k = 1; }
      if (k >= body.size()) return 0;
      unsigned __int128 acc = 0;
      for (; k < body.size(); ++k) { if (!isdigit((unsigned char)body[k])) return 0; acc = acc * 10 + (body[k] - '0'); if (acc > ((unsigned __int128)1 << 64)) return 0; }
      if ((!neg && acc > (unsigned __int128)INT64_MAX) || (neg && acc > ((unsigned __int128)1 << 63))) return 0;
      e = neg ? -(int64_t)(uint64_t)acc : (int64_t)(uint64_t)acc;
      base = 10;
      exponent = (int32_t)(uint32_t)(uint64_t)e;
    } else {
      return 0;
    }
  }
  int precision, scale;
  __int128 mantissa = 1;
  if (!binary) {
    scale = exponent;
    precision = 18 - (int)(num.size() + denom.size());
  } else {
    scale = 0;
    if (exponent >= 0 && denom.empty()) {
      mantissa = (__int128)1 << exponent;
      precision = 15 - (int)num.size() - (int)((float)exponent * 3.0f / 10.0f) - 1;
    } else {
      precision = -1;
    }
  }
  if (precision >= 0) {
    scale -= (int)denom.size();
    if (scale >= -9) {
      std::string sh = num + denom;
      unsigned __int128 v = 0;
      for (char c : sh) { v = v * 10 + (c - '0'); if (v > (unsigned __int128)INT64_MAX) return 0; }
      __int128 r = (__int128)v * mantissa;
      if (r <= (__int128)INT64_MAX) {
        int64_t res = positive ? (int64_t)r : -(int64_t)r;
        out = scale == 0 ? (double)res : (double)res * go_pow10(scale);
        return 1;
      }
    }
  }
  // inf.Dec path: amount = (num.denom) * base^exponent, rounded up to 1e-9, as unscaled at scale 9.
  // inf.Dec.SetString needs at least one digit in the text before the suffix.
  {
    bool digit = false;
    for (size_t k = sign_end; k < end && (isdigit((unsigned char)s[k]) || s[k] == '.'); ++k) digit |= s[k] != '.';
    if (!digit) return 0;
  }
  __int128 M = 0;  // digits of num+denom
  for (char c : num + denom) { if (M > ((__int128)1 << 100)) return -1; M = M * 10 + (c - '0'); }
  int dscale = (int)denom.size();  // value = M / 10^dscale
  // value * base^exponent * 1e9, rounded up
  __int128 numer = M, den = 1;
  int p10 = 9 - dscale + (base == 10 ? exponent : 0);
  if (base == 2) { if (exponent > 100) return -1; for (int k = 0; k < exponent; ++k) { numer *= 2; if (numer > ((__int128)1 << 120)) return -1; } }
  if (p10 >= 0) { for (int k = 0; k < p10; ++k) { numer *= 10; if (numer > ((__int128)1 << 120)) return -1; } }
  else { for (int k = 0; k < -p10; ++k) { den *= 10; if (den > ((__int128)1 << 120)) return -1; } }
  __int128 unscaled = numer / den;
  if (numer % den) unscaled += 1;  // RoundUp
  if (binary && unscaled > (__int128)INT64_MAX * 1000000000) unscaled = (__int128)INT64_MAX * 1000000000;
  double b = (double)unscaled;  // round-half-even conversion (big.Float.Float64)
  out = b * go_pow10(-9);
  if (!positive) out = -out;
  return 1;
}
}  // namespace refcpu

extern "C" int rc_quantity(const char* s, double* out) { return refcpu::quantity_f64(s, *out); }

// ---------------------------------------------------------------- SoA step (CPU baseline)
// TIMING BASELINE ONLY (bench.py cpu_baseline leg, SURVEY.md §8(d)(2) "SoA scalar mode on all
// host cores"): the compiled stage program (include/kwok_engine.h layouts, filled by the host
// stage compiler) stepped over integer columns by N threads, the per-object order of the step
// model (harness -> match -> pick -> delay -> fire -> delta) with the Philox hook.  Supports
// programs without value records (every shipped pod-fast / node program); parity is not claimed
// for it — the GPU is checked against the JSON-level oracle above.
#include "../../include/kwok_engine.h"

namespace {
inline bool soa_matches(const kwk_stage_desc& s, uint32_t pred) {
  bool ok = ((pred ^ s.eq_val) & s.eq_mask) == 0;
  for (uint32_t k = 0; k < s.n_any; ++k) ok &= ((pred & s.any_mask[k]) != 0) == (((s.any_want >> k) & 1u) != 0);
  return ok;
}
}  // namespace

extern "C" int64_t rc_soa_steps(const kwk_stage_table* T, const kwk_delta* deltas, const kwk_harness* H, uint32_t* pred,
                                uint32_t* sched, int64_t* due, uint64_t n, int64_t now0, int64_t dt, int steps,
                                uint64_t seed, int nthreads) {
  std::atomic<int64_t> fired{0};
  const uint32_t ns = T->n_stages, fin = T->fin_group_mask;
  auto body = [&](uint64_t lo, uint64_t hi) {
    int64_t f = 0;
    for (int k = 0; k < steps; ++k) {
      const int64_t now = now0 + k * dt;
      Rng rng{seed, 0, (uint64_t)k};
      for (uint64_t i = lo; i < hi; ++i) {
        uint32_t p = pred[i], s = sched[i];
        if (!(s & KWK_F_MANAGED)) continue;
        if (H->enable) {
          if (!(s & KWK_F_ALIVE)) {
            p &= H->keep_mask;
            s = (s & (KWK_F_MANAGED | KWK_F_HASREC | KWK_CLASS_MASK)) | KWK_F_ALIVE | KWK_F_DIRTY | KWK_STAGE_NONE;
          } else if ((p & H->terminal_mask) && !(p & H->deletion_bit)) {
            p |= H->deletion_bit;
            s |= KWK_F_DIRTY;
          }
        }
        if (s & KWK_F_ALIVE) {
          if (s & KWK_F_DIRTY) {
            s &= ~(KWK_F_DIRTY | KWK_F_MATCHERR);
            uint32_t m = 0;
            for (uint32_t j = 0; j < ns; ++j) m |= (soa_matches(T->stages[j], p) ? 1u : 0u) << j;
            if (m) {
              rng.slot = i;
              int pick = __builtin_ctz(m);
              const int cnt = __builtin_popcount(m);
              if (cnt > 1) {
                int64_t total = 0;
                for (uint32_t mm = m; mm; mm &= mm - 1) total += T->stages[__builtin_ctz(mm)].weight_default;
                if (total <= 0) {
                  int64_t want = rng.below(SITE_PICK, cnt);
                  uint32_t mm = m;
                  while (want-- > 0) mm &= mm - 1;
                  pick = __builtin_ctz(mm);
                } else {
                  int64_t off = rng.below(SITE_PICK, total);
                  for (uint32_t mm = m; mm; mm &= mm - 1) {
                    const int j = __builtin_ctz(mm);
                    const int64_t w = T->stages[j].weight_default;
                    if (w <= 0) continue;
                    off -= w;
                    if (off < 0) { pick = j; break; }
                  }
                }
              }
              const kwk_stage_desc& S = T->stages[pick];
              int64_t delay = S.has_delay ? S.delay_default : 0;
              if (S.has_delay && S.has_jitter && S.jitter_default_ok) {
                if (S.jitter_default < delay) delay = S.jitter_default;
                else if (S.jitter_default > delay) delay += rng.below(SITE_JITTER, S.jitter_default - delay);
              }
              s = (s & ~0xFFu) | (uint32_t)pick;
              due[i] = now + delay;
            }
          }
          const uint32_t st = s & 0xFFu;
          if (st < ns && due[i] <= now) {
            const kwk_stage_desc& S = T->stages[st];
            bool rematch = (S.flags & KWK_NEXT_PATCHES) && (!(S.flags & KWK_NEXT_PATCH_STATIC) || !(p & S.applied_mask));
            if (S.flags & KWK_NEXT_FIN) {
              const uint32_t F = p & fin;
              const uint32_t F2 = ((S.flags & KWK_NEXT_FIN_EMPTY) || ((S.flags & KWK_NEXT_FIN_REMOVE) && (F & ~S.fin_remove) == 0))
                                      ? S.fin_add : ((F & ~S.fin_remove) | (S.fin_add & ~F));
              rematch |= F2 != F;
              p = (p & ~fin) | F2;
            }
            if (S.flags & KWK_NEXT_DELETE) {
              s &= ~KWK_F_ALIVE;
              rematch = false;
            } else if (S.flags & KWK_NEXT_PATCHES) {
              const kwk_delta d = deltas[(s >> KWK_CLASS_SHIFT) * ns + st];
              p = (((p & d.and_mask) | d.or_mask) & ~fin) | (p & fin);
            }
            if (rematch) s |= KWK_F_DIRTY;
            s |= KWK_STAGE_NONE;
            ++f;
          }
        }
        pred[i] = p;
        sched[i] = s;
      }
    }
    fired += f;
  };
  const int T_ = nthreads > 0 ? nthreads : 1;
  std::vector<std::thread> th;
  for (int t = 0; t < T_; ++t) {
    const uint64_t lo = n * (uint64_t)t / (uint64_t)T_, hi = n * (uint64_t)(t + 1) / (uint64_t)T_;
    th.emplace_back(body, lo, hi);
  }
  for (auto& t : th) t.join();
  return fired.load();
}
