// Native ingestion encoder: informer objects (JSON) -> the engine's
// interchange rows, without per-object Python.
//
// Reference: the per-event work of PodController.watchResources / preprocess
// (pkg/kwok/controllers/pod_controller.go:196-254, 412-478): ToJSONStandard
// (pkg/utils/expression/query.go:72-88) and one gojq run per selector requirement and *From
// getter (selector.go:65-120, value_int_from.go:53-81, value_duration_from.go:53-79).  Here each
// object is parsed once; the stage compiler's feature queries — compiled by the host into
// step programs (kwok_amd/host/encoder.py: field / iterate / select-equal) — produce its
// feature bits, the *From getters its pre-parsed value record (Go strconv.ParseInt(s, 0, 0),
// time.ParseDuration, time.Parse(RFC3339Nano)), and its spec shape its delta class.  Threads
// encode disjoint ranges; records are interned afterwards in object order, so ids are
// deterministic.  The encoder is the product mirror of kwok_amd/host/engine.py:Ingest (which
// tests/test_encoder.py checks it against on every object of the C2 workload).
#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/kwok_engine.h"
#include "../../include/kwok_encoder.h"
#include "host_common.hpp"
#include "labelsel.hpp"
#include "nextstate.hpp"

namespace {

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

using kwkjson::JV;
using kwkjson::Parser;
using namespace kwkhost;

// ------------------------------------------------------------------ Go parsers
// strconv.ParseInt(s, 0, 0), time.ParseDuration, time.Parse(RFC3339Nano, s) (Go 1.22),
// as kwok_amd/host/goparse.py restates them for the host's Ingest
char lower(char c) { return (c >= 'A' && c <= 'Z') ? (char)(c + 32) : c; }

bool underscore_ok(std::string s) {
  char saw = '^';
  size_t i = 0;
  if (!s.empty() && (s[0] == '+' || s[0] == '-')) s = s.substr(1);
  bool hexa = false;
  if (s.size() >= 2 && s[0] == '0' && (lower(s[1]) == 'b' || lower(s[1]) == 'o' || lower(s[1]) == 'x')) {
    i = 2;
    saw = '0';
    hexa = lower(s[1]) == 'x';
  }
  for (; i < s.size(); ++i) {
    const char c = s[i];
    if ((c >= '0' && c <= '9') || (hexa && lower(c) >= 'a' && lower(c) <= 'f')) saw = '0';
    else if (c == '_') {
      if (saw != '0') return false;
      saw = '_';
    } else {
      if (saw == '_') return false;
      saw = '!';
    }
  }
  return saw != '_';
}

bool parse_int(const std::string& s, int64_t& out) {
  if (s.empty()) return false;
  bool neg = false;
  std::string body = s;
  if (body[0] == '+') body = body.substr(1);
  else if (body[0] == '-') { neg = true; body = body.substr(1); }
  if (body.empty()) return false;
  const std::string s0 = body;
  int base = 10;
  if (body[0] == '0') {
    if (body.size() >= 3 && lower(body[1]) == 'b') { base = 2; body = body.substr(2); }
    else if (body.size() >= 3 && lower(body[1]) == 'o') { base = 8; body = body.substr(2); }
    else if (body.size() >= 3 && lower(body[1]) == 'x') { base = 16; body = body.substr(2); }
    else { base = 8; body = body.substr(1); }
  }
  unsigned __int128 n = 0;
  bool underscores = false;
  for (char c : body) {
    if (c == '_') { underscores = true; continue; }
    int d;
    if (c >= '0' && c <= '9') d = c - '0';
    else if (lower(c) >= 'a' && lower(c) <= 'z') d = lower(c) - 'a' + 10;
    else return false;
    if (d >= base) return false;
    n = n * (unsigned)base + (unsigned)d;
    if (n > (unsigned __int128)UINT64_MAX) return false;
  }
  if (underscores && !underscore_ok(s0)) return false;
  if (!neg && n >= ((unsigned __int128)1 << 63)) return false;
  if (neg && n > ((unsigned __int128)1 << 63)) return false;
  out = neg ? (int64_t)(-(__int128)n) : (int64_t)n;
  return true;
}

bool parse_duration(const std::string& orig, int64_t& out) {
  std::string s = orig;
  const unsigned __int128 lim = (unsigned __int128)1 << 63;
  unsigned __int128 d = 0;
  bool neg = false;
  if (!s.empty() && (s[0] == '+' || s[0] == '-')) { neg = s[0] == '-'; s = s.substr(1); }
  if (s == "0") { out = 0; return true; }
  if (s.empty()) return false;
  static const std::pair<const char*, uint64_t> units[] = {{"ns", 1ull}, {"us", 1000ull}, {"\xC2\xB5s", 1000ull},
                                                            {"\xCE\xBCs", 1000ull}, {"ms", 1000000ull},
                                                            {"s", 1000000000ull}, {"m", 60000000000ull},
                                                            {"h", 3600000000000ull}};
  while (!s.empty()) {
    if (!(s[0] == '.' || (s[0] >= '0' && s[0] <= '9'))) return false;
    size_t i = 0;
    unsigned __int128 v = 0;
    while (i < s.size() && s[i] >= '0' && s[i] <= '9') {
      if (v > lim / 10) return false;
      v = v * 10 + (unsigned)(s[i] - '0');
      if (v > lim) return false;
      ++i;
    }
    const bool pre = i > 0;
    s = s.substr(i);
    bool post = false;
    unsigned __int128 f = 0;
    double scale = 1.0;
    if (!s.empty() && s[0] == '.') {
      s = s.substr(1);
      size_t j = 0;
      bool overflow = false;
      while (j < s.size() && s[j] >= '0' && s[j] <= '9') {
        if (!overflow) {
          if (f > (lim - 1) / 10) overflow = true;
          else {
            const unsigned __int128 y = f * 10 + (unsigned)(s[j] - '0');
            if (y > lim) overflow = true;
            else { f = y; scale *= 10; }
          }
        }
        ++j;
      }
      post = j > 0;
      s = s.substr(j);
    }
    if (!pre && !post) return false;
    size_t k = 0;
    while (k < s.size() && !(s[k] == '.' || (s[k] >= '0' && s[k] <= '9'))) ++k;
    if (k == 0) return false;
    const std::string u = s.substr(0, k);
    s = s.substr(k);
    uint64_t unit = 0;
    for (const auto& un : units)
      if (u == un.first) unit = un.second;
    if (!unit) return false;
    if (v > lim / unit) return false;
    v *= unit;
    if (f > 0) {
      v += (unsigned __int128)(int64_t)((double)(uint64_t)f * ((double)unit / scale));
      if (v > lim) return false;
    }
    d += v;
    if (d > lim) return false;
  }
  if (neg) { out = (int64_t)(-(__int128)d); return true; }
  if (d > lim - 1) return false;
  out = (int64_t)d;
  return true;
}

int days_in(int m, int64_t y) {
  if (m == 2) return (y % 4 == 0 && (y % 100 != 0 || y % 400 == 0)) ? 29 : 28;
  static const int d[] = {31, 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
  return d[m - 1];
}

bool digits(const std::string& s, size_t pos, size_t n, int64_t& v) {
  if (pos + n > s.size()) return false;
  v = 0;
  for (size_t i = pos; i < pos + n; ++i) {
    if (s[i] < '0' || s[i] > '9') return false;
    v = v * 10 + (s[i] - '0');
  }
  return true;
}

int64_t nanos(const std::string& frac_with_sep, size_t nbytes) {
  nbytes = std::min<size_t>(nbytes, 10);
  int64_t ns = 0;
  for (size_t i = 1; i < nbytes; ++i) ns = ns * 10 + (frac_with_sep[i] - '0');
  for (size_t i = nbytes; i < 10; ++i) ns *= 10;
  return ns;
}

int64_t epoch(int64_t y, int64_t mo, int64_t d, int64_t h, int64_t mi, int64_t se, int64_t zone) {
  const int64_t yy = y - (mo <= 2 ? 1 : 0);
  const int64_t era = (yy >= 0 ? yy : yy - 399) / 400;
  const int64_t yoe = yy - era * 400;
  const int64_t doy = (153 * (mo + (mo > 2 ? -3 : 9)) + 2) / 5 + d - 1;
  const int64_t doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
  const int64_t days = era * 146097 + doe - 719468;
  return days * 86400 + h * 3600 + mi * 60 + se - zone;
}

bool rfc3339_fast(const std::string& s, int64_t& sec, int32_t& nsec) {
  if (s.size() < 19) return false;
  int64_t y, mo, d, h, mi, se;
  if (!digits(s, 0, 4, y) || !digits(s, 5, 2, mo) || !digits(s, 8, 2, d) || !digits(s, 11, 2, h) ||
      !digits(s, 14, 2, mi) || !digits(s, 17, 2, se))
    return false;
  if (mo < 1 || mo > 12 || d < 1 || d > days_in((int)mo, y) || h > 23 || mi > 59 || se > 59) return false;
  if (!(s[4] == '-' && s[7] == '-' && s[10] == 'T' && s[13] == ':' && s[16] == ':')) return false;
  std::string rest = s.substr(19);
  int64_t ns = 0;
  if (rest.size() >= 2 && rest[0] == '.' && rest[1] >= '0' && rest[1] <= '9') {
    size_t n = 2;
    while (n < rest.size() && rest[n] >= '0' && rest[n] <= '9') ++n;
    ns = nanos(rest, n);
    rest = rest.substr(n);
  }
  int64_t zone = 0;
  if (rest != "Z") {
    if (rest.size() != 6) return false;
    int64_t hr, mm;
    if (!digits(rest, 1, 2, hr) || !digits(rest, 4, 2, mm) || hr > 23 || mm > 59) return false;
    if ((rest[0] != '+' && rest[0] != '-') || rest[3] != ':') return false;
    zone = (hr * 60 + mm) * 60 * (rest[0] == '-' ? -1 : 1);
  }
  sec = epoch(y, mo, d, h, mi, se, zone);
  nsec = (int32_t)ns;
  return true;
}

bool rfc3339_generic(const std::string& v, int64_t& sec, int32_t& nsec) {
  size_t p = 0;
  int64_t y, mo, d, mi, se;
  auto at = [&](size_t i) { return i < v.size() ? v[i] : '\0'; };
  if (!digits(v, p, 4, y)) return false;
  p += 4;
  if (at(p) != '-') return false;
  ++p;
  if (!digits(v, p, 2, mo)) return false;
  p += 2;
  if (at(p) != '-') return false;
  ++p;
  if (!digits(v, p, 2, d)) return false;
  p += 2;
  if (at(p) != 'T') return false;
  ++p;
  if (!(at(p) >= '0' && at(p) <= '9')) return false;
  int64_t h = at(p) - '0';
  ++p;
  if (at(p) >= '0' && at(p) <= '9') { h = h * 10 + (at(p) - '0'); ++p; }
  if (at(p) != ':') return false;
  ++p;
  if (!digits(v, p, 2, mi)) return false;
  p += 2;
  if (at(p) != ':') return false;
  ++p;
  if (!digits(v, p, 2, se)) return false;
  p += 2;
  int64_t ns = 0;
  if (p + 1 < v.size() && (v[p] == '.' || v[p] == ',') && v[p + 1] >= '0' && v[p + 1] <= '9') {
    size_t i = 0;
    while (p + i + 1 < v.size() && v[p + i + 1] >= '0' && v[p + i + 1] <= '9') ++i;
    ns = nanos(v.substr(p), 1 + i);
    p += 1 + i;
  }
  int64_t zone = 0;
  if (at(p) == 'Z') {
    ++p;
  } else {
    if (v.size() - p < 6 || v[p + 3] != ':') return false;
    int64_t hr, mm;
    if (!digits(v, p + 1, 2, hr) || !digits(v, p + 4, 2, mm) || hr > 24 || mm > 60 || (v[p] != '+' && v[p] != '-'))
      return false;
    zone = (hr * 60 + mm) * 60 * (v[p] == '-' ? -1 : 1);
    p += 6;
  }
  if (p != v.size()) return false;
  if (mo < 1 || mo > 12 || h >= 24 || mi >= 60 || se >= 60 || d < 1 || d > days_in((int)mo, y)) return false;
  sec = epoch(y, mo, d, h, mi, se, zone);
  nsec = (int32_t)ns;
  return true;
}

bool parse_rfc3339(const std::string& s, int64_t& sec, int32_t& nsec) {
  return rfc3339_fast(s, sec, nsec) || rfc3339_generic(s, sec, nsec);
}

// Go int64(float64) on amd64: NaN / out of range -> INT64_MIN
int64_t f64_to_i64(double x) {
  if (x != x || !(x >= -9223372036854775808.0 && x < 9223372036854775808.0)) return INT64_MIN;
  return (int64_t)x;
}

}  // namespace

// ------------------------------------------------------------------ encoder
struct kwk_encoder {
  std::string err;  // message of the last failing call on this handle
  struct Feature {
    CQuery q;
    int32_t present_bit = -1;
    std::vector<std::pair<std::string, uint32_t>> lits;
  };
  struct Slot {
    bool duration = false;
    CQuery q;
  };
  std::vector<Feature> features;
  std::vector<std::pair<std::string, uint32_t>> fin_bits;
  int32_t fin_other_bit = -1;
  std::vector<Slot> slots;
  // "patch already applied" feature bits (compiler._patch_applied): the stage's patches
  struct Applied {
    int bit;
    std::vector<kwknext::Patch> patches;
  };
  std::vector<Applied> applied;
  kwklabels::Disregard disregard;  // need()'s selectors -> one feature bit
  int disregard_bit = -1;
  std::unordered_map<std::string, uint32_t> classes;
  std::vector<std::string> identity_meta;
  // interned value records (kwk_value x slots each), in order of first appearance
  std::vector<kwk_value> records;
  std::unordered_map<std::string, uint32_t> record_ids;
  uint64_t encoded = 0;
};

namespace {

// per-object result before record interning
struct Row {
  uint32_t pred = 0, flags = 0;
  int64_t del = KWK_DEL_ABSENT;
  uint32_t cls = 0;
  bool has_rec = false;
  std::vector<kwk_value> rec;
  std::string err;
};

void encode_one(const kwk_encoder& E, const char* text, uint32_t len, Row& r, kwktpl::Renderer* R) {
  JV obj;
  Parser P{text, text + len};
  if (!P.value(obj) || obj.t != JV::OBJ) { r.err = "invalid JSON object"; return; }
  typed_presence(obj);
  std::vector<kwkjq::Val> out;
  // feature bits (KindProgram.pred_of)
  for (const auto& f : E.features) {
    if (!exec_query(f.q, obj, out) || out.empty()) continue;
    if (f.present_bit >= 0) r.pred |= 1u << f.present_bit;
    for (const auto& lit : f.lits) {
      for (const kwkjq::Val& d : out) {
        // selector.go hasValue: strings, bools via FormatBool, gojq ints via FormatInt; JSON
        // numbers (float64) never match
        if (kwkjq::has_value(*d.p, lit.first)) {
          r.pred |= 1u << lit.second;
          break;
        }
      }
    }
  }
  for (const auto& ap : E.applied)
    if (kwknext::patch_applied(ap.patches, obj, *R)) r.pred |= 1u << ap.bit;
  if (E.disregard_bit >= 0 && E.disregard.disregarded(obj)) r.pred |= 1u << E.disregard_bit;
  const JV* md = obj.get("metadata");
  if (E.fin_other_bit >= 0 && md && md->t == JV::OBJ) {
    if (const JV* fins = md->get("finalizers"))
      if (fins->t == JV::ARR)
        for (const JV& x : fins->a) {
          int32_t b = E.fin_other_bit;
          if (x.t == JV::STR)
            for (const auto& fb : E.fin_bits)
              if (fb.first == x.s) b = (int32_t)fb.second;
          r.pred |= 1u << b;
        }
  }
  // value record (KindProgram.record_of)
  bool any = false;
  r.rec.assign(E.slots.size(), kwk_value{0, 0, KWK_V_DEFAULT});
  for (size_t s = 0; s < E.slots.size(); ++s) {
    if (!exec_query(E.slots[s].q, obj, out) || out.empty()) continue;
    const JV* t = out[0].p;
    kwk_value& v = r.rec[s];
    if (!E.slots[s].duration) {  // int64From.Get (value_int_from.go:53-81)
      if (t->t == JV::STR) {
        int64_t n;
        if (t->s.empty() || !parse_int(t->s, n)) v = kwk_value{0, 0, KWK_V_NOTOK};
        else v = kwk_value{n, 0, KWK_V_OK};
      } else if (t->t == JV::NUM && !kwkjq::is_gint(*t)) {  // float64 (a gojq int: the default)
        v = kwk_value{f64_to_i64(strtod(t->s.c_str(), nullptr)), 0, KWK_V_OK};
      }
    } else {  // durationFrom.Get (value_duration_from.go:53-79)
      if (t->t == JV::STR) {
        int64_t sec, d;
        int32_t ns;
        if (t->s.empty()) v = kwk_value{0, 0, KWK_V_NOTOK};
        else if (parse_rfc3339(t->s, sec, ns)) v = kwk_value{sec, ns, KWK_V_ABSTIME};
        else if (parse_duration(t->s, d)) v = kwk_value{d, 0, KWK_V_OK};
        else v = kwk_value{0, 0, KWK_V_NOTOK};
      } else {
        v = kwk_value{0, 0, KWK_V_NOTOK};
      }
    }
    any |= v.kind != KWK_V_DEFAULT;
  }
  r.has_rec = any;
  r.flags = KWK_F_ALIVE | KWK_F_MANAGED | KWK_F_DIRTY | (any ? KWK_F_HASREC : 0u);
  // deletion column (KindProgram.deletion_s)
  if (md && md->t == JV::OBJ)
    if (const JV* ts = md->get("deletionTimestamp"))
      if (ts->t == JV::STR && !ts->s.empty()) {
        int64_t sec;
        int32_t ns;
        if (!parse_rfc3339(ts->s, sec, ns)) { r.err = "deletionTimestamp is not RFC3339"; return; }
        r.del = sec;
      }
  // delta class
  const auto it = E.classes.find(class_key(obj, E.identity_meta));
  r.cls = it == E.classes.end() ? KWK_ENCODE_CLASS_UNKNOWN : it->second;
}

}  // namespace

extern "C" {

const char* kwk_encoder_last_error(const kwk_encoder* h) { return h ? h->err.c_str() : g_err.c_str(); }

kwk_status kwk_encoder_create(const char* spec_json, kwk_encoder** out) {
  if (!spec_json || !out) return fail(KWK_EINVAL, "null argument");
  JV spec;
  Parser P{spec_json, spec_json + strlen(spec_json)};
  if (!P.value(spec) || spec.t != JV::OBJ) return fail(KWK_EINVAL, "encoder spec: invalid JSON");
  std::unique_ptr<kwk_encoder> E(new kwk_encoder());
  const JV* feats = spec.get("features");
  if (!feats || feats->t != JV::ARR) return fail(KWK_EINVAL, "encoder spec: features");
  for (const JV& f : feats->a) {
    kwk_encoder::Feature F;
    const JV* src = f.get("query");
    if (!src || src->t != JV::STR) return fail(KWK_EINVAL, "encoder spec: feature query");
    try {
      F.q = compile_query(src->s);
    } catch (const kwkjq::Unsupported& e) {
      return fail(KWK_EINVAL, std::string("encoder spec: ") + e.what());
    }
    const JV* pb = f.get("present_bit");
    F.present_bit = (pb && pb->t == JV::NUM) ? atoi(pb->s.c_str()) : -1;
    if (const JV* lits = f.get("literals"))
      for (size_t i = 0; i < lits->k.size(); ++i) F.lits.emplace_back(lits->k[i], (uint32_t)atoi(lits->a[i].s.c_str()));
    E->features.push_back(std::move(F));
  }
  if (const JV* fb = spec.get("finalizers"))
    for (size_t i = 0; i < fb->k.size(); ++i) E->fin_bits.emplace_back(fb->k[i], (uint32_t)atoi(fb->a[i].s.c_str()));
  if (const JV* fo = spec.get("finalizer_other_bit")) E->fin_other_bit = fo->t == JV::NUM ? atoi(fo->s.c_str()) : -1;
  if (const JV* slots = spec.get("slots"))
    for (const JV& s : slots->a) {
      kwk_encoder::Slot S;
      const JV* typ = s.get("type");
      S.duration = typ && typ->t == JV::STR && typ->s == "duration";
      const JV* src = s.get("query");
      if (!src || src->t != JV::STR) return fail(KWK_EINVAL, "encoder spec: slot query");
      try {
        S.q = compile_query(src->s);
      } catch (const kwkjq::Unsupported& e) {
        return fail(KWK_EINVAL, std::string("encoder spec: ") + e.what());
      }
      E->slots.push_back(std::move(S));
    }
  if (const JV* cls = spec.get("classes"))
    for (size_t i = 0; i < cls->k.size(); ++i) E->classes[cls->k[i]] = (uint32_t)atoi(cls->a[i].s.c_str());
  if (const JV* ap = spec.get("applied"))
    for (const JV& a : ap->a) {
      kwk_encoder::Applied A;
      const JV* bit = a.get("bit");
      const JV* ps = a.get("patches");
      if (!bit || bit->t != JV::NUM || !ps || ps->t != JV::ARR) return fail(KWK_EINVAL, "encoder spec: applied");
      A.bit = atoi(bit->s.c_str());
      for (const JV& p : ps->a) {
        kwknext::Patch P;
        const JV* t = p.get("type");
        const JV* root = p.get("root");
        const JV* tm = p.get("template");
        if (!t || !root || !tm) return fail(KWK_EINVAL, "encoder spec: applied patch");
        P.type = t->s;
        P.root = root->s;
        P.tmpl = tm->s;
        A.patches.push_back(std::move(P));
      }
      E->applied.push_back(std::move(A));
    }
  if (const JV* dg = spec.get("disregard"); dg && dg->t == JV::OBJ) {
    const JV* bit = dg->get("bit");
    const JV* a = dg->get("annotation_selector");
    const JV* l = dg->get("label_selector");
    if (!bit || bit->t != JV::NUM || !a || a->t != JV::STR || !l || l->t != JV::STR)
      return fail(KWK_EINVAL, "encoder spec: disregard");
    try {
      E->disregard = kwklabels::Disregard(a->s, l->s);
    } catch (const std::exception& ex) {
      return fail(KWK_EINVAL, std::string("encoder spec: disregard selector: ") + ex.what());
    }
    E->disregard_bit = atoi(bit->s.c_str());
  }
  if (const JV* im = spec.get("identity_meta"))
    for (const JV& k : im->a) E->identity_meta.push_back(k.s);
  *out = E.release();
  return KWK_OK;
}

kwk_status kwk_encoder_destroy(kwk_encoder* e) {
  ErrScope es_(e ? &e->err : nullptr);
  delete e;
  return KWK_OK;
}

kwk_status kwk_encode(kwk_encoder* E, uint32_t n, const char* buf, const uint64_t* offsets, uint32_t n_threads,
                      kwk_hot* hot, int64_t* deletion_s, uint32_t* rec_idx, uint16_t* cls, uint32_t* n_unknown_class) {
  ErrScope es_(E ? &E->err : nullptr);
  if (!E || (n && (!buf || !offsets || !hot || !deletion_s || !rec_idx || !cls))) return fail(KWK_EINVAL, "null argument");
  for (uint32_t i = 0; i < n; ++i)
    if (offsets[i + 1] < offsets[i]) return fail(KWK_EINVAL, "offsets must be non-decreasing");
  std::vector<Row> rows(n);
  const uint32_t T = std::max<uint32_t>(1, std::min<uint32_t>(n_threads ? n_threads : 1, 256));
  std::atomic<uint32_t> next{0};
  auto work = [&]() {
    // one renderer per thread (its template cache), for the "patch already applied" bits
    std::unique_ptr<kwktpl::Renderer> R;
    if (!E->applied.empty()) R.reset(new kwktpl::Renderer(kwknext::static_renderer()));
    for (;;) {
      const uint32_t lo = next.fetch_add(256);
      if (lo >= n) return;
      const uint32_t hi = std::min(n, lo + 256);
      for (uint32_t i = lo; i < hi; ++i)
        encode_one(*E, buf + offsets[i], (uint32_t)(offsets[i + 1] - offsets[i]), rows[i], R.get());
    }
  };
  if (T == 1 || n < 512) {
    work();
  } else {
    std::vector<std::thread> th;
    for (uint32_t t = 0; t < T; ++t) th.emplace_back(work);
    for (auto& t : th) t.join();
  }
  uint32_t unknown = 0;
  const size_t rb = sizeof(kwk_value) * E->slots.size();
  for (uint32_t i = 0; i < n; ++i) {  // record interning in object order: deterministic ids
    Row& r = rows[i];
    if (!r.err.empty()) return fail(KWK_EINVAL, "object " + std::to_string(i) + ": " + r.err);
    uint32_t rid = 0;
    if (r.has_rec) {
      std::string key(reinterpret_cast<const char*>(r.rec.data()), rb);
      auto it = E->record_ids.find(key);
      if (it == E->record_ids.end()) {
        rid = (uint32_t)(E->records.size() / std::max<size_t>(1, E->slots.size()));
        E->record_ids.emplace(std::move(key), rid);
        E->records.insert(E->records.end(), r.rec.begin(), r.rec.end());
      } else {
        rid = it->second;
      }
    }
    hot[i] = kwk_hot{r.pred, r.flags | KWK_STAGE_NONE, 0};
    deletion_s[i] = r.del;
    rec_idx[i] = rid;
    cls[i] = (uint16_t)(r.cls == KWK_ENCODE_CLASS_UNKNOWN ? 0xFFFFu : r.cls);
    unknown += r.cls == KWK_ENCODE_CLASS_UNKNOWN;
  }
  E->encoded += n;
  if (n_unknown_class) *n_unknown_class = unknown;
  return KWK_OK;
}

kwk_status kwk_encoder_add_classes(kwk_encoder* E, const char* classes_json) {
  ErrScope es_(E ? &E->err : nullptr);
  if (!E || !classes_json) return fail(KWK_EINVAL, "null argument");
  JV cls;
  Parser P{classes_json, classes_json + strlen(classes_json)};
  if (!P.value(cls) || cls.t != JV::OBJ) return fail(KWK_EINVAL, "classes: invalid JSON object");
  for (size_t i = 0; i < cls.k.size(); ++i) {
    if (cls.a[i].t != JV::NUM || !cls.a[i].is_int) return fail(KWK_EINVAL, "classes: ids must be integers");
    const long id = atol(cls.a[i].s.c_str());
    if (id < 0 || id >= 0xFFFF) return fail(KWK_EINVAL, "classes: id out of range");
    const auto it = E->classes.find(cls.k[i]);
    if (it != E->classes.end() && it->second != (uint32_t)id) return fail(KWK_EINVAL, "classes: a known class changes its id");
    E->classes[cls.k[i]] = (uint32_t)id;
  }
  return KWK_OK;
}

kwk_status kwk_encoder_records(kwk_encoder* E, kwk_value* out, uint32_t cap, uint32_t* n_records) {
  ErrScope es_(E ? &E->err : nullptr);
  if (!E || !n_records) return fail(KWK_EINVAL, "null argument");
  const size_t per = std::max<size_t>(1, E->slots.size());
  const uint32_t n = (uint32_t)(E->slots.empty() ? 0 : E->records.size() / per);
  *n_records = n;
  if (!out || !n) return KWK_OK;
  if (n > cap) return fail(KWK_ECAP, "record buffer too small");
  memcpy(out, E->records.data(), sizeof(kwk_value) * E->records.size());
  return KWK_OK;
}

kwk_status kwk_jq_eval(const char* query, const char* json, char* out, uint32_t cap, uint32_t* n_out) {
  ErrScope es_(nullptr);
  if (!query || !json || !n_out || (cap && !out)) return fail(KWK_EINVAL, "null argument");
  JV doc;
  Parser P{json, json + strlen(json)};
  if (!P.value(doc)) return fail(KWK_EINVAL, "invalid JSON input");
  std::string text;
  try {
    const CQuery q = compile_query(query);
    std::vector<kwkjq::Val> res;
    if (!exec_query(q, doc, res)) {
      text = "null";
    } else {
      text = "[";
      for (size_t i = 0; i < res.size(); ++i) {
        if (i) text += ',';
        kwkjq::encode(text, *res[i].p);
      }
      text += "]";
    }
  } catch (const kwkjq::Unsupported& e) {
    return fail(KWK_EINVAL, e.what());
  }
  *n_out = (uint32_t)text.size();
  if (text.size() + 1 > cap) return fail(KWK_ECAP, "output buffer too small: need " + std::to_string(text.size() + 1));
  memcpy(out, text.c_str(), text.size() + 1);
  return KWK_OK;
}

}  // extern "C"
