// Host-side pieces shared by the native host libraries (encoder.cpp, compiler.cpp): the
// canonical JSON of the host compiler's class keys (Python json.dumps(sort_keys=True)), the jq
// query step programs, typed-object presence (ToJSONStandard) and the delta class key.
#pragma once
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "jqc.hpp"
#include "json_dom.hpp"

namespace kwkhost {

using kwkjson::JV;
using kwkjson::Parser;

// ------------------------------------------------------------------ canonical JSON (class keys)
// json.dumps(o, sort_keys=True, separators=(",", ":")) as the host compiler's class_key writes it
// (ensure_ascii escapes, Python float repr)
inline void esc(std::string& o, const std::string& s) {
  o += '"';
  size_t i = 0;
  while (i < s.size()) {
    unsigned char c = (unsigned char)s[i];
    uint32_t cp;
    int n;
    if (c < 0x80) { cp = c; n = 1; }
    else if ((c >> 5) == 6 && i + 1 < s.size()) { cp = ((c & 0x1F) << 6) | (s[i + 1] & 0x3F); n = 2; }
    else if ((c >> 4) == 14 && i + 2 < s.size()) { cp = ((c & 0x0F) << 12) | ((s[i + 1] & 0x3F) << 6) | (s[i + 2] & 0x3F); n = 3; }
    else if (i + 3 < s.size()) { cp = ((c & 0x07) << 18) | ((s[i + 1] & 0x3F) << 12) | ((s[i + 2] & 0x3F) << 6) | (s[i + 3] & 0x3F); n = 4; }
    else { cp = c; n = 1; }
    i += n;
    char buf[16];
    switch (cp) {
      case '"': o += "\\\""; continue;
      case '\\': o += "\\\\"; continue;
      case '\n': o += "\\n"; continue;
      case '\r': o += "\\r"; continue;
      case '\t': o += "\\t"; continue;
      case '\b': o += "\\b"; continue;
      case '\f': o += "\\f"; continue;
      default: break;
    }
    if (cp < 0x20 || (cp >= 0x7F && cp < 0x10000)) {
      if (cp < 0x7F) snprintf(buf, sizeof buf, "\\u%04x", cp);
      else snprintf(buf, sizeof buf, "\\u%04x", cp);
      o += buf;
    } else if (cp >= 0x10000) {
      const uint32_t v = cp - 0x10000;
      snprintf(buf, sizeof buf, "\\u%04x\\u%04x", 0xD800 + (v >> 10), 0xDC00 + (v & 0x3FF));
      o += buf;
    } else {
      o += (char)cp;
    }
  }
  o += '"';
}

inline std::string py_float_repr(double d) {
  if (d != d) return "NaN";
  if (d == __builtin_inf()) return "Infinity";
  if (d == -__builtin_inf()) return "-Infinity";
  char buf[40];
  int prec = 1;
  for (; prec <= 17; ++prec) {
    snprintf(buf, sizeof buf, "%.*e", prec - 1, d);
    if (strtod(buf, nullptr) == d) break;
  }
  // digits and decimal exponent of the shortest form
  std::string m(buf);
  const size_t ep = m.find('e');
  int exp10 = atoi(m.c_str() + ep + 1);
  std::string digits;
  bool neg = false;
  for (size_t i = 0; i < ep; ++i) {
    if (m[i] == '-') neg = true;
    else if (m[i] >= '0' && m[i] <= '9') digits += m[i];
  }
  while (digits.size() > 1 && digits.back() == '0') digits.pop_back();
  std::string out = neg ? "-" : "";
  if (exp10 < -4 || exp10 >= 16) {  // repr switches to scientific notation here
    out += digits.substr(0, 1);
    if (digits.size() > 1) out += "." + digits.substr(1);
    snprintf(buf, sizeof buf, "e%c%02d", exp10 < 0 ? '-' : '+', exp10 < 0 ? -exp10 : exp10);
    out += buf;
  } else if (exp10 < 0) {
    out += "0." + std::string((size_t)(-exp10 - 1), '0') + digits;
  } else {
    if ((int)digits.size() <= exp10 + 1) out += digits + std::string((size_t)(exp10 + 1 - (int)digits.size()), '0') + ".0";
    else out += digits.substr(0, (size_t)exp10 + 1) + "." + digits.substr((size_t)exp10 + 1);
  }
  return out;
}

inline void canon(std::string& o, const JV& v) {
  switch (v.t) {
    case JV::NUL: o += "null"; return;
    case JV::BOOL: o += v.b ? "true" : "false"; return;
    case JV::NUM: {
      if (v.is_int) {  // Python int: the literal without a leading '+' / zeros (JSON has neither)
        o += v.s == "-0" ? "0" : v.s;
      } else {
        o += py_float_repr(strtod(v.s.c_str(), nullptr));
      }
      return;
    }
    case JV::STR: esc(o, v.s); return;
    case JV::ARR:
      o += '[';
      for (size_t i = 0; i < v.a.size(); ++i) {
        if (i) o += ',';
        canon(o, v.a[i]);
      }
      o += ']';
      return;
    case JV::OBJ: {
      // unique keys (the last occurrence wins, as Python's json.loads), sorted by code point
      std::map<std::string, const JV*> m;
      for (size_t i = 0; i < v.k.size(); ++i) m[v.k[i]] = &v.a[i];
      o += '{';
      bool first = true;
      for (const auto& kv : m) {
        if (!first) o += ',';
        first = false;
        esc(o, kv.first);
        o += ':';
        canon(o, *kv.second);
      }
      o += '}';
      return;
    }
  }
}

// ------------------------------------------------------------------ query step programs
// The fast path of the jq queries the shipped Stage CRs use (a lowering of the jqc.hpp syntax
// tree, compile_query below): a list of steps over a stream of values (nullptr = null):
//   F <key>   .key (null -> null; a non-object -> error)
//   I         .[] (array items / object values in gojq's sorted key order; else -> error)
//   S <path> <lit>   select(<path> == <lit>) with <path> a list of keys
// Query.Execute semantics (query.go:48-69): an error makes the result nil; nulls are dropped.
struct Step {
  char op;
  std::string key;
  std::vector<std::string> path;
  JV lit;
};
struct Query {
  std::vector<Step> steps;
};

// jq equality of a value with a literal (numbers compared by value, strings, bools, null)
inline bool jq_eq(const JV* v, const JV& lit) {
  const JV::T t = v ? v->t : JV::NUL;
  if (t != lit.t) return false;
  switch (t) {
    case JV::NUL: return true;
    case JV::BOOL: return v->b == lit.b;
    case JV::STR: return v->s == lit.s;
    case JV::NUM: return strtod(v->s.c_str(), nullptr) == strtod(lit.s.c_str(), nullptr);
    default: return false;
  }
}

// -> false on a jq error
inline bool run_query(const Query& q, const JV* root, std::vector<const JV*>& out) {
  std::vector<const JV*> cur{root}, nxt;
  for (const Step& s : q.steps) {
    nxt.clear();
    for (const JV* v : cur) {
      if (s.op == 'F') {
        if (!v || v->t == JV::NUL) { nxt.push_back(nullptr); continue; }
        if (v->t != JV::OBJ) return false;
        nxt.push_back(v->get(s.key));
      } else if (s.op == 'I') {
        if (!v) return false;
        if (v->t == JV::ARR) {
          for (const JV& x : v->a) nxt.push_back(&x);
        } else if (v->t == JV::OBJ) {
          for (const auto& kv : kwkjq::entries(*v)) nxt.push_back(kv.second);
        } else {
          return false;
        }
      } else {  // S: select(path == lit)
        const JV* w = v;
        bool err = false;
        for (const std::string& k : s.path) {
          if (!w || w->t == JV::NUL) { w = nullptr; continue; }
          if (w->t != JV::OBJ) { err = true; break; }
          w = w->get(k);
        }
        if (err) return false;
        if (jq_eq(w, s.lit)) nxt.push_back(v);
      }
    }
    cur.swap(nxt);
  }
  out.clear();
  for (const JV* v : cur)
    if (v && v->t != JV::NUL) out.push_back(v);
  return true;
}

// A compiled selector key / getter query (expression.NewQuery): the step program when the query
// lowers to one (path steps and select(path == literal), the forms of kustomize/stage/**), else the
// jq evaluator (jqc.hpp).  kwkjq::Unsupported for a query outside the native subset.
struct CQuery {
  std::shared_ptr<kwkjq::Query> jq;
  Query steps;
  bool fast = false;
};

// a path of fields from `.` (for select's operand)
inline bool lower_path(const kwkjq::Node& n, std::vector<std::string>& keys) {
  if (n.k == kwkjq::Node::IDENT) return true;
  if (n.k != kwkjq::Node::FIELD || !lower_path(*n.a, keys)) return false;
  keys.push_back(n.name);
  return true;
}
inline bool lower_steps(const kwkjq::Node& n, Query& q) {
  using K = kwkjq::Node;
  switch (n.k) {
    case K::IDENT: return true;
    case K::FIELD: {
      if (!lower_steps(*n.a, q)) return false;
      Step s;
      s.op = 'F';
      s.key = n.name;
      q.steps.push_back(std::move(s));
      return true;
    }
    case K::ITER: {
      if (!lower_steps(*n.a, q)) return false;
      Step s;
      s.op = 'I';
      q.steps.push_back(std::move(s));
      return true;
    }
    case K::PIPE: return lower_steps(*n.a, q) && lower_steps(*n.b, q);
    case K::FUNC: {
      if (n.name != "select" || n.args.size() != 1 || n.args[0]->k != K::CMP || n.args[0]->name != "==") return false;
      const K& c = *n.args[0];
      const K* path = c.a.get();
      const K* lit = c.b.get();
      if (path->k == K::LIT) std::swap(path, lit);
      Step s;
      s.op = 'S';
      if (lit->k != K::LIT || lit->lit.t == JV::ARR || lit->lit.t == JV::OBJ || !lower_path(*path, s.path)) return false;
      s.lit = lit->lit;
      q.steps.push_back(std::move(s));
      return true;
    }
    default: return false;
  }
}

inline CQuery compile_query(const std::string& src) {
  CQuery q;
  q.jq = std::make_shared<kwkjq::Query>(src);
  q.fast = lower_steps(*q.jq->root, q.steps);
  return q;
}

// Query.Execute on a document (outputs borrow from `doc` or hold computed values)
inline bool exec_query(const CQuery& q, const JV& doc, std::vector<kwkjq::Val>& out) {
  if (!q.fast) return q.jq->execute(doc, out);
  thread_local std::vector<const JV*> raw;
  out.clear();
  if (!run_query(q.steps, &doc, raw)) return false;
  for (const JV* v : raw) out.push_back(kwkjq::Val{v, nullptr});
  return true;
}

// Typed-object presence (expression.ToJSONStandard, query.go:72-88; host mirror typed.py): the
// reference's queries see json.Marshal of the typed *corev1.Pod / *corev1.Node, so an omitempty
// field holding the zero value of its string / number / bool / slice / map type is absent, a
// struct-typed field or a field without omitempty is present, a pointer is present unless nil, a
// zero metav1.Time is null (dropped by Query.Execute like an absent value).  The table holds the
// k8s.io/api v0.30.2 core/v1 tags of the fields on the queried paths; other fields keep a
// non-empty value.  The apiserver's JSON is already in this form; hand-written objects and
// patched ones (the apiserver round trip drops what a patch emptied) are rewritten.
enum PKind : uint8_t { P_KEEP, P_STRUCT, P_PTR, P_LIST, P_LIST_KEEP, P_TIME };
struct PField { const char* type; const char* key; PKind kind; const char* sub; };
const PField kPresence[] = {
    {"Pod", "metadata", P_STRUCT, "ObjectMeta"}, {"Pod", "spec", P_STRUCT, "PodSpec"},
    {"Pod", "status", P_STRUCT, "PodStatus"},
    {"Node", "metadata", P_STRUCT, "ObjectMeta"}, {"Node", "spec", P_STRUCT, ""},
    {"Node", "status", P_STRUCT, "NodeStatus"},
    {"ObjectMeta", "creationTimestamp", P_TIME, ""}, {"ObjectMeta", "deletionTimestamp", P_TIME, ""},
    {"ObjectMeta", "ownerReferences", P_LIST, "OwnerReference"}, {"ObjectMeta", "managedFields", P_LIST, ""},
    {"OwnerReference", "apiVersion", P_KEEP, ""}, {"OwnerReference", "kind", P_KEEP, ""},
    {"OwnerReference", "name", P_KEEP, ""}, {"OwnerReference", "uid", P_KEEP, ""},
    {"PodSpec", "containers", P_LIST_KEEP, "Container"}, {"PodSpec", "initContainers", P_LIST, "Container"},
    {"PodSpec", "ephemeralContainers", P_LIST, "Container"},
    {"Container", "name", P_KEEP, ""}, {"Container", "resources", P_STRUCT, ""},
    {"PodStatus", "conditions", P_LIST, "PodCondition"}, {"PodStatus", "startTime", P_TIME, ""},
    {"PodStatus", "initContainerStatuses", P_LIST, "ContainerStatus"},
    {"PodStatus", "containerStatuses", P_LIST, "ContainerStatus"},
    {"PodStatus", "ephemeralContainerStatuses", P_LIST, "ContainerStatus"},
    {"PodCondition", "type", P_KEEP, ""}, {"PodCondition", "status", P_KEEP, ""},
    {"PodCondition", "lastProbeTime", P_TIME, ""}, {"PodCondition", "lastTransitionTime", P_TIME, ""},
    {"ContainerStatus", "name", P_KEEP, ""}, {"ContainerStatus", "ready", P_KEEP, ""},
    {"ContainerStatus", "restartCount", P_KEEP, ""}, {"ContainerStatus", "image", P_KEEP, ""},
    {"ContainerStatus", "imageID", P_KEEP, ""}, {"ContainerStatus", "state", P_STRUCT, "ContainerState"},
    {"ContainerStatus", "lastState", P_STRUCT, "ContainerState"},
    {"ContainerState", "waiting", P_PTR, ""}, {"ContainerState", "running", P_PTR, "ContainerStateRunning"},
    {"ContainerState", "terminated", P_PTR, "ContainerStateTerminated"},
    {"ContainerStateRunning", "startedAt", P_TIME, ""},
    {"ContainerStateTerminated", "exitCode", P_KEEP, ""}, {"ContainerStateTerminated", "startedAt", P_TIME, ""},
    {"ContainerStateTerminated", "finishedAt", P_TIME, ""},
    {"NodeStatus", "conditions", P_LIST, "NodeCondition"}, {"NodeStatus", "daemonEndpoints", P_STRUCT, ""},
    {"NodeStatus", "nodeInfo", P_STRUCT, "NodeSystemInfo"},
    {"NodeCondition", "type", P_KEEP, ""}, {"NodeCondition", "status", P_KEEP, ""},
    {"NodeCondition", "lastHeartbeatTime", P_TIME, ""}, {"NodeCondition", "lastTransitionTime", P_TIME, ""},
    {"NodeSystemInfo", "machineID", P_KEEP, ""}, {"NodeSystemInfo", "systemUUID", P_KEEP, ""},
    {"NodeSystemInfo", "bootID", P_KEEP, ""}, {"NodeSystemInfo", "kernelVersion", P_KEEP, ""},
    {"NodeSystemInfo", "osImage", P_KEEP, ""}, {"NodeSystemInfo", "containerRuntimeVersion", P_KEEP, ""},
    {"NodeSystemInfo", "kubeletVersion", P_KEEP, ""}, {"NodeSystemInfo", "kubeProxyVersion", P_KEEP, ""},
    {"NodeSystemInfo", "operatingSystem", P_KEEP, ""}, {"NodeSystemInfo", "architecture", P_KEEP, ""},
};

inline const PField* presence_field(const char* type, const std::string& key) {
  for (const PField& f : kPresence)
    if (strcmp(f.type, type) == 0 && key == f.key) return &f;
  return nullptr;
}

// encoding/json isEmptyValue for what JSON holds
inline bool zero_value(const JV& v) {
  switch (v.t) {
    case JV::NUL: return true;
    case JV::BOOL: return !v.b;
    case JV::NUM: return strtod(v.s.c_str(), nullptr) == 0.0;
    case JV::STR: return v.s.empty();
    default: return v.a.empty();
  }
}

inline void typed_presence(JV& obj, const char* type) {
  if (obj.t != JV::OBJ) return;
  // duplicate keys: the last one is what json.Unmarshal keeps
  for (size_t i = obj.k.size(); i-- > 0;) {
    bool later = false;
    for (size_t j = i + 1; j < obj.k.size(); ++j) later |= obj.k[j] == obj.k[i];
    bool drop = later;
    if (!drop) {
      JV& v = obj.a[i];
      const PField* f = presence_field(type, obj.k[i]);
      if (v.t == JV::NUL) drop = true;
      else if (!f) drop = zero_value(v);
      else switch (f->kind) {
        case P_KEEP: break;
        case P_TIME: drop = v.t == JV::STR && v.s.empty(); break;
        case P_STRUCT:
        case P_PTR: typed_presence(v, f->sub); break;
        case P_LIST:
        case P_LIST_KEEP:
          if (v.t == JV::ARR)
            for (JV& x : v.a) typed_presence(x, f->sub);
          drop = f->kind == P_LIST && zero_value(v);
          break;
      }
    }
    if (drop) {
      obj.k.erase(obj.k.begin() + (long)i);
      obj.a.erase(obj.a.begin() + (long)i);
    }
  }
}

// Pods and nodes reach the reference's matcher as typed objects (PodController / NodeController);
// every other kind through the StageController as *unstructured.Unstructured
// (stage_controller.go:174-232), whose json.Marshal writes the object map as it holds it: every
// field, zero values and nulls included — so those objects are left as they are.
inline void typed_presence(JV& obj) {
  const JV* kind = obj.t == JV::OBJ ? obj.get("kind") : nullptr;
  const bool known = kind && kind->t == JV::STR && (kind->s == "Pod" || kind->s == "Node");
  if (known) typed_presence(obj, kind->s.c_str());
}

// compiler.class_key: the spec shape without status, identity metadata, node placement;
// ownerReferences reduced to their sorted kinds (kwok_amd/host/compiler.py class_key)
inline std::string class_key(const JV& obj, const std::vector<std::string>& identity_meta) {
  JV o = obj;
  if (o.t != JV::OBJ) return "null";
  for (size_t i = o.k.size(); i-- > 0;)
    if (o.k[i] == "status") { o.k.erase(o.k.begin() + (long)i); o.a.erase(o.a.begin() + (long)i); }
  for (size_t i = 0; i < o.k.size(); ++i) {
    if (o.k[i] == "metadata" && o.a[i].t == JV::OBJ) {
      JV& md = o.a[i];
      for (size_t j = md.k.size(); j-- > 0;) {
        if (std::find(identity_meta.begin(), identity_meta.end(), md.k[j]) != identity_meta.end()) {
          md.k.erase(md.k.begin() + (long)j);
          md.a.erase(md.a.begin() + (long)j);
        }
      }
      if (const JV* refs = md.get("ownerReferences")) {
        std::vector<std::string> kinds;
        if (refs->t == JV::ARR)
          for (const JV& r : refs->a) {
            const JV* k = r.t == JV::OBJ ? r.get("kind") : nullptr;
            kinds.push_back(k && k->t == JV::STR ? k->s : "");
          }
        std::sort(kinds.begin(), kinds.end());
        JV arr;
        arr.t = JV::ARR;
        for (auto& k : kinds) {
          JV s;
          s.t = JV::STR;
          s.s = k;
          arr.a.push_back(s);
        }
        for (size_t j = 0; j < md.k.size(); ++j)
          if (md.k[j] == "ownerReferences") md.a[j] = arr;
      }
    } else if (o.k[i] == "spec" && o.a[i].t == JV::OBJ) {
      JV& sp = o.a[i];
      for (size_t j = sp.k.size(); j-- > 0;)
        if (sp.k[j] == "nodeName" || sp.k[j] == "hostname") {
          sp.k.erase(sp.k.begin() + (long)j);
          sp.a.erase(sp.a.begin() + (long)j);
        }
    }
  }
  std::string out;
  canon(out, o);
  return out;
}

}  // namespace kwkhost
