// Next-state pieces shared by the native host libraries (compiler.cpp: exploration; encoder.cpp:
// "patch already applied" feature bits): the RFC 7386 merge patch / RFC 6902 subset the apiserver
// applies, the typed round trip (prune_empty), and a Stage's patches rendered with the gotpl mirror
// (kwok_amd/host/nextstate.py; reference pkg/utils/lifecycle/next.go:73-173, finalizers.go:32-111).
#pragma once
#include <stdexcept>
#include <string>
#include <vector>

#include "gotpl.hpp"
#include "host_common.hpp"

namespace kwknext {

using kwkjson::JV;

struct CompileError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// ---- JV helpers
inline JV jstr(const std::string& s) {
  JV v;
  v.t = JV::STR;
  v.s = s;
  return v;
}
inline JV jobj() {
  JV v;
  v.t = JV::OBJ;
  return v;
}
inline JV* obj_get(JV& o, const std::string& k) {
  if (o.t != JV::OBJ) return nullptr;
  for (size_t i = o.k.size(); i-- > 0;)
    if (o.k[i] == k) return &o.a[i];
  return nullptr;
}
inline void obj_set(JV& o, const std::string& k, JV v) {
  if (JV* x = obj_get(o, k)) { *x = std::move(v); return; }
  o.k.push_back(k);
  o.a.push_back(std::move(v));
}
inline bool obj_erase(JV& o, const std::string& k) {
  bool any = false;
  for (size_t i = o.k.size(); i-- > 0;)
    if (o.k[i] == k) {
      o.k.erase(o.k.begin() + (long)i);
      o.a.erase(o.a.begin() + (long)i);
      any = true;
    }
  return any;
}
inline JV& obj_setdefault(JV& o, const std::string& k) {
  if (JV* x = obj_get(o, k)) return *x;
  obj_set(o, k, jobj());
  return o.a.back();
}
inline std::string canon(const JV& v) {
  std::string o;
  kwkhost::canon(o, v);
  return o;
}
inline JV parse_json(const char* b, const char* e, const char* what) {
  JV v;
  kwkjson::Parser P{b, e};
  if (!P.value(v)) throw CompileError(std::string(what) + ": invalid JSON");
  return v;
}
struct Patch {
  std::string root, tmpl, type = "merge", subresource;
};

// ------------------------------------------------------------------ next state (nextstate.py)
inline void prune_empty(JV& o) { kwkhost::typed_presence(o); }

inline std::vector<std::string> json_ptr(const std::string& path) {
  std::vector<std::string> out;
  size_t p = 1;
  if (path.empty()) return out;
  for (;;) {
    const size_t q = path.find('/', p);
    std::string part = path.substr(p, q == std::string::npos ? std::string::npos : q - p);
    std::string o;
    for (size_t i = 0; i < part.size(); ++i) {  // ~1 -> /, then ~0 -> ~
      if (part[i] == '~' && i + 1 < part.size() && part[i + 1] == '1') { o += '/'; ++i; }
      else o += part[i];
    }
    std::string o2;
    for (size_t i = 0; i < o.size(); ++i) {
      if (o[i] == '~' && i + 1 < o.size() && o[i + 1] == '0') { o2 += '~'; ++i; }
      else o2 += o[i];
    }
    out.push_back(o2);
    if (q == std::string::npos) break;
    p = q + 1;
  }
  return out;
}

inline long list_index(const JV& list, const std::string& s, bool for_insert) {
  char* end = nullptr;
  const long i = strtol(s.c_str(), &end, 10);
  if (s.empty() || (end && *end)) throw CompileError("json patch: bad list index " + s);
  const long n = (long)list.a.size();
  const long r = i < 0 ? i + n : i;  // Python negative indices
  if (r < 0 || r > n || (!for_insert && r == n)) throw CompileError("json patch: list index out of range");
  return r;
}

// nextstate.json_patch: the RFC 6902 subset (add / remove / replace) of the finalizer ops
inline JV json_patch(const JV& obj, const std::vector<JV>& ops) {
  JV o = obj;
  for (const JV& op : ops) {
    const JV* p = op.get("path");
    const JV* kind = op.get("op");
    if (!p || p->t != JV::STR || !kind || kind->t != JV::STR) throw CompileError("json patch: bad op");
    const std::vector<std::string> parts = json_ptr(p->s);
    if (parts.empty()) throw CompileError("json patch: empty path");
    JV* parent = &o;
    for (size_t i = 0; i + 1 < parts.size(); ++i) {
      if (parent->t == JV::ARR) parent = &parent->a[(size_t)list_index(*parent, parts[i], false)];
      else if (parent->t == JV::OBJ) parent = &obj_setdefault(*parent, parts[i]);
      else throw CompileError("json patch: path through a scalar");
    }
    const std::string& last = parts.back();
    if (kind->s == "add" || kind->s == "replace") {
      const JV* v = op.get("value");
      JV val = v ? *v : JV();
      if (parent->t == JV::ARR) {
        if (last == "-") parent->a.push_back(val);
        else parent->a.insert(parent->a.begin() + list_index(*parent, last, true), val);
      } else if (parent->t == JV::OBJ) {
        obj_set(*parent, last, val);
      } else {
        throw CompileError("json patch: add into a scalar");
      }
    } else if (kind->s == "remove") {
      if (parent->t == JV::ARR) parent->a.erase(parent->a.begin() + list_index(*parent, last, false));
      else if (parent->t == JV::OBJ) {
        if (!obj_erase(*parent, last)) throw CompileError("json patch: remove of a missing key");
      } else throw CompileError("json patch: remove from a scalar");
    } else {
      throw CompileError("unsupported json patch op " + kind->s);
    }
  }
  return o;
}

// RFC 7386 merge patch (evanphx/json-patch MergePatch semantics)
inline JV merge_patch(const JV* target, const JV& patch) {
  if (patch.t != JV::OBJ) return patch;
  JV out = (target && target->t == JV::OBJ) ? *target : jobj();
  for (size_t i = 0; i < patch.k.size(); ++i) {
    const std::string& k = patch.k[i];
    const JV& v = patch.a[i];
    if (v.t == JV::NUL) {
      obj_erase(out, k);
    } else {
      JV* cur = obj_get(out, k);
      JV merged = merge_patch(cur, v);
      obj_set(out, k, std::move(merged));
    }
  }
  return out;
}

struct Rendered {
  bool json;
  JV data;
};

// nextstate.render_patches: every patch rendered against the same object
inline std::vector<Rendered> render_patches(const std::vector<Patch>& patches, const JV& obj, kwktpl::Renderer& r) {
  std::vector<Rendered> out;
  for (const Patch& p : patches) {
    JV data = kwktpl::yaml_to_json(r.to_text(p.tmpl, obj));
    if (p.type == "json") {
      if (!p.root.empty()) {
        JV ops;
        ops.t = JV::ARR;
        if (data.t == JV::ARR)
          for (const JV& op : data.a) {
            JV o2 = op;
            const JV* path = op.get("path");
            obj_set(o2, "path", jstr("/" + p.root + (path && path->t == JV::STR ? path->s : "")));
            ops.a.push_back(o2);
          }
        data = ops;
      }
      out.push_back({true, data});
    } else {
      if (!p.root.empty()) {
        JV w = jobj();
        obj_set(w, p.root, data);
        data = w;
      }
      out.push_back({false, data});
    }
  }
  return out;
}

inline JV apply_patch(const JV& obj, const Rendered& rp) {
  if (rp.json) {
    if (rp.data.t != JV::ARR) throw CompileError("json patch data is not a list");
    return json_patch(obj, rp.data.a);
  }
  return merge_patch(&obj, rp.data);
}


// compiler._patch_applied: rendering + applying the stage's patches leaves the object unchanged
// (the static renderer: exploration functions, Now fixed at 1.7e18 ns)
inline bool patch_applied(const std::vector<Patch>& patches, const JV& obj, kwktpl::Renderer& r) {
  try {
    JV cur = obj;
    for (const Rendered& rp : render_patches(patches, obj, r)) {
      cur = apply_patch(cur, rp);
      prune_empty(cur);
    }
    return canon(cur) == canon(obj);
  } catch (const std::exception&) {
    return false;
  }
}

inline kwktpl::Renderer static_renderer() {
  kwktpl::Renderer r(1700000000LL * 1000000000LL);
  r.exploration_funcs();
  return r;
}

}  // namespace kwknext
