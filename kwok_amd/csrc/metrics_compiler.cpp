// Native Metric CR compiler (include/kwok_metrics.h): a Metric CR's gauges, counters and
// histograms -> the device programs of kwk_metrics_load / kwk_histograms_load.  Restates
// kwok_amd/host/metrics.py (load_metric_yaml, MetricsProgram) over celc.hpp's lowering.
//
// Reference: pkg/kwok/metrics/metrics.go:168-462 (updateGauge / updateCounter / updateHistogram:
// one compiled CEL program per value and per bucket, node / pod / container series),
// :133-160 (a histogram's visible bounds), pkg/apis/v1alpha1/metric_types.go (the CRD).
#include <cmath>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "../../include/kwok_metrics.h"
#include "celc.hpp"
#include "host_common.hpp"
#include "json_dom.hpp"

using kwkjson::JV;

struct kwk_metric_set {
  std::vector<kwk_metric_desc> metrics;
  std::vector<kwk_metric_op> ops;
  std::vector<kwk_histogram_desc> hists;
  std::vector<kwk_metric_bucket> buckets;
  std::vector<kwk_metric_op> hist_ops;
  std::string describe;
};

namespace {

thread_local std::string g_err;

kwk_status fail(kwk_status code, const std::string& msg) {
  g_err = msg;
  return code;
}

struct BadCR : std::runtime_error { using std::runtime_error::runtime_error; };

const JV* field(const JV& o, const char* k) { return o.t == JV::OBJ ? o.get(k) : nullptr; }

std::string str_field(const JV& o, const char* k, const char* dflt, const std::string& where) {
  const JV* v = field(o, k);
  if (!v || v->t == JV::NUL) return dflt;
  if (v->t != JV::STR) throw BadCR(where + "." + k + ": a string");
  return v->s;
}

bool truthy(const JV* v) {  // Python bool(...) of a YAML / JSON scalar
  if (!v) return false;
  switch (v->t) {
    case JV::NUL: return false;
    case JV::BOOL: return v->b;
    case JV::NUM: return strtod(v->s.c_str(), nullptr) != 0.0;
    case JV::STR: return !v->s.empty();
    default: return !v->a.empty();
  }
}

double le_of(const JV* v, const std::string& where) {  // float(b.get("le", 0))
  if (!v || v->t == JV::NUL) {
    if (!v) return 0.0;
    throw BadCR(where + ".le: a number");
  }
  if (v->t == JV::NUM) return strtod(v->s.c_str(), nullptr);
  if (v->t == JV::STR) {
    char* end = nullptr;
    const double d = strtod(v->s.c_str(), &end);
    if (v->s.empty() || *end) throw BadCR(where + ".le: a number");
    return d;
  }
  throw BadCR(where + ".le: a number");
}

uint32_t dim_of(const std::string& d, const std::string& where) {
  if (d.empty() || d == "node") return KWK_METRIC_DIM_NODE;
  if (d == "pod") return KWK_METRIC_DIM_POD;
  if (d == "container") return KWK_METRIC_DIM_CONTAINER;
  throw BadCR(where + ".dimension: node, pod or container (got '" + d + "')");
}

void put_ops(std::vector<kwk_metric_op>& dst, const std::vector<kwkcel::Op>& prog) {
  for (const kwkcel::Op& o : prog) {
    kwk_metric_op x{};
    x.op = o.op;
    x.arg = o.arg;
    x.value = o.value;
    dst.push_back(x);
  }
}

// one value: its program, or LowerError (host metric); syntax / evaluation errors are BadCR
std::vector<kwkcel::Op> lower_value(const std::string& src, uint32_t dim, const std::string& where) {
  try {
    return kwkcel::lower(src, (kwkcel::Dim)dim);
  } catch (const kwkcel::SyntaxError& e) {
    throw BadCR(where + ": CEL syntax error in '" + src + "': " + e.what());
  } catch (const kwkcel::CELError& e) {
    throw BadCR(where + ": CEL evaluation error in '" + src + "': " + e.what());
  }
}

const char* kDims[] = {"node", "pod", "container"};

void compile(kwk_metric_set& M, const JV& cr) {
  if (cr.t != JV::OBJ) throw BadCR("a Metric object");
  if (const JV* k = cr.get("kind"); k && !(k->t == JV::STR && k->s == "Metric")) throw BadCR("kind: Metric");
  const JV* spec = cr.get("spec");
  if (!spec || spec->t != JV::OBJ) throw BadCR("spec: an object");
  const std::string path = str_field(*spec, "path", "", "spec");
  const JV* list = spec->get("metrics");
  std::string d = "{\"path\":";
  kwkhost::esc(d, path);
  d += ",\"metrics\":[";
  std::vector<std::string> host;
  if (list && list->t != JV::NUL && list->t != JV::ARR) throw BadCR("spec.metrics: a list");
  const size_t n = list && list->t == JV::ARR ? list->a.size() : 0;
  for (size_t i = 0; i < n; ++i) {
    const JV& m = list->a[i];
    const std::string where = "spec.metrics[" + std::to_string(i) + "]";
    if (m.t != JV::OBJ) throw BadCR(where + ": an object");
    const std::string name = str_field(m, "name", "", where);
    if (name.empty()) throw BadCR(where + ".name: required");
    const std::string kind = str_field(m, "kind", "", where);
    if (kind != "gauge" && kind != "counter" && kind != "histogram")
      throw BadCR(where + ": unknown metric kind '" + kind + "'");
    const uint32_t dim = dim_of(str_field(m, "dimension", "node", where), where);
    const std::string help = str_field(m, "help", "", where);
    std::string labels = "[";
    if (const JV* ls = m.get("labels"); ls && ls->t == JV::ARR) {
      for (size_t j = 0; j < ls->a.size(); ++j) {
        const std::string lw = where + ".labels[" + std::to_string(j) + "]";
        if (j) labels += ",";
        labels += "{\"name\":";
        kwkhost::esc(labels, str_field(ls->a[j], "name", "", lw));
        labels += ",\"value\":";
        kwkhost::esc(labels, str_field(ls->a[j], "value", "", lw));
        labels += "}";
      }
    }
    labels += "]";
    bool device = true;
    std::string reason;
    uint32_t index;
    if (kind == "histogram") {
      const JV* bs = m.get("buckets");
      if (!bs || bs->t != JV::ARR || bs->a.empty()) throw BadCR("histogram '" + name + "' has no buckets");
      struct B { double le; bool hidden; std::string value; };
      std::vector<B> bks;
      for (size_t j = 0; j < bs->a.size(); ++j) {
        const std::string bw = where + ".buckets[" + std::to_string(j) + "]";
        const JV& b = bs->a[j];
        if (b.t != JV::OBJ) throw BadCR(bw + ": an object");
        bks.push_back({le_of(b.get("le"), bw), truthy(b.get("hidden")), str_field(b, "value", "0", bw)});
      }
      std::vector<std::vector<kwkcel::Op>> progs;
      try {
        for (size_t j = 0; j < bks.size(); ++j)
          progs.push_back(lower_value(bks[j].value, dim, where + ".buckets[" + std::to_string(j) + "].value"));
      } catch (const kwkcel::LowerError& e) {
        device = false;
        reason = e.what();
        progs.assign(bks.size(), {{kwkcel::OP_CONST, 0, 0.0}});
      }
      index = (uint32_t)M.hists.size();
      kwk_histogram_desc hd{};
      hd.dimension = dim;
      hd.first_bucket = (uint32_t)M.buckets.size();
      hd.n_buckets = (uint32_t)bks.size();
      M.hists.push_back(hd);
      for (size_t j = 0; j < bks.size(); ++j) {
        kwk_metric_bucket mb{};
        mb.le = bks[j].le;
        mb.hidden = bks[j].hidden ? 1u : 0u;
        mb.first_op = (uint32_t)M.hist_ops.size();
        mb.n_ops = (uint32_t)progs[j].size();
        M.buckets.push_back(mb);
        put_ops(M.hist_ops, progs[j]);
      }
    } else {
      const std::string value = str_field(m, "value", "0", where);
      std::vector<kwkcel::Op> prog;
      try {
        prog = lower_value(value, dim, where + ".value");
      } catch (const kwkcel::LowerError& e) {
        device = false;
        reason = e.what();
        prog = {{kwkcel::OP_CONST, 0, NAN}};
      }
      index = (uint32_t)M.metrics.size();
      kwk_metric_desc md{};
      md.dimension = dim;
      md.first_op = (uint32_t)M.ops.size();
      md.n_ops = (uint32_t)prog.size();
      M.metrics.push_back(md);
      put_ops(M.ops, prog);
    }
    if (!device) host.push_back(name);
    if (i) d += ",";
    d += "{\"name\":";
    kwkhost::esc(d, name);
    d += ",\"help\":";
    kwkhost::esc(d, help);
    d += ",\"kind\":\"" + kind + "\",\"dimension\":\"" + kDims[dim] + "\",\"labels\":" + labels;
    d += std::string(",\"device\":") + (device ? "true" : "false") + ",\"reason\":";
    kwkhost::esc(d, reason);
    d += ",\"program\":" + std::to_string(index) + "}";
  }
  d += "],\"host_metrics\":[";
  for (size_t j = 0; j < host.size(); ++j) {
    if (j) d += ",";
    kwkhost::esc(d, host[j]);
  }
  d += "]}";
  M.describe = std::move(d);
}

}  // namespace

extern "C" {

// every failing entry point records its message in the calling thread's g_err (a set's own calls
// never fail after it is built), so the message is g_err whatever `m` is
const char* kwk_metric_set_last_error(const kwk_metric_set* m) {
  (void)m;
  return g_err.c_str();
}

kwk_status kwk_compile_metrics(const char* metric_json, kwk_metric_set** out) {
  if (!metric_json || !out) return fail(KWK_EINVAL, "null argument");
  try {
    JV cr;
    kwkjson::Parser p{metric_json, metric_json + strlen(metric_json)};
    if (!p.value(cr)) return fail(KWK_EINVAL, "metric: malformed JSON");
    p.ws();
    if (p.p != p.e) return fail(KWK_EINVAL, "metric: trailing bytes after the JSON value");
    std::unique_ptr<kwk_metric_set> M(new kwk_metric_set());
    compile(*M, cr);
    *out = M.release();
    return KWK_OK;
  } catch (const std::exception& e) {
    return fail(KWK_EINVAL, e.what());
  }
}

kwk_status kwk_metric_set_destroy(kwk_metric_set* m) {
  delete m;
  return KWK_OK;
}

kwk_status kwk_metric_set_programs(const kwk_metric_set* m, uint32_t* n_metrics, const kwk_metric_desc** metrics,
                                   uint32_t* n_ops, const kwk_metric_op** ops) {
  if (!m || !n_metrics || !metrics || !n_ops || !ops) return fail(KWK_EINVAL, "null argument");
  *n_metrics = (uint32_t)m->metrics.size();
  *metrics = m->metrics.data();
  *n_ops = (uint32_t)m->ops.size();
  *ops = m->ops.data();
  return KWK_OK;
}

kwk_status kwk_metric_set_histograms(const kwk_metric_set* m, uint32_t* n_hist, const kwk_histogram_desc** hists,
                                     uint32_t* n_buckets, const kwk_metric_bucket** buckets, uint32_t* n_ops,
                                     const kwk_metric_op** ops) {
  if (!m || !n_hist || !hists || !n_buckets || !buckets || !n_ops || !ops) return fail(KWK_EINVAL, "null argument");
  *n_hist = (uint32_t)m->hists.size();
  *hists = m->hists.data();
  *n_buckets = (uint32_t)m->buckets.size();
  *buckets = m->buckets.data();
  *n_ops = (uint32_t)m->hist_ops.size();
  *ops = m->hist_ops.data();
  return KWK_OK;
}

kwk_status kwk_metric_set_describe(const kwk_metric_set* m, const char** json) {
  if (!m || !json) return fail(KWK_EINVAL, "null argument");
  *json = m->describe.c_str();
  return KWK_OK;
}

kwk_status kwk_cel_lower(const char* expr, uint32_t dimension, kwk_metric_op* out, uint32_t cap, uint32_t* n_ops) {
  if (!expr || !n_ops || (cap && !out)) return fail(KWK_EINVAL, "null argument");
  if (dimension > 3) return fail(KWK_EINVAL, "dimension: KWK_METRIC_DIM_* or 3");
  try {
    const std::vector<kwkcel::Op> prog = kwkcel::lower(expr, (kwkcel::Dim)dimension);
    *n_ops = (uint32_t)prog.size();
    if (prog.size() > cap) return fail(KWK_ECAP, "program longer than cap");
    for (size_t i = 0; i < prog.size(); ++i) {
      out[i].op = prog[i].op;
      out[i].arg = prog[i].arg;
      out[i].value = prog[i].value;
    }
    return KWK_OK;
  } catch (const kwkcel::LowerError& e) {
    *n_ops = 0;
    return fail(KWK_ENOLOWER, e.what());
  } catch (const kwkcel::SyntaxError& e) {
    *n_ops = 0;
    return fail(KWK_EINVAL, std::string("CEL syntax error: ") + e.what());
  } catch (const std::exception& e) {
    *n_ops = 0;
    return fail(KWK_EINVAL, std::string("CEL error: ") + e.what());
  }
}

}  // extern "C"
